#!/bin/bash
# gen_coop_kernel (N = 8192 on two workgroups per ciphertext): parity, then opt7 against the
# two-launch path.  Usage: tools/r05_coop.sh TAG
TAG=${1:-r05coop}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread \
  -k "coop or N8192" > $O/pytest.log 2>&1
rc=$?; tail -25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  echo "== CONCRETE_HIP_GEN_COOP=$v"
  CONCRETE_HIP_GEN_COOP=$v timeout -k 10 300 python -u bench.py --config opt7 --batch 1024 --steps 2 --warmup 1 \
    --verify 1 --no-cpu-baseline --no-ks --no-e2e --no-sdfg > $O/bench_coop$v.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bit_exact[a-z_]*": [a-z]*' $O/bench_coop$v.log | head -5
done
