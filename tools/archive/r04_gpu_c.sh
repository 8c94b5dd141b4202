#!/bin/bash
# Round 4 GPU pass C: the general path's parity tests (split path N = 2^15 / 2^16, fused N = 4096,
# non-zero log-norm2 rows), then a short 9-bit bench.  Usage: tools/r04_gpu_c.sh TAG
TAG=${1:-r04c}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step generic 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py -k "N32768 or N65536 or 9bit or 10bit"
step generic_all 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py

# opt6 A/B: fused kernel with / without the key prefetch (variants/libconcrete_hip_nopf.so)
step opt6_pf 300 python -u bench.py --config opt6 --steps 3 --warmup 1 --no-cpu-baseline --no-ks --no-e2e
step opt6_nopf 300 env CONCRETE_HIP_LIB=$GRAFT_REPO_ROOT/variants/libconcrete_hip_nopf.so python -u bench.py --config opt6 --steps 3 --warmup 1 --no-cpu-baseline --no-ks --no-e2e
step opt9 600 python -u bench.py --config opt9 --steps 1 --warmup 0 --batch 1024 --no-cpu-baseline --no-ks --no-e2e --verify 0
# N = 8192 one-launch kernel (spilling; CONCRETE_HIP_GEN_FUSED8=1): parity, then opt7 A/B
step fused8_test 600 env CONCRETE_HIP_GEN_FUSED8=1 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py -k "7bit_k1_N8192"
step opt7_fused8 300 env CONCRETE_HIP_GEN_FUSED8=1 python -u bench.py --config opt7 --steps 2 --warmup 1 --no-cpu-baseline --no-ks --no-e2e
step opt7_base 300 python -u bench.py --config opt7 --steps 2 --warmup 1 --no-cpu-baseline --no-ks --no-e2e
echo "pass C done"
