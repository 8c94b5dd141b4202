#!/bin/bash
# Round 4: the small-batch interleaved-transform N = 1024 kernel (pbs1024_ilp_kernel): parity, then
# cfg2 at B = 512 with and without it, and B = 4096.
set -o pipefail
TAG=${1:-r04ilp}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if false; then
echo "pytest pairs $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs.py -x -v -k "pairs_per_workgroup" --timeout 200 --timeout-method thread \
  > $O/pytest_pairs.log 2>&1
rc=$?; echo "  rc=$rc"; tail -3 $O/pytest_pairs.log
[ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for ilp in 1 0; do
    echo "b512 ilp=$ilp rep$rep $(date +%T)"
    CONCRETE_HIP_PBS_ILP=$ilp timeout -k 10 200 python -u bench.py --global-batch 512 --steps 20 --no-cpu-baseline --verify 4 --no-ks --no-e2e > $O/b512_ilp${ilp}_$rep.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', d['value'], d['checks'].get('bitexact'), d['roofline']['kernel_ms'])" $O/b512_ilp${ilp}_$rep.log
  done
done
for b in 256 1024 4096; do
  echo "b$b $(date +%T)"
  timeout -k 10 200 python -u bench.py --global-batch $b --no-cpu-baseline --verify 4 --no-ks --no-e2e > $O/b$b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', d['value'], d['checks'].get('bitexact'), d['roofline']['kernel_ms'])" $O/b$b.log
done
