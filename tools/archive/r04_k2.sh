#!/bin/bash
# Round 4: the k = 2, N = 1024, l = 1 kernel (pbs1024k2.hip) — parity tests, then opt4 bench.
# Usage: tools/r04_k2.sh TAG
set -o pipefail
TAG=${1:-r04k2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "pytest k2 $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs1024k2.py -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_k2.log 2>&1
rc=$?; echo "  rc=$rc"; tail -5 $O/pytest_k2.log
[ $rc -eq 0 ] || exit $rc
echo "bench opt4 $(date +%T)"
timeout -k 10 300 python -u bench.py --config opt4 --no-cpu-baseline --verify 2 --no-ks --no-e2e > $O/bench_opt4.log 2>&1
rc=$?; echo "  rc=$rc"; tail -2 $O/bench_opt4.log
exit $rc
