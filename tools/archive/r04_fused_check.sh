#!/bin/bash
# Round 4: the fused N = 4096 kernel and the lifted level caps on the GPU: parity tests, then a
# short opt6 bench (bit-exact rows, no CPU leg).  Usage: tools/r04_fused_check.sh TAG
set -o pipefail
TAG=${1:-r04f}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py \
  -k "N4096 or ln2 or index_arrays or reference_fixtures" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --config opt6 --steps 3 --warmup 1 --no-cpu-baseline --no-ks > $O/bench_opt6.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_opt6.log; exit 1; }
tail -c 1500 $O/bench_opt6.log
