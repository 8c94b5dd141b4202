#!/bin/bash
# Round 4 GPU pass A: child-process/first-HIP-call experiment, the fused N = 4096 kernel and lifted
# level caps (generic tests), the runtime glue (concurrent calls, SDFG), a short opt6 bench.
# Stops at the first crash / abort / timeout (exit 124, 134, 137, 139); ordinary test failures
# (exit 1) are recorded and the next step runs.  Usage: tools/r04_gpu_a.sh TAG
TAG=${1:-r04a}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -4 $O/$name.log
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step child_init 240 python -u tools/microbench/child_first_init.py
step unmap_stall 180 python -u tools/microbench/unmap_stall.py
step generic 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py -k "N4096 or ln2 or index_arrays"
step runtime 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_sdfg.py
step bench_opt6 300 python -u bench.py --config opt6 --steps 3 --warmup 1 --no-cpu-baseline --no-ks
echo "pass A done"
