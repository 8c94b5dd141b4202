#!/bin/bash
# Round-5 baseline on a fresh box: GPU suite, default bench line, B = 512 line.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05a}
mkdir -p $O
cd $R
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log | cut -c1-600
  case $rc in 0|1) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_b4096 300 python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e
step bench_b512 300 python -u bench.py --batch 512 --steps 10 --no-cpu-baseline --no-sdfg --no-e2e --no-ks
echo done
