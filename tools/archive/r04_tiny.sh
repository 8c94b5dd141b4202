#!/bin/bash
# round 4: ring prologue/tail tests (n = 1..3) of the new kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04tiny}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs1024k2.py tests/test_gpu_pbs_small.py tests/test_gpu_pbs.py -x -v \
  -k "tiny_n" --timeout 200 --timeout-method thread > $O/pytest_tiny.log 2>&1
rc=$?; echo "rc=$rc"; tail -4 $O/pytest_tiny.log; exit $rc
