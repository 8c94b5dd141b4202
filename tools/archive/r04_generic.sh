#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04gen}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "tile|passed|failed" $O/pytest_generic.log | tail -12; exit $rc
