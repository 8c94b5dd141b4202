#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05suite}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log
grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | awk '{print $2}' | sort | uniq -c
exit $rc
