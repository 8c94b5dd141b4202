#!/bin/bash
# k = 2, N = 1024 kernel at l = 1 / 2: parity tests, the general-path tests, one row timing
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04k2l2}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs1024k2.py -x -v --timeout 200 --timeout-method thread > $O/pytest_k2.log 2>&1
rc=$?; tail -3 $O/pytest_k2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; tail -3 $O/pytest_generic.log; [ $rc -ne 0 ] && exit $rc
for row in "2 1024 742 2 15" "2 1024 754 2 15" "2 1024 801 1 23"; do
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
