#!/bin/bash
# k = 2, N = 1024 at l >= 4 (pbs1024k2_many_kernel): parity, row timings vs the general path
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04k2many}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs1024k2.py -x -v --timeout 200 --timeout-method thread > $O/pytest_k2.log 2>&1
rc=$?; tail -3 $O/pytest_k2.log; [ $rc -ne 0 ] && exit $rc
for row in "2 1024 731 4 9" "2 1024 722 5 8" "2 1024 743 8 5" "2 1024 736 11 4" "2 1024 754 15 3" "2 1024 727 44 1"; do
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
  GENERIC=1 timeout -k 10 300 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; tail -3 $O/pytest_generic.log; exit $rc
