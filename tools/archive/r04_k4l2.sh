#!/bin/bash
# k = 4, N = 512, l = 2 on 13-bit key limbs (pbs512k4.hip): parity tests, row timings, general-path tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04k4l2}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_small.py -x -v --timeout 200 --timeout-method thread > $O/pytest_small.log 2>&1
rc=$?; tail -3 $O/pytest_small.log; [ $rc -ne 0 ] && exit $rc
for row in "4 512 693 6 7" "4 512 668 8 5" "4 512 731 11 4" "4 512 690 22 2" "4 512 629 44 1"; do
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
GENERIC=1 timeout -k 10 240 python -u tools/row_bench.py 4 512 693 6 7 >> $O/rows.log 2>&1 || exit 1
tail -1 $O/rows.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; tail -3 $O/pytest_generic.log; exit $rc
