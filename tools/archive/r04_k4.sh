#!/bin/bash
# small-ring kernels (pbs_small.hip levels, pbs512k4.hip): parity tests, row timings, general-path tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04k4}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_small.py -x -v --timeout 200 --timeout-method thread > $O/pytest_small.log 2>&1
rc=$?; tail -3 $O/pytest_small.log; [ $rc -ne 0 ] && exit $rc
for row in "4 512 731 1 23" "4 512 700 3 12" "4 512 702 4 9" "4 512 689 5 8" "5 256 594 2 10" "6 256 601 3 9" "3 512 700 3 9"; do
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
[ -n "$NOFULL" ] && exit 0
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; tail -3 $O/pytest_generic.log; exit $rc
