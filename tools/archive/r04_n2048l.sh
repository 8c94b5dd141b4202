#!/bin/bash
# N = 2048 and k = 2 kernels with whole-digit levels: parity tests, row timings vs the general path, cfg4 bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04n2048l}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs2048.py tests/test_gpu_pbs1024k2.py -x -v --timeout 200 --timeout-method thread > $O/pytest_2048.log 2>&1
rc=$?; tail -3 $O/pytest_2048.log; [ $rc -ne 0 ] && exit $rc
for row in "1 2048 783 2 15" "1 2048 784 3 11" "1 2048 761 4 9" "2 1024 742 3 12"; do
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
  GENERIC=1 timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 3 > $O/bench_cfg4.log 2>&1 || exit 1
tail -1 $O/bench_cfg4.log | cut -c1-300
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread > $O/pytest_generic.log 2>&1
rc=$?; tail -3 $O/pytest_generic.log; exit $rc
