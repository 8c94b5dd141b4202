#!/bin/bash
# general-path timings of rows that moved to hand-tuned kernels (tools/row_bench.py GENERIC=1)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04rowsgen}; mkdir -p $O; cd $R
for row in "4 512 731 1 23" "4 512 700 3 12" "4 512 702 4 9" "4 512 689 5 8" "5 256 594 2 10" "6 256 601 3 9" "3 512 700 3 9"; do
  GENERIC=1 timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows_generic.log 2>&1 || exit 1
  tail -1 $O/rows_generic.log
done
