#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04many; mkdir -p $O; cd $R
for row in "4 512 731 11 4" "4 512 690 22 2" "4 512 629 44 1"; do
  GENERIC=1 timeout -k 10 300 python -u tools/row_bench.py $row >> $O/rows_generic.log 2>&1 || exit 1
  tail -1 $O/rows_generic.log
done
