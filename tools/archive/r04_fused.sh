#!/bin/bash
# N = 4096 one-launch kernel at l = 2..4 vs the two-launch path (row timings)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04fused}; mkdir -p $O; cd $R
for row in "1 4096 880 2 15" "1 4096 880 3 11" "1 4096 880 4 9"; do
  timeout -k 10 240 python -u tools/row_bench.py $row 2048 >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
  CONCRETE_HIP_GEN_FUSED=0 timeout -k 10 240 python -u tools/row_bench.py $row 2048 >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done
