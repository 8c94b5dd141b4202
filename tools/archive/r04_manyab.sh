#!/bin/bash
# one-level-at-a-time kernels against the all-levels-in-registers ones at l = 2 .. 5 (A/B of
# variants/libconcrete_hip_m3.so: K2_MANY_MIN_LEVEL=2, K4_MANY_MIN_LEVEL=3)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04manyab}; mkdir -p $O; cd $R
for row in "2 1024 754 2 15" "2 1024 769 3 12" "4 512 709 3 12" "4 512 712 4 9" "4 512 689 5 8"; do
  for V in base m3; do
    if [ $V = base ]; then L=$R/concrete_amd/libconcrete_hip.so; else L=$R/variants/libconcrete_hip_$V.so; fi
    echo -n "$V " >> $O/rows.log
    CONCRETE_HIP_LIB=$L timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
    tail -1 $O/rows.log
  done
done
