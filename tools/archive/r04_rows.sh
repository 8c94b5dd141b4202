#!/bin/bash
# timing of optimizer rows without a bench config (tools/row_bench.py)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04rows}; mkdir -p $O; cd $R
while read -r row; do
  [ -z "$row" ] && continue
  timeout -k 10 240 python -u tools/row_bench.py $row >> $O/rows.log 2>&1 || exit 1
  tail -1 $O/rows.log
done <<ROWS
6 256 596 1 18
4 512 800 1 23
4 512 800 2 16
5 256 604 2 10
2 1024 801 2 15
ROWS
