#!/bin/bash
# row census: every N <= 2048 shape of the optimizer's table, kernel vs general path
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04census}; mkdir -p $O; cd $R
timeout -k 10 1150 python -u tools/row_census.py $O/row_census.json 4096 > $O/census.log 2>&1
rc=$?; tail -3 $O/census.log | cut -c1-300; exit $rc
