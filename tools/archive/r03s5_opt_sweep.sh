#!/bin/bash
# GPU box: bench lines for the optimizer rows opt1..opt7 and cfg4 on the final sources (one file per
# row under gpurun_out/TAG, written as each finishes).  Usage: tools/r03s5_opt_sweep.sh TAG
set -e -o pipefail
TAG=${1:-r03s5v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in opt1 opt2 opt3 opt4 opt6 opt7; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.log 2>&1
  echo "$c: $(tail -1 $O/bench_$c.log | cut -c1-150)"
done
timeout -k 10 300 python bench.py --config cfg4 > $O/bench_cfg4.log 2>&1
echo "cfg4: $(tail -1 $O/bench_cfg4.log | cut -c1-150)"
echo sweep done
