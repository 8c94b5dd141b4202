#!/bin/bash
# GPU box: bench lines for cfg2 (default), cfg4 and opt8 on the final sources.  Usage: tools/r03s5_bench.sh TAG
set -e -o pipefail
TAG=${1:-r03s5b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_cfg2.log 2>&1
tail -1 $O/bench_cfg2.log | cut -c1-160
timeout -k 10 300 python bench.py --config cfg4 > $O/bench_cfg4.log 2>&1
tail -1 $O/bench_cfg4.log | cut -c1-160
timeout -k 10 300 python bench.py --config opt8 --steps 2 --warmup 1 > $O/bench_opt8.log 2>&1
tail -1 $O/bench_opt8.log | cut -c1-160
# (opt8 PMC passes run silently for > 3 min under the profiler: not collected here)

echo bench done
