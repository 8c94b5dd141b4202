#!/bin/bash
# Round-end evidence on the GPU box: gpu tests, smoke, default bench line, cfg4 bench line,
# kernel-trace stats (cfg2, cfg4), HBM-traffic PMC passes (cfg2, cfg4) and SQ counters (cfg2).
# Usage: tools/round_profile.sh TAG
set -e -o pipefail
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg2.log 2>&1
timeout -k 10 300 python bench.py --config cfg4 > $O/bench_cfg4.log 2>&1
bash tools/profile_round.sh $TAG
echo round_profile done
