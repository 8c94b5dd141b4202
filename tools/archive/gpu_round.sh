#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, kernel-trace stats, HBM-traffic PMC.  Usage: tools/gpu_round.sh TAG
set -e -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --verify 0 > $O/prof.log 2>&1
cd $R
bash tools/pmc.sh $TAG/pmc de
echo gpu_round done
