#!/bin/bash
# Round-3 first probe (GPU box): cfg2 throughput vs batch (strong-scaling question), cfg4 SQ counters.
# Usage: tools/r03_probe.sh TAG
set -e -o pipefail
TAG=${1:-r03probe}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for B in 256 512 1024 2048 4096; do
  timeout -k 10 200 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu-baseline --verify 4 --no-ks > $O/cfg2_b$B.log 2>&1
done
bash tools/pmc.sh $TAG/pmc_cfg4_sq abc --config cfg4
echo probe done
