#!/bin/bash
# PMC evidence on the current kernel sources (GPU box): cfg2 at the metric's batch (every pass),
# cfg2 at B = 512 (SQ mix, the strong-scaling question), cfg4 (traffic + f64 mix + SQ waits).
# tools/pmc_record.py turns the b/d/e passes into the profiles/*_pmc.json records bench.py reads.
# Usage: tools/r03_pmc.sh TAG
set -e -o pipefail
TAG=${1:-r03pmc}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc.sh $TAG/cfg2 abcde --no-ks
bash tools/pmc.sh $TAG/cfg2_b512 ab --global-batch 512 --no-ks
bash tools/pmc.sh $TAG/cfg4 abde --config cfg4 --no-ks
echo pmc evidence done
