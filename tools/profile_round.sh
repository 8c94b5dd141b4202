#!/bin/bash
# Profile artifacts for profiles/: kernel-trace stats + HBM-traffic PMC passes, cfg2 and cfg4.
# Usage (GPU box): tools/profile_round.sh TAG
set -e -o pipefail
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --no-ks > $O/trace_$C.log 2>&1
done
cd $R
bash tools/pmc.sh $TAG/pmc_cfg2 de
bash tools/pmc.sh $TAG/pmc_cfg4 de --config cfg4
bash tools/pmc.sh $TAG/pmc_cfg2_sq abc
echo profile done
