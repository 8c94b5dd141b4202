#!/bin/bash
# Round-3 evidence pass (GPU box): kernel-trace stats and HBM-traffic PMC for the large-N optimizer
# rows (opt6/7/8), SQ counters for the small-batch cfg2 kernel (B = 512, 2 ciphertexts per
# workgroup) next to B = 4096.  Usage: tools/r03_evidence.sh TAG
set -e -o pipefail
TAG=${1:-r03ev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in opt6 opt7 opt8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --verify 1 --no-ks > $O/trace_$C.log 2>&1
done
cd $R
for C in opt6 opt8; do
  bash tools/pmc.sh $TAG/pmc_$C de --config $C --no-ks
  bash tools/pmc.sh $TAG/pmc_${C}_sq a --config $C --no-ks
done
bash tools/pmc.sh $TAG/pmc_cfg2_b512 ab --global-batch 512 --no-ks
bash tools/pmc.sh $TAG/pmc_cfg2_b4096 a --no-ks
echo evidence done
