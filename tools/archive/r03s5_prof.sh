#!/bin/bash
# Round-3 session-5 evidence on the final kernel sources: kernel-trace stats (cfg2, cfg4) and the
# PMC passes tools/pmc_record.py turns into the profiles/*_pmc.json records bench.py reads.
# Usage: tools/r03s5_prof.sh TAG
set -e -o pipefail
TAG=${1:-r03s5p}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --verify 0 > $O/trace_$C.log 2>&1
done
cd $R
bash tools/pmc.sh $TAG/cfg2 abcde --no-ks
bash tools/pmc.sh $TAG/cfg4 abde --config cfg4 --no-ks
echo prof done
