#!/bin/bash
# Round-4 evidence for the general path's large-N rows (opt6/7/8): kernel-trace stats of a short
# bench run, then the PMC passes tools/pmc_record.py turns into profiles/<tag>_<cfg>_pmc.json
# (traffic: FETCH_SIZE / WRITE_SIZE; f64 mix: SQ_INSTS_VALU_*_F64), one PBS call per pass.
# Usage: tools/r04_big_prof.sh TAG "opt6 opt7 opt8"
set -e -o pipefail
TAG=${1:-r04big}
CFGS=${2:-"opt6 opt7 opt8"}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
# heartbeat: a PMC pass over the 8-bit row runs minutes without printing
( while sleep 30; do date +%T >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
for C in $CFGS; do
  echo "trace $C $(date +%T)"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --no-ks --no-e2e \
    > $O/trace_$C.log 2>&1
  cd $R
  echo "pmc $C $(date +%T)"
  bash tools/pmc.sh $TAG/$C bde --config $C --no-ks
done
echo prof done
