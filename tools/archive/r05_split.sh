#!/bin/bash
# PMC traffic passes of opt7 and opt8 (one stream: under --pmc dispatches serialise), split per kernel
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05split}
mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
export CONCRETE_HIP_GEN_STREAMS=1 PMC_TIMEOUT=500
for C in opt7 opt8; do
  timeout -k 10 1000 bash tools/pmc.sh ${1:-r05split}/$C de --config $C --no-ks --no-sdfg --batch ${BATCH:-1024} || exit 1
done
echo split done
