#!/bin/bash
# GPU box: opt8 bench at several chunk sizes of the two-launch path (CONCRETE_HIP_GEN_CHUNK, with
# the scratch budget raised so the cap decides).  Usage: tools/chunk_ab.sh TAG CFG CHUNK...
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export CONCRETE_HIP_GEN_BUDGET_MB=16384
for C in "$@"; do
  CONCRETE_HIP_GEN_CHUNK=$C timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-ks --verify 1 > $O/bench_$C.log 2>&1
  echo "chunk $C: $(python -c "import json; d=json.loads([l for l in open('$O/bench_$C.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks']['decrypt_ok'])")"
done
