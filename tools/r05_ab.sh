#!/bin/bash
# A/B of library variants on one box: tools/r05_ab.sh TAG "ENV1" "ENV2" ... ; each ENV is a set of
# VAR=value words (CONCRETE_HIP_LIB=variants/... selects a variant build); runs alternate, 2 rounds.
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 1 ${BENCH_ARGS:---global-batch 512 --steps 10}"
for round in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    echo "== round $round variant $i: $E"
    env $E timeout -k 10 200 $B > $O/v${i}_r$round.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 $O/v${i}_r$round.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open('$O/v${i}_r$round.log').read().strip().splitlines()[-1]); print('  ', d['value'], d['ms_per_step'])"
  done
done
