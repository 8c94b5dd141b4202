#!/bin/bash
# Round 6: the N = 2^15 / 2^16 split path with the S class workgroups of a polynomial placed on one XCD
# (CONCRETE_HIP_SPLIT_XCD, variant library given as $1).  Usage on the GPU box: tools/r06_split.sh LIB TAG
LIB=$1
TAG=${2:-r06sx}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 30; do date +%T >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log | cut -c1-300
  case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
}
export CONCRETE_HIP_LIB=$R/$LIB
step pytest 400 python -u -m pytest tests/test_gpu_pbs_generic.py -v --timeout 300 --timeout-method thread \
  -k "32768 or 65536 or 9bit or 10bit"
for C in "opt9 1024" "opt10 512"; do
  set -- $C
  for round in 1 2; do
    for X in 0 1; do
      CONCRETE_HIP_SPLIT_XCD=$X step b_$1_x${X}_r$round 300 python -u bench.py --config $1 --batch $2 --steps 2 --warmup 1 \
        --verify 1 --no-cpu-baseline --no-ks --no-e2e --no-sdfg --no-share
    done
  done
done
