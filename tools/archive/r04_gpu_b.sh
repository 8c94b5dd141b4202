#!/bin/bash
# Round 4 GPU pass B: the whole GPU suite (no pre-open in the SDFG test), then PMC records and
# kernel-trace stats for cfg2 / cfg4 / opt6 on the current sources.  Usage: tools/r04_gpu_b.sh TAG
TAG=${1:-r04b}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
( while sleep 30; do date +%T >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
export TMPDIR=/tmp
for C in cfg2 cfg4 opt6; do
  cd /tmp
  step trace_$C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg
  cd $GRAFT_REPO_ROOT
  step pmc_$C 600 bash tools/pmc.sh $TAG/$C abde --config $C --no-ks --no-sdfg
done
echo "pass B done"
