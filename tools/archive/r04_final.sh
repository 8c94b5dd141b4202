#!/bin/bash
# Round 4 closing evidence on the final sources.  Usage: tools/r04_final.sh TAG PART
#   a: the whole GPU suite, smoke(), the default bench line, kernel-trace stats + PMC records of
#      cfg2 / cfg4 / opt4 / opt1 / opt3
#   b: kernel-trace stats + PMC records of opt6 / opt7, bench lines of every config
#   c: kernel-trace stats + PMC record of opt8 (long PMC passes)
TAG=${1:-r04f}
PART=${2:-a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 30; do date +%T >> $O/heartbeat_$PART.log; done ) &
HB=$!
trap "kill $HB" EXIT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -2 $O/$name.log | cut -c1-400
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
export TMPDIR=/tmp
prof() {  # config passes [pmc timeout]
  local C=$1 P=$2 T=${3:-240}
  cd /tmp
  step trace_$C 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg
  cd $R
  PMC_TIMEOUT=$T step pmc_$C $((T * 4 + 60)) bash tools/pmc.sh $TAG/$C $P --config $C --no-ks --no-sdfg
}
case $PART in
a)
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench_default 400 python -u bench.py
  prof cfg2 abde
  prof cfg4 abde
  prof opt4 abde
  prof opt1 bde
  prof opt3 bde
  ;;
b)
  prof opt6 bde
  prof opt7 bde 300
  for C in cfg4 opt1 opt2 opt3 opt4 opt5 opt6 opt7 opt8; do
    step bench_$C 300 python -u bench.py --config $C --no-cpu-baseline --verify 2 --no-e2e --no-sdfg
  done
  ;;
c)
  # one stream: under --pmc the profiler serialises dispatches, and the chunked two-launch path's
  # cross-stream event waits made a pass run > 600 s (r04f); the bytes and instructions of one
  # call do not depend on the stream count
  export CONCRETE_HIP_GEN_STREAMS=1
  prof opt8 bde 500
  ;;
esac
echo "part $PART done"
