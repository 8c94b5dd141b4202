#!/bin/bash
# Round-5 closing evidence on the final sources.  Usage: tools/r05_final.sh TAG PART
#   a: GPU suite, smoke(), the default bench line, kernel-trace stats + PMC records of cfg2 (4096,
#      pair kernel) and cfg2 at 512 (six-wave kernel), cfg4
#   b: kernel-trace stats + PMC records of opt1..opt6 (batch 4096)
#   c: the N = 8192 tests, PMC records of opt6 (4096), opt7 / opt8 (batch 1024, one stream under --pmc)
#   d: bench lines of cfg4, opt1..opt6 (CPU baseline, bit-exact rows)
#   e: bench lines of opt7..opt10 (opt7 also on the two-launch path)
#   f: the GPU suite, smoke() and the default bench line again (after the PMC records are in)
#   g: after a general-path edit: the N = 8192 tests, PMC records and bench lines of opt6..opt8
#   h: the opt6..opt8 bench lines again, once g's records are committed (bench.py attaches them)
TAG=${1:-r05f}
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
  tail -2 $O/$name.log | cut -c1-300
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
export TMPDIR=/tmp
prof() {  # config passes batch-args [pmc timeout]
  local C=$1 P=$2 BA=$3 T=${4:-240}
  cd /tmp
  step trace_$C$5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C$5 -o run -- \
    python3 $R/bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg --no-share $BA
  cd $R
  PMC_TIMEOUT=$T step pmc_$C$5 $((T * 4 + 60)) bash tools/pmc.sh $TAG/$C$5 $P --config $C --no-ks --no-sdfg $BA
}
case $PART in
a)
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench_default 400 python -u bench.py
  prof cfg2 bde ""
  prof cfg2 bde "--global-batch 512" 240 _b512
  prof cfg4 bde ""
  ;;
b)
  for C in opt1 opt2 opt3 opt4 opt5 opt6; do prof $C bde ""; done
  ;;
c)
  step pytest_coop 400 python -u -m pytest tests/test_gpu_pbs_generic.py -v --timeout 200 --timeout-method thread -k "coop or N8192"
  prof opt6 bde ""
  export CONCRETE_HIP_GEN_STREAMS=1
  prof opt7 bde "--batch 1024" 400
  prof opt8 bde "--batch 1024" 500
  ;;
d)
  for C in cfg4 opt1 opt2 opt3 opt4 opt5 opt6; do
    step bench_$C 400 python -u bench.py --config $C --verify 2 --no-e2e --no-sdfg
  done
  ;;
e)
  step pytest_coop_e 400 python -u -m pytest tests/test_gpu_pbs_generic.py -v --timeout 200 --timeout-method thread -k "coop"
  for C in opt7 opt8 opt9; do
    step bench_$C 500 python -u bench.py --config $C --batch 1024 --verify 1 --no-e2e --no-sdfg
  done
  CONCRETE_HIP_GEN_COOP=0 step bench_opt7_twolaunch 500 python -u bench.py --config opt7 --batch 1024 --verify 1 --no-e2e --no-sdfg
  step bench_opt10 700 python -u bench.py --config opt10 --batch 512 --verify 1 --no-e2e --no-sdfg
  ;;
g)
  step pytest_coop_g 400 python -u -m pytest tests/test_gpu_pbs_generic.py -v --timeout 200 --timeout-method thread -k "coop or N8192"
  prof opt6 bde ""
  CONCRETE_HIP_GEN_STREAMS=1 prof opt7 bde "--batch 1024" 400
  CONCRETE_HIP_GEN_STREAMS=1 prof opt8 bde "--batch 1024" 500
  step bench_opt6 400 python -u bench.py --config opt6 --verify 2 --no-e2e --no-sdfg
  for C in opt7 opt8; do
    step bench_$C 500 python -u bench.py --config $C --batch 1024 --verify 1 --no-e2e --no-sdfg
  done
  CONCRETE_HIP_GEN_COOP=0 step bench_opt7_twolaunch 500 python -u bench.py --config opt7 --batch 1024 --verify 1 --no-e2e --no-sdfg
  ;;
h)
  step bench_opt6 400 python -u bench.py --config opt6 --verify 2 --no-e2e --no-sdfg
  for C in opt7 opt8; do
    step bench_$C 500 python -u bench.py --config $C --batch 1024 --verify 1 --no-e2e --no-sdfg
  done
  ;;
f)
  step pytest_gpu_f 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
  step smoke_f 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench_default 400 python -u bench.py
  ;;
esac
echo "part $PART done"
