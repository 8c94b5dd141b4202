#!/bin/bash
# Round-6 GPU evidence.  Usage: tools/r06.sh TAG PART
#   sweep: the split tests, then the cfg2 batch sweep (tools/batch_sweep.py)
#   suite: the whole GPU suite, smoke() and the default bench line
#   prof:  kernel-trace stats + PMC records (cfg2 at 4096 and 512, cfg4)
#   ks:    the keyswitch secondary: trace + PMC passes (int8 MFMA ops, L2 bytes)
#   opt:   bench lines + PMC records of opt9 / opt10
TAG=${1:-r06}
PART=${2:-sweep}
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
  tail -3 $O/$name.log | cut -c1-400
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
export TMPDIR=/tmp
prof() {  # config passes batch-args [pmc timeout] [suffix]
  local C=$1 P=$2 BA=$3 T=${4:-240}
  cd /tmp
  step trace_$C$5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C$5 -o run -- \
    python3 $R/bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg --no-share $BA
  cd $R
  PMC_TIMEOUT=$T step pmc_$C$5 $((T * 4 + 60)) bash tools/pmc.sh $TAG/$C$5 $P --config $C --no-ks --no-sdfg $BA
}
case $PART in
sweep)
  step pytest_split 400 python -u -m pytest tests/test_gpu_pbs.py -v --timeout 200 --timeout-method thread -k "split or hex or pair or status"
  step batch_sweep 600 python -u tools/batch_sweep.py --out $O/batch_sweep.json
  ;;
suite)
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench_default 400 python -u bench.py
  ;;
prof)
  prof cfg2 bde ""
  prof cfg2 bde "--global-batch 512" 240 _b512
  prof cfg4 bde ""
  ;;
ks)
  PMC_TIMEOUT=240 step pmc_ks 900 bash tools/pmc.sh $TAG/ks defg --no-sdfg --no-share
  ;;
optprof1)
  for C in opt1 opt2 opt3 opt4 opt5 opt6; do prof $C bde ""; done
  ;;
optprof2)
  CONCRETE_HIP_GEN_STREAMS=1 prof opt7 bde "--batch 1024" 400
  CONCRETE_HIP_GEN_STREAMS=1 prof opt8 bde "--batch 1024" 500
  CONCRETE_HIP_GEN_STREAMS=1 prof opt9 bde "--batch 1024" 500
  CONCRETE_HIP_GEN_STREAMS=1 prof opt10 bde "--batch 512" 700
  ;;
bench1)
  for C in cfg4 opt1 opt2 opt3 opt4 opt5 opt6; do
    step bench_$C 400 python -u bench.py --config $C --verify 2 --no-e2e --no-sdfg
  done
  ;;
bench2)
  for C in opt7 opt8 opt9; do
    step bench_$C 500 python -u bench.py --config $C --batch 1024 --verify 1 --no-e2e --no-sdfg
  done
  CONCRETE_HIP_GEN_COOP=0 step bench_opt7_twolaunch 500 python -u bench.py --config opt7 --batch 1024 --verify 1 --no-e2e --no-sdfg
  step bench_opt10 700 python -u bench.py --config opt10 --batch 512 --verify 1 --no-e2e --no-sdfg
  ;;
bench3)  # the general-path rows (opt6 .. opt10) after the split-path change
  step bench_opt6 400 python -u bench.py --config opt6 --verify 2 --no-e2e --no-sdfg
  for C in opt7 opt8 opt9; do
    step bench_$C 500 python -u bench.py --config $C --batch 1024 --verify 1 --no-e2e --no-sdfg
  done
  CONCRETE_HIP_GEN_COOP=0 step bench_opt7_twolaunch 500 python -u bench.py --config opt7 --batch 1024 --verify 1 --no-e2e --no-sdfg
  step bench_opt10 700 python -u bench.py --config opt10 --batch 512 --verify 1 --no-e2e --no-sdfg
  ;;
list)
  cd /tmp
  step counters 120 rocprofv3 -L
  ;;
opt9)
  CONCRETE_HIP_GEN_STREAMS=1 prof opt9 bde "--batch 1024" 500
  ;;
keybound)
  step pytest_keybound 300 python -u -m pytest tests/test_gpu_robustness.py -v --timeout 200 --timeout-method thread
  CONCRETE_HIP_GEN_STREAMS=1 PMC_TIMEOUT=600 step pmc_opt9 2460 bash tools/pmc.sh $TAG/opt9 bde --config opt9 --no-ks --no-sdfg --batch 1024
  ;;
genprof)  # every general-path row after the round-6 split-path change (pbs_generic.hip)
  prof opt6 bde ""
  CONCRETE_HIP_GEN_STREAMS=1 prof opt7 bde "--batch 1024" 400
  CONCRETE_HIP_GEN_STREAMS=1 prof opt8 bde "--batch 1024" 500
  CONCRETE_HIP_GEN_STREAMS=1 prof opt9 bde "--batch 128" 240
  CONCRETE_HIP_GEN_STREAMS=1 prof opt10 bde "--batch 64" 240
  ;;
p2prof)  # cfg4 / opt5 after the deferred limb inverses (pbs2048.hip)
  prof cfg4 bde ""
  prof opt5 bde ""
  step bench_cfg4 400 python -u bench.py --config cfg4 --verify 2 --no-e2e --no-sdfg
  ;;
bench45)
  step bench_cfg4 400 python -u bench.py --config cfg4 --verify 2 --no-e2e --no-sdfg
  step bench_opt5 400 python -u bench.py --config opt5 --verify 2 --no-e2e --no-sdfg
  ;;
pmc910)
  export CONCRETE_HIP_GEN_STREAMS=1 PMC_TIMEOUT=240
  step pmc_opt9_deb 800 bash tools/pmc.sh $TAG/opt9 deb --config opt9 --no-ks --no-sdfg --batch 128
  step pmc_opt10_deb 800 bash tools/pmc.sh $TAG/opt10 deb --config opt10 --no-ks --no-sdfg --batch 64
  ;;
opt10)
  CONCRETE_HIP_GEN_STREAMS=1 prof opt10 bde "--batch 512" 700
  ;;
*)
  echo "unknown part $PART"; exit 2
  ;;
esac
