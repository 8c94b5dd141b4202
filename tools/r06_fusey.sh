#!/bin/bash
# Round 6, VERDICT r5 item 1: the N = 16384 step kernel with the products fused into its inverse side
# (MODE_FUSEY, CONCRETE_HIP_GEN_FUSEDY=1; variants built by tools/variant.sh fusey / fuseysb).
# Usage on the GPU box: tools/r06_fusey.sh TAG
TAG=${1:-r06fy}
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
  tail -3 $O/$name.log | cut -c1-400
  case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
}
export TMPDIR=/tmp
FY=$R/variants/libconcrete_hip_fusey.so
FYSB=$R/variants/libconcrete_hip_fuseysb.so
FYNP=$R/variants/libconcrete_hip_fuseynp.so
CONCRETE_HIP_LIB=$FY CONCRETE_HIP_GEN_FUSEDY=1 step pytest_fusey 500 python -u -m pytest tests/test_gpu_pbs_generic.py \
  -v --timeout 300 --timeout-method thread -k "N16384 and not wide_state"
CONCRETE_HIP_LIB=$FYNP CONCRETE_HIP_GEN_FUSEDY=1 step pytest_fuseynp 400 python -u -m pytest tests/test_gpu_pbs_generic.py \
  -v --timeout 300 --timeout-method thread -k "N16384 and not wide_state and not chunked"
BENCH_ARGS="--config opt8 --batch 1024 --steps 3 --warmup 1" step ab 900 bash tools/r05_ab.sh $TAG/ab \
  "CONCRETE_HIP_LIB=$FY CONCRETE_HIP_GEN_FUSEDY=0" "CONCRETE_HIP_LIB=$FY CONCRETE_HIP_GEN_FUSEDY=1" \
  "CONCRETE_HIP_LIB=$FYSB CONCRETE_HIP_GEN_FUSEDY=1" "CONCRETE_HIP_LIB=$FYNP CONCRETE_HIP_GEN_FUSEDY=1"
cd /tmp
for V in 0 1; do
  CONCRETE_HIP_LIB=$FY CONCRETE_HIP_GEN_FUSEDY=$V CONCRETE_HIP_GEN_STREAMS=1 step trace_fy$V 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/trace_fy$V -o run -- python3 $R/bench.py --config opt8 --batch 1024 --steps 2 --warmup 1 \
    --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg --no-share
done
