#!/bin/bash
# Round 6: the split path's slot spectra split by class in the product kernel (HPRE), with and without
# the next slot prefetched in the back kernel, against the XCD-placement-only build.
# Usage on the GPU box: tools/r06_split2.sh TAG
TAG=${1:-r06sh}
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
  tail -2 $O/$name.log | cut -c1-220
  case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
}
for V in ${TESTV:-splith splithnp}; do
  CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so step pytest_$V 300 python -u -m pytest tests/test_gpu_pbs_generic.py -v \
    --timeout 200 --timeout-method thread -k "32768 or 65536 or 9bit or 10bit"
done
B="python -u bench.py --steps 2 --warmup 1 --verify 1 --no-cpu-baseline --no-ks --no-e2e --no-sdfg --no-share"
for round in 1 2; do
  for V in ${ABV:-splitxcd splith splithnp}; do
    CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so step b_opt9_${V}_r$round 200 $B --config opt9 --batch 1024
  done
done
for V in ${ABV:-splitxcd splith splithnp}; do
  CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so step b_opt10_$V 300 $B --config opt10 --batch 512
done
