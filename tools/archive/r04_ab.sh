#!/bin/bash
# A/B of library variants on one box: tools/r04_ab.sh TAG CONFIG "base k2a k2b ..." [extra bench args]
# base = the in-tree library; NAME = variants/libconcrete_hip_NAME.so.  Each bench runs twice, interleaved.
set -o pipefail
TAG=$1; CFG=$2; VARS=$3; shift 3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for V in $VARS; do
    if [ $V = base ]; then L=$R/concrete_amd/libconcrete_hip.so; else L=$R/variants/libconcrete_hip_$V.so; fi
    echo "$V rep$rep $(date +%T)"
    CONCRETE_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --verify 2 --no-ks --no-e2e "$@" \
      > $O/${V}_$rep.log 2>&1
    rc=$?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', d['value'], d['checks'].get('bitexact'), d['roofline']['kernel_ms'])" $O/${V}_$rep.log || exit 1
    [ $rc -eq 0 ] || exit $rc
  done
done
