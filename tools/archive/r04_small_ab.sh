#!/bin/bash
# small-ring kernel: parity on the current build, then an opt1/opt2 A/B against variants
set -o pipefail
TAG=${1:-r04smab}; VARS=${2:-"base"}; CFGS=${3:-"opt1"}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
[ -n "$NOTEST" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_small.py -x -q --timeout 200 --timeout-method thread > $O/pytest_small.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for C in $CFGS; do for V in $VARS; do
  if [ $V = base ]; then L=$R/concrete_amd/libconcrete_hip.so; else L=$R/variants/libconcrete_hip_$V.so; fi
  CONCRETE_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --verify ${VERIFY:-2} --no-ks --no-e2e --no-sdfg > $O/${C}_${V}_$rep.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', sys.argv[2], d['value'], d['checks'].get('bitexact'), d['roofline']['kernel_ms'])" $O/${C}_${V}_$rep.log "$C $V"
done; done; done
