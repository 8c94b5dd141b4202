#!/bin/bash
# Round 4: the small-ring kernel (pbs_small.hip) — parity, the general-path tests whose cases moved,
# then opt1 / opt3 benches.
set -o pipefail
TAG=${1:-r04small}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "pytest small $(date +%T)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_small.py -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_small.log 2>&1
rc=$?; echo "  rc=$rc"; tail -4 $O/pytest_small.log
[ $rc -eq 0 ] || exit $rc
echo "pytest generic $(date +%T)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs_generic.py -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_generic.log 2>&1
rc=$?; echo "  rc=$rc"; tail -3 $O/pytest_generic.log
[ $rc -eq 0 ] || exit $rc
for C in opt1 opt3 opt2; do
  echo "bench $C $(date +%T)"
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --verify 2 --no-ks --no-e2e --no-sdfg > $O/bench_$C.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', d['value'], d['checks'].get('bitexact'), d['checks'].get('decrypt_ok'), d['roofline']['kernel_ms'])" $O/bench_$C.log
done
