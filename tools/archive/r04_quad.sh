#!/bin/bash
# Round 4: the four-wave small-batch N = 1024 kernel (pbs1024_quad.hip): parity, then cfg2 at small
# global batches with it (default / forced ciphertexts per workgroup) and without it.
set -o pipefail
TAG=${1:-r04quad}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "pytest pairs $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs.py -x -v -k "pairs_per_workgroup" --timeout 200 --timeout-method thread \
  > $O/pytest_pairs.log 2>&1
rc=$?; echo "  rc=$rc"; tail -3 $O/pytest_pairs.log
[ $rc -eq 0 ] || exit $rc
row() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', d['value'], d['checks'].get('bitexact'), d['checks'].get('decrypt_ok'), d['roofline']['kernel_ms'])" $1; }
for b in 512 256; do
  for q in def 0 1 2; do
    echo "b$b quad=$q $(date +%T)"
    if [ $q = def ]; then unset CONCRETE_HIP_PBS_QUAD; else export CONCRETE_HIP_PBS_QUAD=$q; fi
    timeout -k 10 200 python -u bench.py --global-batch $b --steps 20 --no-cpu-baseline --verify 4 --no-ks --no-e2e > $O/b${b}_q$q.log 2>&1 || exit 1
    row $O/b${b}_q$q.log
  done
done
unset CONCRETE_HIP_PBS_QUAD
for b in 1024 4096; do
  echo "b$b $(date +%T)"
  timeout -k 10 200 python -u bench.py --global-batch $b --no-cpu-baseline --verify 4 --no-ks --no-e2e > $O/b$b.log 2>&1 || exit 1
  row $O/b$b.log
done
