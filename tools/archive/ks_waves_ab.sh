#!/bin/bash
# GPU box: four-wave keyswitch kernel parity tests, then the bench's keyswitch row with the
# eight-wave (default) and four-wave LDS kernels.  Usage: tools/ks_waves_ab.sh TAG
set -e -o pipefail
TAG=${1:-ksw}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs.py -k "keyswitch" -x -v --timeout 120 --timeout-method thread > $O/pytest_ks.log 2>&1
tail -1 $O/pytest_ks.log
for W in 8 4 8 4; do
  CONCRETE_HIP_KS_WAVES=$W timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 > $O/bench_w$W.log 2>&1
  echo "waves $W: $(python -c "import json; d=json.loads([l for l in open('$O/bench_w$W.log') if l.startswith('{')][-1]); k=d['secondary']['keyswitch']; print(k['value'], k['kernel_ms'], k['bitexact'])")"
done
