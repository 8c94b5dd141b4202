#!/bin/bash
# GPU box: the c-fastest product kernel (CONCRETE_HIP_MAC_SPLITC=1) — generic-path parity with it,
# then opt8 / opt7 bench lines alternating default and variant.  Usage: tools/mac_ab.sh TAG
set -e -o pipefail
TAG=${1:-mac}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
CONCRETE_HIP_MAC_SPLITC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 300 --timeout-method thread > $O/pytest_generic_splitc.log 2>&1
tail -1 $O/pytest_generic_splitc.log
i=0
for CFG in opt8 opt7; do
  for V in 0 1 0 1; do
    i=$((i + 1))
    CONCRETE_HIP_MAC_SPLITC=$V timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-ks --verify 1 > $O/bench_$i.log 2>&1
    echo "$CFG splitc=$V: $(grep '^{' $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks']['decrypt_ok'])")"
  done
done
