#!/bin/bash
# GPU box: bench lines for the optimizer rows on the general path.  Usage: tools/opt_bench.sh TAG "ARGS" CFG:BATCH...
set -e -o pipefail
TAG=$1; ARGS=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
for CB in "$@"; do
  C=${CB%%:*}; BT=${CB##*:}
  timeout -k 10 400 python bench.py --config $C --batch $BT $ARGS > $O/$C.log 2>&1
  echo "$C b=$BT: $(python -c "import json; d=json.loads([l for l in open('$O/$C.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['checks'], d['cpu_baseline'] and d['cpu_baseline']['value'])")"
done
