#!/bin/bash
# GPU box: bench lines of one config under several environment settings (A/B of runtime knobs).
# Usage: tools/env_ab.sh TAG CFG "VAR=val [VAR2=val2]" ...   ("-" = no extra setting)
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
i=0
for S in "$@"; do
  i=$((i + 1))
  if [ "$S" = "-" ]; then E=""; else E="$S"; fi
  env $E timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-ks --verify 1 > $O/bench_$i.log 2>&1
  echo "[$S]: $(python -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks']['decrypt_ok'])")"
done
