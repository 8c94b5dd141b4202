#!/bin/bash
# GPU box: screen variant libraries on a large-N optimizer row (default opt8): bench line per
# variant (timing; diagnostic variants give wrong results).  Usage: tools/screen_big.sh TAG CFG NAME...
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 200 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-ks --verify 1 > $O/bench.log 2>&1 || true
  echo "$V: $(python -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks'])" 2>&1 | tail -1)"
done
