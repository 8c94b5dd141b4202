#!/bin/bash
# GPU box: quick screen of variant libraries — bench line (decrypt check on every row + 8 rows
# bit-exact vs the oracle) for each.  Usage: tools/screen.sh TAG [cfg2|cfg4] NAME...
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline --no-ks > $O/bench.log 2>&1
  echo "$V: $(python -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks'])")"
done
