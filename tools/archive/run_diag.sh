#!/bin/bash
# timing-only runs of diagnostic variants (results are wrong by construction): bench + stamps
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so
  timeout -k 10 200 python bench.py --no-cpu-baseline --verify 0 > $O/bench.log 2>&1
  timeout -k 10 200 python tools/stamps.py > $O/stamps.log 2>&1
  echo "$V: $(python -c "import json,sys; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])")"
done
