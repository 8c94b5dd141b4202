#!/bin/bash
# On the GPU box: for each variant NAME, gpu tests + bench + stamps with variants/libconcrete_hip_NAME.so
# Usage: tools/run_variants.sh TAG NAME...
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so
  timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
  timeout -k 10 200 python tools/stamps.py > $O/stamps.log 2>&1
  echo "$V: $(tail -1 $O/pytest.log) $(python -c "import json,sys; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['checks'])")"
done
