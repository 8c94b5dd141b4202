#!/bin/bash
# GPU box: cfg4 parity tests, then cfg4 bench lines for the given libraries (base = the in-tree build).
# Usage: tools/cfg4_check.sh TAG NAME...
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs2048.py -x -v --timeout 200 --timeout-method thread > $O/pytest_2048.log 2>&1
for V in "$@"; do
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-ks > $O/bench_$V.log 2>&1
  echo "$V: $(python -c "import json; d=json.loads([l for l in open('$O/bench_$V.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks'])")"
done
