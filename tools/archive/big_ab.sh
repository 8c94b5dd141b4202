#!/bin/bash
# GPU box: generic-path parity tests on the in-tree build, then bench lines of a large-N row for
# the in-tree build (base) and variant libraries.  Usage: tools/big_ab.sh TAG CFG NAME...
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 300 --timeout-method thread > $O/pytest_generic.log 2>&1
tail -1 $O/pytest_generic.log
for V in "$@"; do
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-ks --verify 2 > $O/bench_$V.log 2>&1
  echo "$V: $(python -c "import json; d=json.loads([l for l in open('$O/bench_$V.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks'])")"
done
