#!/bin/bash
# GPU box: cfg4 tests + bench for variant libraries.  Usage: tools/cfg4_variants.sh TAG NAME...
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so
  timeout -k 10 600 python -m pytest tests/test_gpu_pbs2048.py -x -q > $O/pytest.log 2>&1
  timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-ks > $O/bench4.log 2>&1
  echo "$V: $(tail -1 $O/pytest.log) $(python -c "import json; d=json.loads([l for l in open('$O/bench4.log') if l.startswith('{')][-1]); print(d['value'], d['checks'])")"
done
