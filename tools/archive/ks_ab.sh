#!/bin/bash
# GPU box: keyswitch A/B of variant libraries on the cfg2 bench's secondary KS line.
# Usage: tools/ks_ab.sh TAG NAME...
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  O=$R/gpurun_out/$TAG/$V; mkdir -p $O
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench.log 2>&1
  echo "$V: $(python -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); k=d['secondary']['keyswitch']; print(d['value'], k['value'], k['kernel_ms'], k['bitexact'])")"
done
