#!/bin/bash
# GPU box: opt8 timing with diagnostic builds of the generic path (wrong results by design:
# DG_NOY no Y loads, DG_NOCOL no column DFTs, DG_NOROW no row transforms, DG_NOFRONT no forward
# side).  Usage: tools/diag_opt8.sh TAG NAME...   (base = the in-tree build)
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for V in "$@"; do
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so; fi
  timeout -k 10 300 python bench.py --config opt8 --steps 1 --warmup 1 --no-cpu-baseline --no-ks --verify 0 > $O/bench_$V.log 2>&1
  echo "$V: $(grep '^{' $O/bench_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])")"
done
