#!/bin/bash
# GPU box: opt1 A/B of the N = 256 tile's output-group size (variants built by tools/variant.sh)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
for V in base "$@"; do
  if [ "$V" = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$GRAFT_REPO_ROOT/variants/libconcrete_hip_$V.so; fi
  tools/opt_bench.sh cp_$V "--steps 3 --warmup 1 --no-cpu" opt1:4096
done
