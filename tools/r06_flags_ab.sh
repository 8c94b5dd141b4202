#!/bin/bash
# Round 6: LLVM scheduler options (variants built by tools/variant.sh) on cfg2 at 4096 and 512 and cfg4.
# Usage on the GPU box: tools/r06_flags_ab.sh TAG "VARIANTS"
TAG=${1:-r06fl}; VS=${2:-"base trk nocl"}
R=$GRAFT_REPO_ROOT; cd $R
ENVS=(); for V in $VS; do ENVS+=("CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so"); done
BENCH_ARGS="--global-batch 4096 --steps 10 --warmup 2" bash tools/r05_ab.sh $TAG/b4096 "${ENVS[@]}" || exit 1
BENCH_ARGS="--global-batch 512 --steps 10 --warmup 2" bash tools/r05_ab.sh $TAG/b512 "${ENVS[@]}" || exit 1
[ -n "$NOCFG4" ] || BENCH_ARGS="--config cfg4 --steps 5 --warmup 2" bash tools/r05_ab.sh $TAG/cfg4 "${ENVS[@]}" || exit 1
