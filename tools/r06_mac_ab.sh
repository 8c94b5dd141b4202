#!/bin/bash
# Round 6: ciphertexts per product-kernel block (MAC_CTS 8 / 16 / 32: variants built by tools/variant.sh)
# on the two-launch (opt8) and split (opt9) paths.  Usage on the GPU box: tools/r06_mac_ab.sh TAG
TAG=${1:-r06mac}
R=$GRAFT_REPO_ROOT
cd $R
for C in "opt8 1024" "opt9 1024"; do
  set -- $C
  BENCH_ARGS="--config $1 --batch $2 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/$1 \
    "CONCRETE_HIP_GEN_STREAMS=2" "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_mc8.so" \
    "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_mc32.so" || exit 1
done
