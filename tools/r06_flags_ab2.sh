#!/bin/bash
# Round 6: the AMDGPU register-pressure trackers on every kernel file (variant trkall) against the
# tree (trackers on the cfg2 files only), per optimizer row.  Usage on the GPU box: tools/r06_flags_ab2.sh TAG
TAG=${1:-r06fl2}
R=$GRAFT_REPO_ROOT; cd $R
A="CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_base.so"; Bv="CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_trkall.so"
for C in "opt1 4096" "opt3 4096" "opt4 4096" "opt6 4096" "opt7 1024" "opt8 1024" "opt9 1024"; do
  set -- $C
  BENCH_ARGS="--config $1 --batch $2 --steps 3 --warmup 1" bash tools/r05_ab.sh $TAG/$1 "$A" "$Bv" || exit 1
done
BENCH_ARGS="--global-batch 256 --steps 10 --warmup 2" bash tools/r05_ab.sh $TAG/b256 "$A" "$Bv" || exit 1
