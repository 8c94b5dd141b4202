#!/bin/bash
# Round 6: streaming loads on the split path, H (back kernel) or X (product kernel) alone.  Usage: tools/r06_splitnt_ab.sh TAG
TAG=${1:-r06sn}
R=$GRAFT_REPO_ROOT; cd $R
L() { echo "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$1.so"; }
BENCH_ARGS="--config opt9 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt9 "$(L base)" "$(L ntH)" "$(L ntX)" || exit 1
BENCH_ARGS="--config opt10 --batch 512 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt10 "$(L base)" "$(L ntH)" "$(L ntX)" || exit 1
