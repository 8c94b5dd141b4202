#!/bin/bash
# Round 6: six-wave kernel variants at B = 512 (variant $1 against the tree).  Usage: tools/r06_hex_ab.sh VARIANT TAG
V=$1; TAG=${2:-r06hx}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs.py -v \
  --timeout 200 --timeout-method thread -k "hex or split" > $O/pytest_$V.log 2>&1 || { tail -30 $O/pytest_$V.log; exit 1; }
tail -1 $O/pytest_$V.log
BENCH_ARGS="--global-batch 512 --steps 10 --warmup 2" bash tools/r05_ab.sh $TAG/b512 \
  "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_base.so" "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so" || exit 1
