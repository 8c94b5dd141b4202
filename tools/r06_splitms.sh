#!/bin/bash
# Round 6: split-path chunk groups on several streams (variant library $1).  Usage: tools/r06_splitms.sh LIB TAG
LIB=$1; TAG=${2:-r06ms}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export CONCRETE_HIP_LIB=$R/$LIB
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -v --timeout 200 --timeout-method thread \
  -k "32768 or 65536 or 9bit or 10bit" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--config opt9 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt9 \
  "CONCRETE_HIP_GEN_STREAMS=1" "CONCRETE_HIP_GEN_STREAMS=2" "CONCRETE_HIP_GEN_STREAMS=3" || exit 1
BENCH_ARGS="--config opt10 --batch 512 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt10 \
  "CONCRETE_HIP_GEN_STREAMS=1" "CONCRETE_HIP_GEN_STREAMS=2" || exit 1
