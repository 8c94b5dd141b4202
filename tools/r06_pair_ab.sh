#!/bin/bash
# Round 6: the pair kernel's per-limb pair syncs removed (each limb's inverse deferred past the next
# limb's first key-window barrier, PAIR_DEFER_INV).  Usage on the GPU box: tools/r06_pair_ab.sh TAG
TAG=${1:-r06pd}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_pdefer.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pbs.py -v \
  --timeout 300 --timeout-method thread > $O/pytest_pdefer.log 2>&1 || { tail -30 $O/pytest_pdefer.log; exit 1; }
tail -1 $O/pytest_pdefer.log
BENCH_ARGS="--global-batch 4096 --steps 10 --warmup 2" bash tools/r05_ab.sh $TAG/b4096 \
  "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_pbase.so" "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_pdefer.so" || exit 1
