#!/bin/bash
# Round 6, VERDICT r5 item 3: cfg4's per-limb quad syncs removed (each limb's inverse deferred past the
# next limb's first key-window barrier, P2_DEFER_INV).  Usage on the GPU box: tools/r06_cfg4_ab.sh TAG
TAG=${1:-r06c4}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_${TV:-defer}.so timeout -k 10 500 python -u -m pytest tests/test_gpu_pbs2048.py -v \
  --timeout 300 --timeout-method thread > $O/pytest_${TV:-defer}.log 2>&1 || { tail -30 $O/pytest_${TV:-defer}.log; exit 1; }
tail -1 $O/pytest_${TV:-defer}.log
BENCH_ARGS="--config cfg4 --steps 5 --warmup 2" bash tools/r05_ab.sh $TAG/cfg4 \
  "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_${AV:-nodefer}.so" "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_${TV:-defer}.so" || exit 1
