#!/bin/bash
# Round 6: gen_coop_kernel's hand-off payloads with the non-temporal bit (variant coopnt).  Usage: tools/r06_coopnt_ab.sh TAG
TAG=${1:-r06cn}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_coopnt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -q \
  --timeout 300 --timeout-method thread -k "coop or 8192" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--config opt7 --batch 1024 --steps 3 --warmup 1" bash tools/r05_ab.sh $TAG/opt7 \
  "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_base.so" "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_coopnt.so" || exit 1
