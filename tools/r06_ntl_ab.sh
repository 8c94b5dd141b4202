#!/bin/bash
# Round 6: streaming loads of the spectra read once (variant ntl, GEN_NT_LOADS=1) against streaming
# stores alone (nt2 = the tree).  Usage on the GPU box: tools/r06_ntl_ab.sh TAG
TAG=${1:-r06ntl}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
L() { echo "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$1.so"; }
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_${TV:-ntl}.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -q \
  --timeout 300 --timeout-method thread > $O/pytest_${TV:-ntl}.log 2>&1 || { tail -20 $O/pytest_${TV:-ntl}.log; exit 1; }
tail -1 $O/pytest_${TV:-ntl}.log
BENCH_ARGS="--config opt8 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt8 "$(L nt2)" "$(L ${TV:-ntl})" || exit 1
BENCH_ARGS="--config opt9 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt9 "$(L nt2)" "$(L ${TV:-ntl})" || exit 1
BENCH_ARGS="--config opt10 --batch 512 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt10 "$(L nt2)" "$(L ${TV:-ntl})" || exit 1
