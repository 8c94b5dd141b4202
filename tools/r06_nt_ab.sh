#!/bin/bash
# Round 6: streaming (non-temporal) stores of the spectra / accumulators the next launch reads
# (GEN_NT_STORES: 1 = two-launch X and Y, 2 = also the accumulators and the split path), variants
# built by tools/variant.sh.  Usage on the GPU box: tools/r06_nt_ab.sh TAG
TAG=${1:-r06nt}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
L() { echo "CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$1.so"; }
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_nt2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -q \
  --timeout 300 --timeout-method thread > $O/pytest_nt2.log 2>&1 || { tail -20 $O/pytest_nt2.log; exit 1; }
tail -1 $O/pytest_nt2.log
BENCH_ARGS="--config opt8 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt8 "$(L base)" "$(L nt)" "$(L nt2)" || exit 1
BENCH_ARGS="--config opt9 --batch 1024 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt9 "$(L base)" "$(L nt2)" || exit 1
BENCH_ARGS="--config opt10 --batch 512 --steps 2 --warmup 1" bash tools/r05_ab.sh $TAG/opt10 "$(L base)" "$(L nt2)" || exit 1
BENCH_ARGS="--config opt6 --steps 3 --warmup 1" bash tools/r05_ab.sh $TAG/opt6 "$(L base)" "$(L nt2)" || exit 1
