#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs.py -x -q --timeout 120 --timeout-method thread -k "hex or per_stream" 2>&1 | tail -3 || exit 1
bash tools/r05_ab.sh ${1:-r05ab6} "CONCRETE_HIP_PBS_HEX=2" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_nopolysync.so" || exit 1
BENCH_ARGS="--global-batch 4096 --steps 5" bash tools/r05_ab.sh ${1:-r05ab6}_4096 "CONCRETE_HIP_PBS_HEX=2" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_nopolysync.so" || exit 1
python -u tools/hex_stamps.py 512 2>&1 | tail -14
