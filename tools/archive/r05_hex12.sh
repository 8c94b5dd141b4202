#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
bash tools/r05_ab.sh ${1:-r05ab3} "CONCRETE_HIP_PBS_HEX=2" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_nokey.so" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_nox.so" || exit 1
for V in nokey nox; do CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_$V.so python -u tools/hex_stamps.py 512 2>&1 | tail -14; done
