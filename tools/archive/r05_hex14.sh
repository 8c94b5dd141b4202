#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
bash tools/r05_ab.sh ${1:-r05ab5} "CONCRETE_HIP_PBS_HEX=2" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_prio1.so" "CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_prio2.so" || exit 1
bash tools/r05_sweep.sh ${1:-r05ab5}_sweep
