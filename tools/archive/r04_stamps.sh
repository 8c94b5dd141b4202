#!/bin/bash
# per-phase stamps of the pair kernel at B = 512 (P = 2) and B = 4096 (P = 4)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04st}; mkdir -p $O; cd $R
CONCRETE_HIP_PBS_PAIRS=2 timeout -k 10 200 python -u tools/stamps.py 512 > $O/stamps_512.txt 2>&1 || exit 1
cat $O/stamps_512.txt
CONCRETE_HIP_PBS_PAIRS=4 timeout -k 10 200 python -u tools/stamps.py 4096 > $O/stamps_4096.txt 2>&1 || exit 1
cat $O/stamps_4096.txt
