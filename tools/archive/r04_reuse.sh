#!/bin/bash
# fused N = 4096 kernel: key limbs read once per step (FUSED_REUSE) — parity, then A/B against the
# slot-by-slot form (variants/libconcrete_hip_noreuse.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04reuse}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 200 --timeout-method thread -k "N4096" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/r04_ab.sh ${1:-r04reuse} opt6 "base noreuse"
