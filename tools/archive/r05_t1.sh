#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05t1}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 300 --timeout-method thread -k "large_n_many or configs4_atomic" > $O/pytest_large.log 2>&1; rc=$?
tail -8 $O/pytest_large.log; [ $rc -ne 0 ] && exit $rc
bash tools/r05_pmc_hex.sh ${1:-r05t1}/pmc
