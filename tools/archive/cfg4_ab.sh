#!/bin/bash
# GPU box: cfg4 parity tests of the current tree, then bench A/B vs saved variants.
# Usage: tools/cfg4_ab.sh TAG VARIANT...
set -e -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs2048.py -x -q --timeout 120 --timeout-method thread > $O/pytest4.log 2>&1
tail -2 $O/pytest4.log
bash tools/screen.sh $TAG cfg4 base "$@"
