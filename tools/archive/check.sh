#!/bin/bash
# GPU box: gpu tests + smoke + default bench line.  Usage: tools/check.sh TAG
set -e -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log
