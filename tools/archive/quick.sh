#!/bin/bash
# GPU-box quick check: all gpu tests, cfg2 + cfg4 bench lines, stamps.  Usage: tools/quick.sh TAG
set -e -o pipefail
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ks > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-ks > $O/bench4.log 2>&1
timeout -k 10 200 python tools/stamps.py > $O/stamps.log 2>&1
echo done
