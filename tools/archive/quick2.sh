#!/bin/bash
# GPU box: N=1024 parity tests + cfg2 bench line (no CPU leg).  Usage: tools/quick2.sh TAG
set -e -o pipefail
TAG=${1:-q}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pbs.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pbs.log 2>&1
tail -1 $O/pytest_pbs.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ks > $O/bench.log 2>&1
python -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['kernel_ms'], d['checks'])"
