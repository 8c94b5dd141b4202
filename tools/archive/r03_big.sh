#!/bin/bash
# Four-step large-N step kernel: generic-path parity tests, then opt6/7/8 bench lines and a
# kernel-trace profile of opt8.  Usage: tools/r03_big.sh TAG [quick]
set -e -o pipefail
TAG=${1:-r03big}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pbs_generic.py -x -v --timeout 300 --timeout-method thread > $O/pytest_generic.log 2>&1
for C in opt6 opt7 opt8; do
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-ks > $O/bench_$C.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_opt8 -o run -- \
  python3 $R/bench.py --config opt8 --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --no-ks > $O/trace_opt8.log 2>&1
echo big done
