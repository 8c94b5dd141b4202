#!/bin/bash
# Round-3 GPU pass: multirank rehearsal, bench (cfg2 / strong-scaling batches / cfg4), kernel-trace
# stats and PMC passes (traffic + f64 mix) for tools/pmc_record.py.  Usage: tools/r03_round.sh TAG [STEPS]
set -e -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 850 --timeout-method thread > $O/multirank.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg2.log 2>&1
for G in 512 1024 2048; do
  timeout -k 10 200 python bench.py --global-batch $G --steps 10 --no-cpu-baseline --no-ks > $O/bench_cfg2_g$G.log 2>&1
done
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.log 2>&1
cd /tmp && export TMPDIR=/tmp
for C in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$C -o run -- \
    python3 $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --verify 0 > $O/trace_$C.log 2>&1
done
cd $R
bash tools/pmc.sh $TAG/pmc_cfg2 bde
bash tools/pmc.sh $TAG/pmc_cfg4 bde --config cfg4
echo round done
