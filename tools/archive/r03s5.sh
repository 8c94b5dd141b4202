#!/bin/bash
# Round-3 session-5 GPU pass: gpu tests, smoke, cfg2 bench, then opt8 under chunk / stream
# settings of the two-launch path (small chunks keep a group's X / Y spectra within the MALL).
# Usage: tools/r03s5.sh TAG
set -e -o pipefail
TAG=${1:-r03s5}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg2.log 2>&1
tail -1 $O/bench_cfg2.log | cut -c1-200
bash tools/env_ab.sh $TAG/opt8 opt8 "-" "CONCRETE_HIP_GEN_CHUNK=128 CONCRETE_HIP_GEN_STREAMS=2" \
  "CONCRETE_HIP_GEN_CHUNK=128 CONCRETE_HIP_GEN_STREAMS=4" "CONCRETE_HIP_GEN_CHUNK=64 CONCRETE_HIP_GEN_STREAMS=4" \
  "CONCRETE_HIP_GEN_CHUNK=256 CONCRETE_HIP_GEN_STREAMS=4"
echo r03s5 done
