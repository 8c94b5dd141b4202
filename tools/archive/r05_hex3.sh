#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05hex3}
mkdir -p $O
cd $R
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-300; case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac; }
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 2"
step pytest_hex 300 python -u -m pytest tests/test_gpu_pbs.py -x -v --timeout 120 --timeout-method thread -k "hex"
CONCRETE_HIP_PBS_HEX=2 step b512_hex 200 $B --global-batch 512 --steps 10
CONCRETE_HIP_PBS_HEX=2 step b4096_hex 200 $B --steps 5
TAILN=14 step stamps512 200 python -u tools/hex_stamps.py 512
echo done
