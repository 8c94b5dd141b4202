#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05hex2}
mkdir -p $O
cd $R
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -12 $O/$name.log | cut -c1-300; case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac; }
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 2"
step b512_pair 200 $B --global-batch 512 --steps 10
CONCRETE_HIP_PBS_HEX=2 step b512_hex 200 $B --global-batch 512 --steps 10
step stamps512 200 python -u tools/hex_stamps.py 512
step stamps4096 200 python -u tools/hex_stamps.py 4096
echo done
