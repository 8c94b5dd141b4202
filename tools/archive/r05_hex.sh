#!/bin/bash
# Six-wave kernel: parity tests, then A/B against the pair kernel at B = 512 and B = 4096.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05hex}
mkdir -p $O
cd $R
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log | cut -c1-600
  case $rc in 0) ;; 1) [ "${3:-}" = "soft" ] || true;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return $rc
}
step pytest_hex 300 python -u -m pytest tests/test_gpu_pbs.py -x -v --timeout 120 --timeout-method thread -k "hex" || exit 1
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 2"
step b512_pair 200 $B --batch 512 --steps 10
CONCRETE_HIP_PBS_HEX=2 step b512_hex 200 $B --batch 512 --steps 10
step b4096_pair 200 $B --steps 5
CONCRETE_HIP_PBS_HEX=2 step b4096_hex 200 $B --steps 5
echo done
