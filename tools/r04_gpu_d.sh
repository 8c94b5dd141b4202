#!/bin/bash
# Round 4 GPU pass D: the N = 8192 one-launch kernel (CONCRETE_HIP_GEN_FUSED8=1) parity + opt7 A/B,
# opt6 PMC on the current sources.  Usage: tools/r04_gpu_d.sh TAG
TAG=${1:-r04d}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 $O/$name.log | cut -c1-600
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step fused8_test 600 env CONCRETE_HIP_GEN_FUSED8=1 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pbs_generic.py -k "7bit_k1_N8192 or (many_workgroups and N4096)"
step opt7_fused8 300 env CONCRETE_HIP_GEN_FUSED8=1 python -u bench.py --config opt7 --steps 2 --warmup 1 --no-cpu-baseline --no-ks --no-e2e
step pmc_opt6 600 bash tools/pmc.sh $TAG/opt6 abde --config opt6 --no-ks
echo "pass D done"
