set -e -o pipefail
cd $GRAFT_REPO_ROOT
for V in base th64; do
 for TC in 2 1; do
  if [ $V = base ]; then unset CONCRETE_HIP_LIB; else export CONCRETE_HIP_LIB=$GRAFT_REPO_ROOT/variants/libconcrete_hip_$V.so; fi
  CONCRETE_HIP_TILE_C=$TC timeout -k 10 300 python bench.py --config opt4 --batch 4096 --steps 3 --warmup 1 --no-cpu > gpurun_out/v_$V$TC.log 2>&1
  echo "$V C=$TC: $(grep '^{' gpurun_out/v_$V$TC.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["checks"])')"
 done
done
