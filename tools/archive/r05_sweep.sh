#!/bin/bash
# batch sweep: six-wave kernel vs the default dispatch
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05sweep}
mkdir -p $O
cd $R
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 1"
run() { local name=$1; shift; env "$@" > /dev/null; timeout -k 10 200 env "$@" $B --global-batch $GB --steps $ST > $O/$name.log 2>&1 || { echo "fail $name"; tail -3 $O/$name.log; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"; }
for GB in 256 512 768 1024 1536 2048 3072 4096; do
  ST=$(( GB >= 2048 ? 5 : 10 ))
  run hex2_$GB CONCRETE_HIP_PBS_HEX=2
  run pair_$GB CONCRETE_HIP_PBS_HEX=0
  [ $GB -le 256 ] && run hex1_$GB CONCRETE_HIP_PBS_HEX=1
done
echo done
