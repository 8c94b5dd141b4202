#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05hex6}
mkdir -p $O
cd $R
step() { local name=$1 to=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-300; case $rc in 0) ;; *) echo "stopping after $name (rc $rc)"; exit $rc;; esac; }
B="python -u bench.py --no-cpu-baseline --no-sdfg --no-e2e --no-ks --verify 0"
CONCRETE_HIP_PBS_HEX=2 CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_noatomic.so step b512_noatomic 200 $B --global-batch 512 --steps 10
export TMPDIR=/tmp
cd /tmp
for K in pair hex; do
  [ $K = hex ] && export CONCRETE_HIP_PBS_HEX=2
  TAILN=1 step pmcb_$K 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pmcb_$K -o run -- python3 $R/bench.py --global-batch 512 --steps 1 --warmup 0 --no-cpu-baseline --verify 0 --no-e2e --no-ks --no-sdfg
  TAILN=1 step pmca_$K 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmca_$K -o run -- python3 $R/bench.py --global-batch 512 --steps 1 --warmup 0 --no-cpu-baseline --verify 0 --no-e2e --no-ks --no-sdfg
done
cd $R
for K in pair hex; do python tools/pmc_summary.py $O/pmcb_$K pbs1024; python tools/pmc_summary.py $O/pmca_$K pbs1024; done
echo done
