#!/bin/bash
# PMC passes a/b/c over one B=512 step of the six-wave kernel
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05pmchex}
mkdir -p $O
export TMPDIR=/tmp CONCRETE_HIP_PBS_HEX=${HEX:-2}
cd /tmp
run() { local name=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 $R/bench.py --global-batch 512 --steps 1 --warmup 0 --no-cpu-baseline --verify 0 --no-e2e --no-ks --no-sdfg > $O/$name.log 2>&1 || exit 1; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run b SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_INSTS_SALU
run c SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_CVT SQ_LDS_ADDR_CONFLICT
echo pmc done
