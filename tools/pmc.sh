#!/bin/bash
# PMC passes over one bench step (run on the GPU box from the repo root).
# Usage: tools/pmc.sh TAG [PASSES]   PASSES = subset of "abcdefg" (default abcde; "de" = HBM traffic only)
set -e
TAG=${1:-pmc}
PASSES=${2:-abcde}
shift 2 || true
EXTRA="$*"   # extra bench.py arguments (e.g. --config cfg4)
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp PYTHONUNBUFFERED=1 CONCRETE_BENCH_PROGRESS=1
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 ${PMC_TIMEOUT:-240} rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --verify 0 --no-e2e --no-share $EXTRA > $OUT/$name.log 2>&1
}
# HBM traffic passes first (a later pass that fails or hangs leaves them in place)
[[ $PASSES == *d* ]] && run d FETCH_SIZE
[[ $PASSES == *e* ]] && run e WRITE_SIZE TCC_HIT TCC_MISS
[[ $PASSES == *a* ]] && run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
[[ $PASSES == *b* ]] && run b SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_INSTS_SALU
[[ $PASSES == *c* ]] && run c SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_CVT SQ_LDS_ADDR_CONFLICT
# matrix-core and L2 passes (the keyswitch's int8 MFMA kernel, round 6)
[[ $PASSES == *f* ]] && run f SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
[[ $PASSES == *g* ]] && run g TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum
echo pmc done
