#!/bin/bash
# Counters of the logistic NUTS kernels (lg_grad_kernel / lg_ctl_kernel), separate passes.
set -e
OUT=${1:-gpurun_out/pmc_lg}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--workload logistic --steps 40 --warmup 40 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_CACHE_MISS_sum SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p3 -o run -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
