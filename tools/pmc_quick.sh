#!/bin/bash
# Quick PMC passes of the rats sweep kernel (one rocprofv3 --pmc pass per counter group, each
# under its own time limit): VALU issue, instruction mix, waits.  Usage: tools/pmc_quick.sh OUT
set -e
OUT=${1:-gpurun_out/pmcq}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 100 --warmup 50 --no-cpu-baseline $BENCH_EXTRA"
echo "pass 1"
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
echo "pass 2"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
echo "pass 3"
timeout -k 10 200 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d $OUT/p3 -o run -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
python3 tools/pmc_quick_summary.py $OUT
