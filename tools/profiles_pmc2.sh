#!/bin/bash
# Instruction-fetch / LDS-pipe counters of the rats sweep kernel (separate --pmc passes).
set -e
OUT=${1:-gpurun_out/pmc2}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 100 --warmup 100 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_IFETCH SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS --output-format csv -d $OUT/p3 -o run -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
