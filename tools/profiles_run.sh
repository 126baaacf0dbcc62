#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root).  Each GPU step has its
# own time limit and the chain stops at the first failure (set -e).
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 200 --warmup 200 --no-cpu-baseline $BENCH_EXTRA"  # BENCH_EXTRA e.g. "--scheme reference"
timeout -k 10 600 python bench.py $BENCH_EXTRA > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq1 -o run -- python3 bench.py $ARGS > $OUT/pmc_sq1.log 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --output-format csv -d $OUT/pmc_sq2 -o run -- python3 bench.py $ARGS > $OUT/pmc_sq2.log 2>&1
