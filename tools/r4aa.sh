#!/bin/bash
# Round-4 GPU session AA: rats iterations per launch 16 (default) vs 32.
mkdir -p gpurun_out
BENCH_ARGS="--steps 384 --warmup 192" timeout -k 10 900 bash tools/exp.sh base base:MMB_ITERS_PER_LAUNCH=32 base base:MMB_ITERS_PER_LAUNCH=32 base base:MMB_ITERS_PER_LAUNCH=32 > gpurun_out/exp_r4aa.log 2>&1 || exit 1
cat gpurun_out/exp_r4aa.log
