#!/bin/bash
# Round-4 GPU session F: node-IR counters, rats through the IR with the reference scheme,
# specialised kernel vs interpreter (one rocprofv3 --pmc pass per counter group).
set -e
BENCH_EXTRA="--workload rats_ir --steps 96 --warmup 32" bash tools/pmc_quick.sh gpurun_out/pmc_r4_rats_ir_jit > gpurun_out/pmc_r4_rats_ir_jit.log 2>&1
echo "jit done"
MMB_IR_JIT=0 BENCH_EXTRA="--workload rats_ir --steps 96 --warmup 32" bash tools/pmc_quick.sh gpurun_out/pmc_r4_rats_ir_interp > gpurun_out/pmc_r4_rats_ir_interp.log 2>&1
echo "interp done"
