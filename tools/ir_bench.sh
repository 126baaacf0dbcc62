#!/bin/bash
# Node-IR workloads on the GPU box: bench lines (+ the hand-fused rats reference scheme for
# comparison) and a rocprofv3 kernel trace of the seeds IR sweep.  Run via gpurun from the
# repo root; each GPU step has its own time limit, the chain stops at the first failure.
set -e
OUT=${1:-gpurun_out/ir_bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload seeds_ir > $OUT/seeds_ir.json 2> $OUT/seeds_ir.err
timeout -k 10 300 python bench.py --workload rats_ir > $OUT/rats_ir.json 2> $OUT/rats_ir.err
timeout -k 10 300 python bench.py --workload rats --scheme reference --no-cpu-baseline > $OUT/rats_ref.json 2> $OUT/rats_ref.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload seeds_ir --no-cpu-baseline > $OUT/trace.log 2>&1
