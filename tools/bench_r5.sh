#!/bin/bash
# Round-5 final bench lines (run via gpurun from the repo root), each step under its own limit.
set -e
OUT=${1:-gpurun_out/r5bench}
mkdir -p $OUT
run() { n=$1; shift; echo "$n"; timeout -k 10 400 python bench.py "$@" > $OUT/$n.json 2> $OUT/$n.err; }
run rats_default
run rats_driver --gpus 1 --steps 20 --warmup 5
run rats_400 --steps 400 --warmup 20 --no-cpu-baseline
run rats_reference --scheme reference
run logistic --workload logistic
run logistic_forward --workload logistic --gradient forward --no-cpu-baseline
run line_amm --workload line_amm
run seeds_ir --workload seeds_ir
run rats_ir --workload rats_ir
echo "torchrun nccl 1 rank"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/torchrun1.json 2> $OUT/torchrun1.err
