#!/bin/bash
# Timing experiments: run bench.py against each variant library given as arguments
# (mamba.jl_amd/lib/exp_<name>.so); one JSON line per variant into gpurun_out/exp/<name>.json.
# BENCH_ARGS overrides the bench arguments (default: rats, 200 timed steps after 100 warm-up).
set -e
mkdir -p gpurun_out/exp
ARGS=${BENCH_ARGS:-"--steps 200 --warmup 100"}
for n in "$@"; do
  echo "running $n"
  MMB_LIB=mamba.jl_amd/lib/exp_$n.so timeout -k 10 150 python bench.py --no-cpu-baseline $ARGS \
    > gpurun_out/exp/$n.json 2> gpurun_out/exp/$n.err
  python -c "import json;d=json.load(open('gpurun_out/exp/$n.json'));print('$n', '%.4g'%d['value'], round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
