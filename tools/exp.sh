#!/bin/bash
# Timing experiments: run bench.py against each variant library given as arguments
# (mamba.jl_amd/lib/exp_<name>.so); one JSON line per variant into gpurun_out/exp/<name>.json.
set -e
mkdir -p gpurun_out/exp
for n in "$@"; do
  MMB_LIB=mamba.jl_amd/lib/exp_$n.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 100 \
    > gpurun_out/exp/$n.json 2> gpurun_out/exp/$n.err
  python -c "import json;d=json.load(open('gpurun_out/exp/$n.json'));print('$n', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
