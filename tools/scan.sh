#!/bin/bash
# Throughput vs chains per GPU and iterations per launch (rats Gibbs+AMM), one JSON line each.
set -e
mkdir -p gpurun_out/scan
for cfg in "16384 8" "32768 8" "65536 8" "16384 4" "16384 16" "16384 2"; do
  set -- $cfg
  MMB_ITERS_PER_LAUNCH=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 160 --warmup 80 --chains $1 \
    > gpurun_out/scan/c$1_w$2.json 2> gpurun_out/scan/c$1_w$2.err
  python -c "import json;d=json.load(open('gpurun_out/scan/c$1_w$2.json'));print('chains $1 W $2', '%.3e'%d['value'], round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
