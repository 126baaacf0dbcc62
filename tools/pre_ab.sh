#!/bin/bash
# Sensitivity of the driver's 20-step window to the untimed AMM pre-run and the warm-up length
# (bench.py --adapt-prerun / --warmup): one bench line per setting, kernel ms per step printed.
set -e
mkdir -p gpurun_out/pre
for cfg in "128 5" "512 5" "128 100" "2000 5" "128 5" "512 5"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 20 --warmup $2 --adapt-prerun $1 --no-cpu-baseline > gpurun_out/pre/p$1_w$2.json 2> gpurun_out/pre/p$1_w$2.err
  python -c "import json; d=json.load(open('gpurun_out/pre/p$1_w$2.json')); r=d['roofline']; print('pre $1 warm $2', '%.4g' % d['value'], round(r['timed_window_kernel_ms_per_step'],4), d['config'].get('amm'))"
done
