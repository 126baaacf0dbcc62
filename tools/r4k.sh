#!/bin/bash
# Round-4 GPU session K: logistic control kernel at 4 waves per SIMD (one round for 4096 chains;
# MMB_LG_CTL_WAVES=4, 128 VGPRs with spills) against the default build.
mkdir -p gpurun_out
BENCH_ARGS="--workload logistic" timeout -k 10 600 bash tools/exp.sh base ctl4 base ctl4 > gpurun_out/exp_r4k.log 2>&1 || exit 1
cat gpurun_out/exp_r4k.log
for f in gpurun_out/exp/*_base.json gpurun_out/exp/*_ctl4.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f', r.get('frac'), r.get('frac_wall'), r.get('avg_launch_ms'))"; done
