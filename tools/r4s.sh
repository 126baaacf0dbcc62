#!/bin/bash
# Round-4 GPU session S: logistic gradient kernel with double-buffered X staging (MMB_LG_DB:
# one barrier per 32-row pass instead of two) against the default build.
mkdir -p gpurun_out
BENCH_ARGS="--workload logistic" timeout -k 10 900 bash tools/exp.sh base lgdb base lgdb > gpurun_out/exp_r4s.log 2>&1 || exit 1
cat gpurun_out/exp_r4s.log
for f in gpurun_out/exp/*_base.json gpurun_out/exp/*_lgdb.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f', round(r.get('frac'),4), round(r.get('frac_wall'),4), round(r.get('avg_launch_ms'),4))"; done
