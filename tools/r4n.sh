#!/bin/bash
# Round-4 GPU session N: logistic gradient group layout (MMB_LG_NG x MMB_LG_NS: 32x2 default,
# 16x4, 16x2 -- half the partials the control kernel folds) against the default build.
mkdir -p gpurun_out
BENCH_ARGS="--workload logistic" timeout -k 10 900 bash tools/exp.sh base lg16x4 lg16x2 lps base lg16x4 lg16x2 lps > gpurun_out/exp_r4n.log 2>&1 || exit 1
cat gpurun_out/exp_r4n.log
for f in gpurun_out/exp/*_base.json gpurun_out/exp/*_lg16x*.json gpurun_out/exp/*_lps.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f', round(r.get('frac'),4), round(r.get('frac_wall'),4), round(r.get('avg_launch_ms'),4))"; done
