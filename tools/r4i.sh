#!/bin/bash
# Round-4 GPU session I: lane-parallel AMWG decisions (samplers.h amwg_lanes) -- rats parity
# tests (reference scheme, the three AMWG modes), then the reference-scheme A/B against the
# previous build.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "rats_parity or amwg" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4i.log 2>&1
rc=$?
echo "tests_rc=$rc"
tail -5 gpurun_out/gpu_tests_r4i.log
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scheme reference --steps 200 --warmup 100" timeout -k 10 600 bash tools/exp.sh amwgpar:MMB_AMWG_EXACT=1 amwgpar amwgpar:MMB_AMWG_EXACT=1 amwgpar > gpurun_out/exp_r4i.log 2>&1 || exit 1
cat gpurun_out/exp_r4i.log
