#!/bin/bash
# Round-4 GPU session M: Slice shrink candidates four at a time on the rats scalar blocks
# (samplers.h slice_uni_cand / slice_multi_cand) -- rats parity + overflow tests, then the
# reference-scheme A/B (MMB_AMWG_EXACT=1: sequential AMWG and Slice).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -k "rats or amwg" --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_r4m.log 2>&1
rc=$?
echo "tests_rc=$rc"
tail -5 gpurun_out/gpu_tests_r4m.log
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scheme reference --steps 200 --warmup 100" timeout -k 10 600 bash tools/exp.sh slc:MMB_AMWG_EXACT=1 slc slc:MMB_AMWG_EXACT=1 slc > gpurun_out/exp_r4m.log 2>&1 || exit 1
cat gpurun_out/exp_r4m.log
