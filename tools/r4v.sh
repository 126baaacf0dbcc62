#!/bin/bash
# Round-4 GPU session V: Slice candidates per round, 4 (default) vs 8 (MMB_SLICE_NC=8) -- rats
# parity on the 8-candidate build, then the reference-scheme A/B.
mkdir -p gpurun_out
timeout -k 10 600 env MMB_LIB=mamba.jl_amd/lib/exp_nc8.so python -u -m pytest tests/test_gpu_parity.py -q -k "rats_parity or amwg or slice_overflow" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4v.log 2>&1
rc=$?
echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests_r4v.log
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scheme reference --steps 200 --warmup 100" timeout -k 10 600 bash tools/exp.sh nc4 nc8 nc4 nc8 > gpurun_out/exp_r4v.log 2>&1 || exit 1
cat gpurun_out/exp_r4v.log
