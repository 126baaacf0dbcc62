#!/bin/bash
# Round-4 GPU session W: Slice candidate evaluation with memoised candidate-independent pieces
# (prior terms of the other nodes, target scale) -- rats parity, then the reference-scheme A/B.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "rats_parity or amwg or slice_overflow" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4w.log 2>&1
rc=$?
echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests_r4w.log
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scheme reference --steps 200 --warmup 100" timeout -k 10 600 bash tools/exp.sh nc4 memo nc4 memo > gpurun_out/exp_r4w.log 2>&1 || exit 1
cat gpurun_out/exp_r4w.log
