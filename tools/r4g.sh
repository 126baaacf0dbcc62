#!/bin/bash
# Round-4 GPU session G: rats A/B -- done flag from work (DW) and the joint AMM logpdf butterfly
# (default) vs their ablations, iterations per launch 16 / 4; the GPU test suite.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4g.log 2>&1
echo "tests_rc=$?"
timeout -k 10 800 bash tools/exp.sh base doneflag logf1 base:MMB_ITERS_PER_LAUNCH=16 base:MMB_ITERS_PER_LAUNCH=4 base doneflag logf1 > gpurun_out/exp_r4g.log 2>&1 || exit 1
echo "exp done"
