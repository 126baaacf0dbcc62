#!/bin/bash
# Round-4 GPU session B: gpu tests on the rebuilt library (chain ordering in the kernel), the
# post-hoc check x chain-ordering A/B.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4b.log 2>&1
echo "tests_rc=$?"
timeout -k 10 600 bash tools/exp.sh base stepcheck base:MMB_ORDER_CHAINS=0 stepcheck:MMB_ORDER_CHAINS=0 base stepcheck > gpurun_out/exp_r4b.log 2>&1 || exit 1
echo "exp done"
