#!/bin/bash
# Round-4 GPU session D: rats A/B -- chain order by validity class only vs class + mean rank,
# next-block AMM tune prefetch; parity tests of the changed paths.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "rats or amm_stats or order" > gpurun_out/gpu_tests_r4d.log 2>&1
echo "tests_rc=$?"
timeout -k 10 600 bash tools/exp.sh base base:MMB_ORDER_RANK=0 prefetch base base:MMB_ORDER_RANK=0 prefetch > gpurun_out/exp_r4d.log 2>&1 || exit 1
echo "exp done"
