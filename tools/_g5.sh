set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_line_amm.py tests/test_gpu_ir.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -40 gpurun_out/t5.log; exit 1; }
tail -3 gpurun_out/t5.log
