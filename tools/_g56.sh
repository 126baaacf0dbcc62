set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_line_amm.py tests/test_gpu_ir.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -40 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
MMB_LIB=mamba.jl_amd/lib/exp_v4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_line_amm.py tests/test_gpu_parity.py -k "line" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_v4.log 2>&1 || { tail -30 gpurun_out/t_v4.log; exit 1; }
tail -2 gpurun_out/t_v4.log
cp mamba.jl_amd/lib/libmambahip.so mamba.jl_amd/lib/exp_v3.so
BENCH_ARGS="--workload line_amm" bash tools/exp.sh v3 v4 v3 v4
bash tools/_g6.sh
