set -e
mkdir -p gpurun_out
MMB_LIB=mamba.jl_amd/lib/exp_v3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_line_amm.py tests/test_gpu_parity.py -k "line" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_line3.log 2>&1 || { tail -30 gpurun_out/t_line3.log; exit 1; }
tail -2 gpurun_out/t_line3.log
BENCH_ARGS="--workload line_amm" bash tools/exp.sh v1 v3 v1 v3
BENCH_ARGS="--workload line_amm --steps 20 --warmup 5" bash tools/exp.sh profv3
grep MMB_PROF gpurun_out/exp/profv3.err | grep line
