set -e
mkdir -p gpurun_out
timeout -k 10 400 env MMB_LIB=mamba.jl_amd/lib/exp_all5.so python -u -m pytest tests/test_gpu_parity.py -x -q -k "rats" --timeout 120 --timeout-method thread > gpurun_out/t_all5.log 2>&1
tail -3 gpurun_out/t_all5.log
bash tools/exp.sh base all4 all5 base all5
BENCH_ARGS="--workload line_amm --steps 20 --warmup 5" bash tools/exp.sh prof
grep MMB_PROF gpurun_out/exp/prof.err | head -20
