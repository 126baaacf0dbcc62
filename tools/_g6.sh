set -e
mkdir -p gpurun_out
MMB_LIB=mamba.jl_amd/lib/exp_lgn1024.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "logistic" -x -q --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
BENCH_ARGS="--workload logistic" bash tools/exp.sh lgbase lgn448 lgn1024 lgbase lgn448 lgn1024
