#!/bin/bash
# Round-4 GPU session A: the gpu test suite, the pchol32 post-hoc-check A/B, the node-IR benches
# (specialised kernel vs interpreter) and the default bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4a.log 2>&1
echo "tests_rc=$?"
timeout -k 10 500 bash tools/exp.sh base base:MMB_ORDER_CHAINS=0 stepcheck base base:MMB_ORDER_CHAINS=0 stepcheck > gpurun_out/exp_r4a.log 2>&1 || exit 1
echo "exp done"
for w in seeds_ir rats_ir; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/r4a_${w}_jit.json 2> gpurun_out/r4a_${w}_jit.err || exit 1
  MMB_IR_JIT=0 timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/r4a_${w}_interp.json 2> gpurun_out/r4a_${w}_interp.err || exit 1
done
echo "ir done"
timeout -k 10 200 python tools/lg_walltime.py --out gpurun_out/r4a_lg_walltime.json > gpurun_out/r4a_lg_walltime.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4a_lg_trace -o run -- python3 tools/lg_walltime.py --trace-only > gpurun_out/r4a_lg_trace.log 2>&1 || exit 1
python tools/lg_trace_split.py gpurun_out/r4a_lg_trace --out gpurun_out/r4a_lg_split.json
echo "lg done"
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench_default.json 2> gpurun_out/r4a_bench_default.err
echo "bench_rc=$?"
