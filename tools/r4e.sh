#!/bin/bash
# Round-4 GPU session E: profiles of the final headline build (rats Gibbs+AMM: kernel trace, HBM
# bytes, SQ counters over the bench's timed window), the f1 reference scheme, the logistic
# config window (bench line + kernel trace), the node-IR benches with their CPU baselines, and
# the GPU test suite.
set -e
mkdir -p gpurun_out
bash tools/profiles_run.sh gpurun_out/prof_r4e > gpurun_out/prof_r4e.log 2>&1
echo "rats profiles done"
BENCH_EXTRA="--scheme reference" bash tools/profiles_run.sh gpurun_out/prof_r4e_ref > gpurun_out/prof_r4e_ref.log 2>&1
echo "f1 profiles done"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload logistic > gpurun_out/r4e_logistic.json 2> gpurun_out/r4e_logistic.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4e_lg_trace -o run -- python3 bench.py --workload logistic --no-cpu-baseline > gpurun_out/r4e_lg_trace.log 2>&1
echo "logistic done"
for w in seeds_ir rats_ir; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/r4e_${w}.json 2> gpurun_out/r4e_${w}.err
done
echo "ir done"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4e.log 2>&1
echo "tests_rc=$?"
