# final-build profiles (round 3): rats gibbs_amm (metric), rats reference scheme, line AMM, logistic
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
echo rats; bash tools/profiles_run.sh gpurun_out/prof_r3f
echo ref; bash tools/profiles_ref.sh gpurun_out/prof_ref_r3f profiles/r3_rats_reference
echo line
timeout -k 10 300 python bench.py --workload line_amm > gpurun_out/line_bench.json 2> gpurun_out/line_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/line_trace -o run -- python3 bench.py --workload line_amm --no-cpu-baseline > gpurun_out/line_trace.log 2>&1
echo logistic
timeout -k 10 400 python bench.py --workload logistic > gpurun_out/lg_bench.json 2> gpurun_out/lg_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lg_trace -o run -- python3 bench.py --workload logistic --no-cpu-baseline > gpurun_out/lg_trace.log 2>&1
echo final bench
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
cat gpurun_out/final_bench.json
