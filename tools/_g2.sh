set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_line_amm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_line.log 2>&1 || { tail -30 gpurun_out/t_line.log; exit 1; }
tail -3 gpurun_out/t_line.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 200 python bench.py --workload line_amm --no-cpu-baseline > gpurun_out/b_line.json 2> gpurun_out/b_line.err
MMB_LINE_GENERIC=1 timeout -k 10 200 python bench.py --workload line_amm --no-cpu-baseline > gpurun_out/b_line_generic.json 2> gpurun_out/b_line_generic.err
timeout -k 10 300 python bench.py > gpurun_out/b_rats.json 2> gpurun_out/b_rats.err
for f in b_line b_line_generic b_rats; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', '%.4g'%d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
