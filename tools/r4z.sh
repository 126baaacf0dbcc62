#!/bin/bash
# Round-4 GPU session Z: every bench line of the final build (the headline with its CPU
# baseline and the PMC traffic of this build, the reference scheme priced with its own flops).
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py > gpurun_out/final/rats.json 2> gpurun_out/final/rats.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --scheme reference > gpurun_out/final/reference.json 2> gpurun_out/final/reference.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload logistic > gpurun_out/final/logistic.json 2> gpurun_out/final/logistic.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload line_amm > gpurun_out/final/line_amm.json 2> gpurun_out/final/line_amm.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload seeds_ir > gpurun_out/final/seeds_ir.json 2> gpurun_out/final/seeds_ir.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload rats_ir > gpurun_out/final/rats_ir.json 2> gpurun_out/final/rats_ir.err || exit 1
for f in gpurun_out/final/*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', '%.4g'%d['value'], r.get('bound'), round(r.get('frac'),4), r.get('frac_wall'), r.get('traffic'))"; done
