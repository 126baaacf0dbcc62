#!/bin/bash
# Round-4 GPU session T: final checks of the round's build -- GPU test suite, smoke, and every
# bench line (headline with its CPU baseline, reference scheme, logistic, line AMM, node IR).
mkdir -p gpurun_out/final
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?
echo "tests_rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit 1
cat gpurun_out/final/smoke.log | tail -1
timeout -k 10 300 python bench.py > gpurun_out/final/rats.json 2> gpurun_out/final/rats.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --scheme reference > gpurun_out/final/reference.json 2> gpurun_out/final/reference.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload logistic > gpurun_out/final/logistic.json 2> gpurun_out/final/logistic.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload line_amm > gpurun_out/final/line_amm.json 2> gpurun_out/final/line_amm.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload seeds_ir > gpurun_out/final/seeds_ir.json 2> gpurun_out/final/seeds_ir.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload rats_ir > gpurun_out/final/rats_ir.json 2> gpurun_out/final/rats_ir.err || exit 1
for f in gpurun_out/final/*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', '%.4g'%d['value'], r.get('bound'), round(r.get('frac'),4), r.get('frac_wall'))"; done
