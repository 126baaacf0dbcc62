#!/bin/bash
# Round-4 GPU session P: rank-deficiency certificates (samplers.h amm_cert) -- the GPU test
# suite, then the headline A/B against MMB_AMM_CERT=0 (every update factorized).
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4p.log 2>&1
rc=$?
echo "tests_rc=$rc"
tail -5 gpurun_out/gpu_tests_r4p.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 800 bash tools/exp.sh cert:MMB_AMM_CERT=0 cert cert:MMB_AMM_CERT=0 cert > gpurun_out/exp_r4p.log 2>&1 || exit 1
cat gpurun_out/exp_r4p.log
python -c "import json;d=json.load(open('gpurun_out/exp/1_cert.json'));print(json.dumps(d['config'].get('amm')))"
