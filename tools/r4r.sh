#!/bin/bash
# Round-4 GPU session R: certificates with the certificate vector prefetched -- A/B against
# MMB_AMM_CERT=0, and the phase profile of both.
mkdir -p gpurun_out
timeout -k 10 800 bash tools/exp.sh cert:MMB_AMM_CERT=0 cert cert:MMB_AMM_CERT=0 cert > gpurun_out/exp_r4r.log 2>&1 || exit 1
cat gpurun_out/exp_r4r.log
BENCH_ARGS="--steps 160 --warmup 80" timeout -k 10 400 bash tools/exp.sh prof:MMB_AMM_CERT=0 prof > gpurun_out/exp_r4r2.log 2>&1 || exit 1
for f in gpurun_out/exp/0_prof_MMB_AMM_CERT_0.err gpurun_out/exp/1_prof.err; do echo $f; grep MMB_PROF $f | grep -v " 0$"; done
