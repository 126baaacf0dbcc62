#!/bin/bash
# Round-4 GPU session Q: phase profile of the headline kernel with and without the AMM
# rank-deficiency certificates (-DMMB_PHASE_PROF build).
mkdir -p gpurun_out
BENCH_ARGS="--steps 160 --warmup 80" timeout -k 10 400 bash tools/exp.sh prof:MMB_AMM_CERT=0 prof > gpurun_out/exp_r4q.log 2>&1 || exit 1
cat gpurun_out/exp_r4q.log
for f in gpurun_out/exp/0_prof_MMB_AMM_CERT_0.err gpurun_out/exp/1_prof.err; do echo $f; grep MMB_PROF $f | grep -v " 0$"; done
