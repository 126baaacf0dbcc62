#!/bin/bash
# Round-4 GPU session J: phase profile of the reference scheme (AMWG / slice / iteration
# cycles, -DMMB_PHASE_PROF build), then the headline profiles (gibbs_amm) of the current build.
mkdir -p gpurun_out
BENCH_ARGS="--scheme reference --steps 100 --warmup 50" timeout -k 10 300 bash tools/exp.sh prof > gpurun_out/exp_r4j.log 2>&1 || exit 1
grep MMB_PROF gpurun_out/exp/0_prof.err
timeout -k 10 1000 bash tools/profiles_run.sh gpurun_out/prof_r4j || exit 1
echo profiles_done
