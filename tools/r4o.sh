#!/bin/bash
# Round-4 GPU session O: reference-scheme profiles of the current build (trace + PMC passes,
# the VALU-flop file bench.py prices the f1 line with) and its phase profile.
mkdir -p gpurun_out
BENCH_ARGS="--scheme reference --steps 100 --warmup 50" timeout -k 10 300 bash tools/exp.sh prof > gpurun_out/exp_r4o.log 2>&1 || exit 1
grep -E "amwg|slice|iteration" gpurun_out/exp/0_prof.err
BENCH_EXTRA="--scheme reference" timeout -k 10 1000 bash tools/profiles_run.sh gpurun_out/prof_ref_r4o || exit 1
echo profiles_done
