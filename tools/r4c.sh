#!/bin/bash
# Round-4 GPU session C: profiles of the HEAD build -- rats Gibbs+AMM (trace, HBM bytes, SQ
# counters), its phase split (MMB_PHASE_PROF build), the f1 reference scheme, line AMM.
set -e
mkdir -p gpurun_out
bash tools/profiles_run.sh gpurun_out/prof_r4c > gpurun_out/prof_r4c.log 2>&1
echo "rats profiles done"
MMB_LIB=mamba.jl_amd/lib/exp_phase.so timeout -k 10 200 python bench.py --steps 200 --warmup 100 --no-cpu-baseline \
  > gpurun_out/r4c_phase.json 2> gpurun_out/r4c_phase.err
echo "phase done"
BENCH_EXTRA="--scheme reference" bash tools/profiles_run.sh gpurun_out/prof_r4c_ref > gpurun_out/prof_r4c_ref.log 2>&1
echo "f1 profiles done"
timeout -k 10 200 python bench.py --workload line_amm > gpurun_out/r4c_line_amm.json 2> gpurun_out/r4c_line_amm.err
echo "line done"
