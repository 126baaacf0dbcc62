#!/bin/bash
# Round-4 GPU session L: PMC passes of the logistic kernels (tools/profiles_lg.sh), per-kernel
# summaries of the last 400 launches.
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/profiles_lg.sh gpurun_out/pmc_lg_r4l || exit 1
python3 tools/pmc_quick_summary.py gpurun_out/pmc_lg_r4l lg_grad 400 > gpurun_out/pmc_lg_r4l/grad.json
python3 tools/pmc_quick_summary.py gpurun_out/pmc_lg_r4l lg_ctl 400 > gpurun_out/pmc_lg_r4l/ctl.json
cat gpurun_out/pmc_lg_r4l/grad.json gpurun_out/pmc_lg_r4l/ctl.json
