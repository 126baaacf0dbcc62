#!/bin/bash
# Round-4 GPU session X: per-chain LDS stride padding (MMB_RATS_LDS_PAD doubles: shifts the
# second chain of a wavefront by that many banks pairs) on the rats headline.
mkdir -p gpurun_out
timeout -k 10 900 bash tools/exp.sh pad0 pad4 pad8 pad16 pad0 pad4 pad8 pad16 > gpurun_out/exp_r4x.log 2>&1 || exit 1
cat gpurun_out/exp_r4x.log
