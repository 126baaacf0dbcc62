#!/bin/bash
# Round-4 GPU session U: carried proposal loaded with the tune words (default) vs after the
# flag / tag compare (MMB_EXP_CARRY_DEP), rats headline.
mkdir -p gpurun_out
timeout -k 10 800 bash tools/exp.sh dep pre dep pre dep pre > gpurun_out/exp_r4u.log 2>&1 || exit 1
cat gpurun_out/exp_r4u.log
