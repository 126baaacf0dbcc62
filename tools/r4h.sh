#!/bin/bash
# Round-4 GPU session H: DPP accumulator hazard probe; if the hardware shows no accumulator
# hazard, A/B the blocked asm dot product (MMB_EXP_DOTBLK) against the default and run the rats
# parity tests on that variant.
mkdir -p gpurun_out
( cd tools/probes && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 dpp_acc_hazard.hip -o /tmp/dpp_acc_hazard 2>/dev/null )
timeout -k 10 60 /tmp/dpp_acc_hazard > gpurun_out/dpp_acc_hazard.json 2>&1
rc=$?
cat gpurun_out/dpp_acc_hazard.json
echo "probe_rc=$rc"
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 env MMB_LIB=mamba.jl_amd/lib/exp_dotblk.so python -u -m pytest tests/test_gpu_parity.py -q -k rats --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4h_dotblk.log 2>&1
echo "tests_rc=$?"
tail -3 gpurun_out/gpu_tests_r4h_dotblk.log
timeout -k 10 800 bash tools/exp.sh base dotblk base dotblk base:MMB_ITERS_PER_LAUNCH=16 dotblk:MMB_ITERS_PER_LAUNCH=16 > gpurun_out/exp_r4h.log 2>&1 || exit 1
cat gpurun_out/exp_r4h.log
