#!/bin/bash
# Round-4 GPU session Y: final build -- GPU test suite, smoke, and the rocprofv3 trace + PMC
# passes of the headline (gibbs_amm) and reference-scheme workloads (tools/profiles_run.sh).
mkdir -p gpurun_out/final
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?
echo "tests_rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/final/smoke.log
timeout -k 10 1000 bash tools/profiles_run.sh gpurun_out/prof_final || exit 1
echo headline_profiles_done
BENCH_EXTRA="--scheme reference" timeout -k 10 1000 bash tools/profiles_run.sh gpurun_out/prof_ref_final || exit 1
echo reference_profiles_done
