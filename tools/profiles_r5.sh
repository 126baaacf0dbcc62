#!/bin/bash
# Round-5 final-build profiles (run via gpurun from the repo root; every GPU step under its own
# time limit, the chain stops at the first failure).  Part A: the headline's trace + PMC passes
# (tools/profiles_run.sh) and the reference scheme's.  Part B: the phase profile of the same
# sources (mamba.jl_amd/lib/exp_phase.so, -DMMB_PHASE_PROF) and kernel traces of the other
# workloads.   tools/profiles_r5.sh A|B [OUT]
set -e
PART=${1:-A}
OUT=${2:-gpurun_out/r5prof}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$PART" = A ]; then
  echo "headline"
  tools/profiles_run.sh $OUT/rats
  echo "reference scheme"
  BENCH_EXTRA="--scheme reference" tools/profiles_run.sh $OUT/ref
else
  echo "phase profile"
  MMB_LIB=mamba.jl_amd/lib/exp_phase.so timeout -k 10 300 python bench.py --steps 200 --warmup 100 --no-cpu-baseline \
    > $OUT/phase.json 2> $OUT/phase.err
  for w in logistic line_amm seeds_ir rats_ir; do
    echo "trace $w"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$w -o run -- \
      python3 bench.py --workload $w --no-cpu-baseline > $OUT/trace_$w.json 2> $OUT/trace_$w.err
  done
fi
