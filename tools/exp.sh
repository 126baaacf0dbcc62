#!/bin/bash
# Timing experiments: run bench.py against each variant given as an argument, NAME[:VAR=VAL[,VAR=VAL]]
# (library mamba.jl_amd/lib/exp_NAME.so, optional environment); one JSON line per variant into
# gpurun_out/exp/<tag>.json.  BENCH_ARGS overrides the bench arguments (default: rats, 200 timed
# steps after 100 warm-up).
set -e
mkdir -p gpurun_out/exp
ARGS=${BENCH_ARGS:-"--steps 200 --warmup 100"}
i=0
for spec in "$@"; do
  n=${spec%%:*}
  envs=""
  [[ "$spec" == *:* ]] && envs=${spec#*:}
  tag="${i}_${n}${envs:+_${envs//[=,]/_}}"
  i=$((i+1))
  echo "running $tag"
  env ${envs//,/ } MMB_LIB=mamba.jl_amd/lib/exp_$n.so timeout -k 10 150 python bench.py --no-cpu-baseline $ARGS \
    > gpurun_out/exp/$tag.json 2> gpurun_out/exp/$tag.err
  python -c "import json;d=json.load(open('gpurun_out/exp/$tag.json'));print('$tag', '%.4g'%d['value'], round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
