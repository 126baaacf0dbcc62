#!/bin/bash
# A/B of node-IR kernel variants on one box: rats_ir bench lines alternating the env switch given
#   tools/ir_ab.sh VAR VAL_A VAL_B [reps]   (outputs under gpurun_out/ir_ab/)
set -e
mkdir -p gpurun_out/ir_ab
V=$1; A=$2; B=$3; N=${4:-2}
for r in $(seq 1 $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 200 python bench.py --workload rats_ir --no-cpu-baseline \
      > gpurun_out/ir_ab/${V}_${val}_$r.json 2> gpurun_out/ir_ab/${V}_${val}_$r.err
    python -c "import json; d=json.load(open('gpurun_out/ir_ab/${V}_${val}_$r.json')); print('$V=$val', d['value'])"
  done
done
