#!/bin/bash
# usage: tools_mp.sh NPROC CHAINS STEPS -> NPROC simultaneous tools/mp.py processes on the GPU
N=$1; K=$2; S=$3
T=$(python -c "import time;print(time.time()+25)")
pids=()
for i in $(seq 1 $N); do timeout -k 10 120 python tools/mp.py $K $S $T 2>/dev/null & pids+=($!); done
rc=0; for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
