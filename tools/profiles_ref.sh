#!/bin/bash
# Reference Slice+AMWG scheme (SURVEY §8f row 1, §8(d) row 3'): kernel trace + FP64 VALU counter
# pass, summarised into profiles/r3_rats_reference_* (valu_flops.json is what bench.py reads for
# the "valu" roofline of --scheme reference), then the bench line with that roofline.
set -e
OUT=${1:-gpurun_out/prof_ref}
PREFIX=${2:-profiles/r3_rats_reference}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--scheme reference --steps 200 --warmup 200 --no-cpu-baseline"
echo "bench"
timeout -k 10 300 python bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
echo "trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "pmc f64"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq1 -o run -- python3 bench.py $ARGS > $OUT/pmc_sq1.log 2>&1
python3 tools/profiles_pmc_summary.py $OUT $PREFIX --scheme reference
echo "bench with the valu roofline"
timeout -k 10 300 python bench.py --scheme reference > $OUT/bench_final.json 2> $OUT/bench_final.err
cp $OUT/bench_final.json ${PREFIX}_bench.json
