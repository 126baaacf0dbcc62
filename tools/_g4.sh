set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/gridsync_probe.bin
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --output-format csv -d gpurun_out/pmc2 -o run -- python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1
ls gpurun_out/pmc2
