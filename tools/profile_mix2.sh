#!/bin/bash
# Instruction-class and pipe-busy counters for a likelihood path (run on the GPU box from the repo root).
# Usage: tools/profile_mix2.sh <tag> [bench args]; output gpurun_out/mix_<tag>/{m1,m2}/*.csv
set -uo pipefail
TAG=${1:-cur}; shift || true
OUT=$PWD/gpurun_out/mix_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --cpu-budget 0 --no-alt $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 -d "$OUT/m1" -o m1 --output-format csv -- python3 bench.py $ARGS > "$OUT/m1.json" || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES -d "$OUT/m2" -o m2 --output-format csv -- python3 bench.py $ARGS > "$OUT/m2.json" || exit 1
echo mix-done
