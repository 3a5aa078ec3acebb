#!/bin/bash
# VALU instruction-mix and co-issue counters for the bench workload (GPU box, repo root).
set -uo pipefail
TAG=${1:-cur}
OUT=$PWD/gpurun_out/mix_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0"
i=0
for set in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_F64 SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.json" || exit 1
done
echo mix-profile-done
