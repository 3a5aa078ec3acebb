#!/bin/bash
# Stall/issue counter passes for the likelihood kernel (run on the GPU box from the repo root).
# Output: gpurun_out/stall_<tag>/{a,b,c}/*.csv  (+ the available-counter list)
set -uo pipefail
TAG=${1:-cur}; shift || true
OUT=$PWD/gpurun_out/stall_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0 $*"
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d "$OUT/a" -o a --output-format csv -- python3 bench.py $ARGS > "$OUT/a.json" || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/b" -o b --output-format csv -- python3 bench.py $ARGS > "$OUT/b.json" || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d "$OUT/c" -o c --output-format csv -- python3 bench.py $ARGS > "$OUT/c.json" || exit 1
echo stall-profile-done
