#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1) kernel trace + stats   2) FETCH_SIZE   3) WRITE_SIZE   4) SQ instruction mix
# Output: gpurun_out/prof_<tag>/...
set -euo pipefail
TAG=${1:-r1}
shift || true
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-budget 0 --no-alt $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_fetch.json"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_write.json"
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq" -o sq --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_sq.json"
echo profile-done
