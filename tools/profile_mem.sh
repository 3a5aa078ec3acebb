#!/bin/bash
# Memory-path counter passes (TLB, L2 hit/miss, TCP->TCC read latency) for a bench workload, run on
# the GPU box from the repo root; each pass its own run.  Output: gpurun_out/mem_<tag>/{a,b}/*.csv
set -uo pipefail
TAG=${1:-cur}; shift || true
OUT=$PWD/gpurun_out/mem_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --no-alt $*"
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d "$OUT/a" -o a --output-format csv -- python3 bench.py $ARGS > "$OUT/a.json" || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d "$OUT/b" -o b --output-format csv -- python3 bench.py $ARGS > "$OUT/b.json" || exit 1
echo mem-profile-done
