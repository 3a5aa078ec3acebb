#!/bin/bash
# configs[4] chain counters (run on the GPU box from the repo root), one stream so the kernels do not overlap:
#   a) L1 -> L2 read requests, sectors, hit/miss and request latency (the Gram GEMM's "A digits from L2" bound)
#   b) the texture path's stall cycles (L1 / TA / TD) and L2 busy
#   c) VALU instruction mix (the weights kernel's issue floor: f64 FMA / MUL / ADD, transcendentals, int, cvt)
#   d) VMEM issue and SQ instruction levels (memory parallelism of the LDL^T)
# Each pass is its own run.  Output: gpurun_out/l2_<tag>/{a,b,c,d}/*.csv
set -uo pipefail
TAG=${1:-cur}; shift || true
OUT=$PWD/gpurun_out/l2_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--workload c5 --steps 2 --warmup 1 --cpu-budget 0 --no-alt --panel-streams 1 $*"
timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_READ_SECTORS_sum TCC_REQ_sum GRBM_GUI_ACTIVE -d "$OUT/a" -o a --output-format csv -- python3 bench.py $ARGS > "$OUT/a.json" || exit 1
echo pass-a-done
timeout -s KILL 240 rocprofv3 --pmc TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_BUSY_avr TCC_TAG_STALL_sum GRBM_GUI_ACTIVE -d "$OUT/b" -o b --output-format csv -- python3 bench.py $ARGS > "$OUT/b.json" || exit 1
echo pass-b-done
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/c" -o c --output-format csv -- python3 bench.py $ARGS > "$OUT/c.json" || exit 1
echo pass-c-done
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/d" -o d --output-format csv -- python3 bench.py $ARGS > "$OUT/d.json" || exit 1
echo l2-profile-done
