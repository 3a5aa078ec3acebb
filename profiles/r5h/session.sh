# r5h: final-tree rehearsals -- the multi-rank bench path with 8 ranks sharing the leased GPU
# (configs[1] per rank), and configs[2] end to end on files on one GPU.
set -uo pipefail
bash tools/gpu_run.sh r5h "dist=8=c2_n8_shared_gpu=--steps 3 --warmup 1 --cpu-budget 0 --no-alt" \
  "bench=e2e_n1=--workload e2e --steps 1 --warmup 0 --cpu-budget 0"
