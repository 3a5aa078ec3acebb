# r5o: configs[2] end to end with 8 ranks sharing the leased GPU (torch.distributed.run started before
# any GPU call), after the bulk cell reads and the host-buffer pipeline.
set -uo pipefail
bash tools/gpu_run.sh r5o "dist=8=e2e_n8_shared_gpu=--workload e2e --steps 1 --warmup 0 --cpu-budget 0"
