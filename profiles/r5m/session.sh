# r5m: bulk cell reads for preloaded_qsos / catalogue cells (matv73 header templates, run-coalesced
# copies) and the lazily decoded release catalogue: GPU file tests, then configs[2] end to end on files.
set -uo pipefail
bash tools/gpu_run.sh r5m "tests=files" "bench=e2e_n1=--workload e2e --steps 1 --warmup 0 --cpu-budget 0"
