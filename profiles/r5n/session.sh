# r5n: host-buffer pipeline in gpdla_engine_process (two device stages; inputs in and results out on
# a copy stream beside the kernels): whole GPU suite + smoke, configs[2] end to end, configs[1] bench.
set -uo pipefail
bash tools/gpu_run.sh r5n tests smoke "bench=e2e_n1=--workload e2e --steps 1 --warmup 0 --cpu-budget 0" \
  "bench=bench_c2=--cpu-budget 0 --no-alt"
