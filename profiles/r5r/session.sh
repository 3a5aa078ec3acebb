# r5r: final tree: whole GPU suite + smoke, the driver's default bench line (configs[1], CPU baseline
# included), configs[4], and configs[2] end to end on files.
set -uo pipefail
bash tools/gpu_run.sh r5r tests smoke bench=bench_c2 "bench=bench_c5=--workload c5 --cpu-budget 0" \
  "bench=e2e_n1=--workload e2e --steps 1 --warmup 0 --cpu-budget 0"
