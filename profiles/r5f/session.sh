# r5f: final tree of the session -- whole GPU suite + smoke, bench lines (c2, c5 int8-24, c5 fp64),
# rocprof summaries of c5 (int8-24 and fp64 panel paths).
set -uo pipefail
bash tools/gpu_run.sh r5f tests smoke bench=bench_c2 "bench=bench_c5=--workload c5 --cpu-budget 0" \
  "bench=bench_c5f64=--workload c5 --path panel_gemm --cpu-budget 0 --no-alt" "prof=c5=--workload c5" \
  "prof=c5f64=--workload c5 --path panel_gemm"
