# r5k: final tree (B-stationary Gram GEMM, XCD split 4 x 2): whole GPU suite + smoke, bench lines,
# rocprof summary of configs[4].
set -uo pipefail
bash tools/gpu_run.sh r5k tests smoke bench=bench_c2 "bench=bench_c5=--workload c5 --cpu-budget 0" "prof=c5=--workload c5"
