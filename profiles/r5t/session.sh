# r5t: the driver's default bench line on the final tree (reads profiles/r5s_c2_summary.json).
set -uo pipefail
bash tools/gpu_run.sh r5t bench=bench_c2
