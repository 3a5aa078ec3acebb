# r5s: rocprofv3 summary of configs[1] on the final tree (kernel trace + stats, FETCH_SIZE, WRITE_SIZE,
# SQ instruction mix), for bench.py's roofline.traffic.
set -uo pipefail
bash tools/gpu_run.sh r5s prof=c2
