#!/bin/bash
# Kernel-trace each tools/variants/*.so on a bench workload (args passed through); prints the
# per-kernel average durations.  Run on the GPU box from the repo root.
set -uo pipefail
export TMPDIR=/tmp
for so in tools/variants/*.so; do
  n=$(basename $so .so)
  GPDLA_LIB=$PWD/$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tv_$n -o t --output-format csv -- python3 bench.py --cpu-budget 0 --steps 2 --warmup 1 --no-alt "$@" > gpurun_out/tv_$n.json 2> gpurun_out/tv_$n.err || { echo "FAIL $n"; tail -5 gpurun_out/tv_$n.err; exit 1; }
  echo "== $n"; cut -d, -f1-4 gpurun_out/tv_$n/t_kernel_stats.csv | head -5
done
