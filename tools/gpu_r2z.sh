#!/bin/bash
# configs[4] per-batch kernels: prep_kernel<0> Khatri-Rao rows from an (r, c) table in tile-major
# order (coalesced), convert_gemm_i8 over 512 threads (2 halves of each segment).  Full GPU suite on
# the in-tree build (= p_c5prep), then A/B against the previous commit, with kernel traces.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for round in 1 2; do
  for n in a_base p_c5prep; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 --steps 5 --warmup 2 > $O/c5_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5_${n}_$round.json'));print('c5 $n $round', round(d['value']/1e6,2), d['kernel_ms'], d['checks_ok'])"
  done
done
for n in a_base p_c5prep; do
  GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$n -o trace --output-format csv -- python3 bench.py --workload c5 --cpu-budget 0 --steps 2 --warmup 1 --no-alt > $O/trace_$n.json 2>/dev/null || { echo "trace FAIL $n"; exit 1; }
  echo "$n: $(grep -i 'prep_kernel\|convert_gemm' $O/trace_$n/trace_kernel_stats.csv | cut -d, -f1-4)"
done
echo all-done
