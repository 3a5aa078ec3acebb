#!/bin/bash
# GEMM A/B on configs[4]: a_base (4 waves x 32 samples, 168 VGPRs, 3 waves/SIMD) vs k_rt1 (8 waves x
# 16 samples per 128 x 64 tile, 98 VGPRs, 4 waves/SIMD).  Panel-path GPU tests on every variant first.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2u; mkdir -p $O
for n in a_base k_rt1; do
  GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_panel_gemm.py tests/test_gpu_i8.py tests/test_gpu_baseline_configs.py -k "not config2" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$n.log 2>&1 || { echo "tests FAIL $n"; tail -20 $O/tests_$n.log; exit 1; }
  echo "$n $(tail -1 $O/tests_$n.log)"
done
for round in 1 2; do
  for n in a_base k_rt1; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 --steps 5 --warmup 2 --no-alt > $O/c5_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5_${n}_$round.json'));print('c5 $n $round', round(d['value']/1e6,2), round(d['roofline']['avg_launch_ms'],3), d['checks_ok'])"
  done
done
for n in a_base k_rt1; do
  GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$n -o trace --output-format csv -- python3 bench.py --workload c5 --cpu-budget 0 --steps 2 --warmup 1 --no-alt > $O/trace_$n.json 2>/dev/null || { echo "trace FAIL $n"; exit 1; }
  echo "$n: $(grep -i 'weights_i8\|gemm_i8_kernel' $O/trace_$n/trace_kernel_stats.csv | cut -d, -f1-5)"
done
echo all-done
