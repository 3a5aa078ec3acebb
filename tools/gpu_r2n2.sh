#!/bin/bash
# weights_i8 batched-wing A/B on c5 (e_base vs f_wts) + i8 GPU tests of the in-tree build (= f_wts).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2n2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_baseline_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for n in e_base f_wts; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 --steps 5 --warmup 2 > $O/c5_${n}_$round.json 2>$O/err || exit 1
    python3 -c "import json;d=json.load(open('$O/c5_${n}_$round.json'));print('c5 $n $round', round(d['value']/1e6,2), round(d['roofline']['avg_launch_ms'],3), d['checks_ok'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --workload c5 --cpu-budget 0 --steps 2 --warmup 1 > $O/trace.json 2>/dev/null || exit 1
grep -i "weights_i8\|ldl_mfma\|gemm_i8" $O/trace/trace_kernel_stats.csv | cut -d, -f1-5
