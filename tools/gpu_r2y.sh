#!/bin/bash
# prep_kernel pass 3a: the slot scalars (mu, log omega interpolation, pow / exp) one thread per slot
# instead of lane 0 of each slot-wave.  Full GPU suite on the in-tree build (= o_prep3a), then A/B.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for round in 1 2; do
  for n in a_base o_prep3a; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 5 --warmup 2 > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), d['kernel_ms'], d['alternatives']['fused_i8']['kernel_ms'], d['checks_ok'])"
  done
done
for n in a_base o_prep3a; do
  GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 --steps 3 --warmup 1 > $O/c5_${n}.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_${n}.json'));print('c5 $n', round(d['value']/1e6,2), d['kernel_ms'], d['checks_ok'])"
done
echo all-done
