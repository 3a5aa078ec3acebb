#!/bin/bash
# prep_kernel blocks per spectrum on the fused layout: a_prep1 (1, r2v), m_prep4 (4), n_prep8 (8).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2w; mkdir -p $O
for n in m_prep4 n_prep8; do
  GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_i8.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$n.log 2>&1 || { echo "tests FAIL $n"; tail -20 $O/tests_$n.log; exit 1; }
  echo "$n $(tail -1 $O/tests_$n.log)"
done
for round in 1 2; do
  for n in a_prep1 m_prep4 n_prep8; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 5 --warmup 2 > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), d['kernel_ms'], d['alternatives']['fused_i8']['kernel_ms'], d['checks_ok'])"
  done
done
echo all-done
