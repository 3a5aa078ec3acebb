#!/bin/bash
# Fused fix-up A/B: head vs fx_incr (lanes with no line core: replace only the lines with
# |x| < kOuterX, outer -> inner wing, instead of recomputing all three lines).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3j; mkdir -p $O
V=$PWD/tools/variants
GPDLA_LIB=$V/fx_incr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_fx_incr.log 2>&1 || { tail -30 $O/tests_fx_incr.log; exit 1; }
echo "fx_incr $(tail -1 $O/tests_fx_incr.log)"
for round in 1 2 3; do
  for n in head fx_incr; do
    GPDLA_LIB=$V/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 --no-alt > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'])"
  done
done
echo all-done
