#!/bin/bash
# Fused fp64 wave priority A/B: head, prio_mfma (s_setprio 1 around a chunk's MFMAs), prio_valu
# (s_setprio 1 around its profile + weight VALU phase).  Parity subset on both, c2 x3.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3l; mkdir -p $O
V=$PWD/tools/variants
for n in prio_mfma prio_valu; do
  GPDLA_LIB=$V/$n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; exit 1; }
  echo "$n $(tail -1 $O/tests_$n.log)"
done
for round in 1 2 3; do
  for n in head prio_mfma prio_valu; do
    GPDLA_LIB=$V/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 --no-alt > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'])"
  done
done
echo all-done
