#!/bin/bash
# Outer wing degree/threshold A/B: o6x14 (HEAD), o5x20, o4x32.  Fused-path GPU tests per variant,
# then c2 bench x3 rounds and c5 once.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e; mkdir -p $O
V=$PWD/tools/variants
for n in o5x20 o4x32; do
  GPDLA_LIB=$V/$n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_i8.py tests/test_gpu_panel_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; exit 1; }
  echo "$n $(tail -1 $O/tests_$n.log)"
done
for round in 1 2 3; do
  for n in o6x14 o5x20 o4x32; do
    GPDLA_LIB=$V/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 --no-alt > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'])"
  done
done
for n in o6x14 o5x20 o4x32; do
  GPDLA_LIB=$V/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 > $O/c5_${n}.json 2>$O/err || { echo "c5 FAIL $n"; tail -5 $O/err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_${n}.json'));print('c5 $n', round(d['value']/1e6,2))"
done
echo all-done
