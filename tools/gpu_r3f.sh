#!/bin/bash
# Outer wing degree 4 beyond |x| = 32, far-wing tables and the fused_i8 far branch removed:
# full GPU suite + smoke, then bench A/B against the previous commit's library (o6x14):
# c2 (with the fused_i8 alternative) x2, c5 x1.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f; mkdir -p $O
V=$PWD/tools/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for round in 1 2; do
  for n in o6x14 new; do
    L=$PWD/gp_dla_detection_amd/libgpdla.so; [ $n = o6x14 ] && L=$V/o6x14.so
    GPDLA_LIB=$L timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'], d.get('alternatives'))"
  done
done
for n in o6x14 new; do
  L=$PWD/gp_dla_detection_amd/libgpdla.so; [ $n = o6x14 ] && L=$V/o6x14.so
  GPDLA_LIB=$L timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 > $O/c5_${n}.json 2>$O/err || { echo "c5 FAIL $n"; tail -5 $O/err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_${n}.json'));print('c5 $n', round(d['value']/1e6,2))"
done
echo all-done
