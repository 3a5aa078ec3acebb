#!/bin/bash
# Outer damping-wing polynomial (degree 6 beyond |x| = 14, fix-up below) in the batched sweeps:
# full GPU suite on the new tree, then bench A/B against HEAD's library (a_base): c2 (with the
# int8 fused alternative) x3, c5 x2.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for round in 1 2 3; do
  for n in a_base new; do
    L=$PWD/gp_dla_detection_amd/libgpdla.so; [ $n = a_base ] && L=$PWD/tools/variants/a_base.so
    GPDLA_LIB=$L timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), [ (a.get('path'), round(a['value']/1e6,2)) for a in d.get('alternatives',[])])"
  done
done
for round in 1 2; do
  for n in a_base new; do
    L=$PWD/gp_dla_detection_amd/libgpdla.so; [ $n = a_base ] && L=$PWD/tools/variants/a_base.so
    GPDLA_LIB=$L timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 > $O/c5_${n}_$round.json 2>$O/err || { echo "c5 FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5_${n}_$round.json'));print('c5 $n $round', round(d['value']/1e6,2), d['kernel_ms'])"
  done
done
echo all-done
