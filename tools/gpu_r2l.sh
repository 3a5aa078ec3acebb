#!/bin/bash
# Round-2 session l: A/B of the fix-up per-line core branch (b_new vs c_fix, c2) and the sc1 Gram
# stores (c_fix vs d_sc1, c5) + parity of the in-tree build (= d_sc1).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_i8.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for round in 1 2; do
  for n in b_new c_fix; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --no-alt --steps 10 --warmup 3 > $O/c2_${n}_$round.json 2>$O/err || exit 1
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'])"
  done
  for n in c_fix d_sc1; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --workload c5 --cpu-budget 0 --steps 5 --warmup 2 > $O/c5_${n}_$round.json 2>$O/err || exit 1
    python3 -c "import json;d=json.load(open('$O/c5_${n}_$round.json'));print('c5 $n $round', round(d['value']/1e6,2), round(d['roofline']['avg_launch_ms'],3), d['checks_ok'])"
  done
done
