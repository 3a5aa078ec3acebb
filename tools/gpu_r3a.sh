#!/bin/bash
# Fused fp64 kernel: per-line wave-uniform far-wing branch (degree-4 far polynomial, no core test)
# for chunks where every lane is >= kFarX from the line centre.  Fused-path GPU tests on q_far, then
# the default bench line A/B against HEAD (a_base), 3 rounds.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a; mkdir -p $O
GPDLA_LIB=$PWD/tools/variants/q_far.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py tests/test_gpu_pipeline.py tests/test_gpu_files.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2 3; do
  for n in a_base q_far; do
    GPDLA_LIB=$PWD/tools/variants/$n.so timeout -k 10 300 python bench.py --cpu-budget 0 --steps 5 --warmup 2 --no-alt > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), d['kernel_ms'], d['checks_ok'])"
  done
done
echo all-done
