#!/bin/bash
# Round-2 session i: GPU suite (zero-padded ranks, wide Gram GEMM cross-check), c2 bench, c5 wide vs narrow.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "gpu tests rc=$rc"; exit $rc; fi
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-alt > $O/c2.json 2> $O/c2.err || exit 1
tail -c 700 $O/c2.json | head -c 400; echo
for w in 1 0 1 0; do
  GPDLA_GEMM_WIDE=$w timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --cpu-budget 0 > $O/c5_w$w.json 2> $O/c5_w$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c5_w$w.json'));print('wide=$w', d['value'], d['roofline']['avg_launch_ms'], d['kernel_ms'])"
done
