#!/bin/bash
# Round-2 session l: fix-up per-line core branch A/B (b_new vs c_fix) + parity of the in-tree build.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
bash tools/ab_variants.sh --steps 10 --warmup 3 || exit 1
