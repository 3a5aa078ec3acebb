#!/bin/bash
# Round-2 session k: sweep-restructure A/B (tools/variants a_old / b_new), parity tests of the new
# kernel, stall counters of the headline kernel, then configs[2] end to end on files.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
bash tools/ab_variants.sh --steps 10 --warmup 3 || exit 1
bash tools/profile_stalls.sh r2k || exit 1
timeout -k 10 900 python bench.py --workload e2e > $O/e2e.json 2> $O/e2e.err || { echo e2e failed; tail -5 $O/e2e.err; exit 1; }
cat $O/e2e.json
