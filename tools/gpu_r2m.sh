#!/bin/bash
# Round-2 session m: full GPU suite + smoke on the current tree, then e2e with the compute split.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py --workload e2e > $O/e2e.json 2> $O/e2e.err || { echo e2e failed; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));print(d['e2e'])"
