#!/bin/bash
# Round-2 session o: session-start check of HEAD in a fresh container (rebuilt .so):
# GPU suite + smoke, the default bench line (with the CPU baseline), kernel trace of c2 and c5.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -5 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 600 python bench.py --workload c5 --cpu-budget 0 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail -5 $O/bench_c5.err; exit 1; }
tail -c 400 $O/bench_c5.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --no-alt > $O/trace_c2.json 2> $O/trace_c2.err || { echo trace failed; exit 1; }

timeout -k 10 900 bash tools/profile_stalls.sh c5 --workload c5 --no-alt > $O/stall_c5.log 2>&1 || { echo stall failed; tail -5 $O/stall_c5.log; exit 1; }
echo all-done
