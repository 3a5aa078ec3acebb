#!/bin/bash
# Round-2 final tree: GPU suite + smoke, the default bench line, the c5 line and the rocprofv3 passes
# (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ mix) of both workloads.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
V=$PWD/tools/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -5 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 600 python bench.py --workload c5 --cpu-budget 0 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 900 bash tools/profile.sh r3i > $O/prof_c2.log 2>&1 || { echo prof c2 failed; tail -5 $O/prof_c2.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh r3i_c5 --workload c5 > $O/prof_c5.log 2>&1 || { echo prof c5 failed; tail -5 $O/prof_c5.log; exit 1; }
echo all-done
