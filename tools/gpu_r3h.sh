#!/bin/bash
# HEAD candidate (outer wing 4/32, inner wing from the shared T_j, NaN repair pass for a lane exactly
# on a line centre): GPU suite + smoke, c2 A/B against fx_tj (no repair pass) x2, then the default
# bench line, the c5 line and the rocprofv3 passes of both workloads (r3c).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3h; mkdir -p $O
V=$PWD/tools/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for round in 1 2; do
  for n in fx_tj new; do
    L=$PWD/gp_dla_detection_amd/libgpdla.so; [ $n = fx_tj ] && L=$V/fx_tj.so
    GPDLA_LIB=$L timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 --warmup 2 --no-alt > $O/c2_${n}_$round.json 2>$O/err || { echo "bench FAIL $n"; tail -5 $O/err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${n}_$round.json'));print('c2 $n $round', round(d['value']/1e6,2), round(d['kernel_ms']['likelihood'],2), d['checks_ok'])"
  done
done
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -5 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 600 python bench.py --workload c5 --cpu-budget 0 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 900 bash tools/profile.sh r3c > $O/prof_c2.log 2>&1 || { echo prof c2 failed; tail -5 $O/prof_c2.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh r3c_c5 --workload c5 > $O/prof_c5.log 2>&1 || { echo prof c5 failed; tail -5 $O/prof_c5.log; exit 1; }
echo all-done
