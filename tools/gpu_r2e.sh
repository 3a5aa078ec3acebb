set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_baseline_configs.py::test_config4_panel_gemm_i8_k50_100k "tests/test_gpu_panel_gemm.py::test_high_rank_ldl_buckets_match_oracle" tests/test_gpu_i8.py > $O/t.log 2>&1; r=$?; tail -3 $O/t.log; grep "vs fp64" $O/t.log
[ $r -le 1 ] || exit $r
timeout -k 10 300 python bench.py --workload c5 --path panel_gemm_i8_24 --cpu-budget 0 --steps 3 --warmup 1 > $O/c5_24.json 2> $O/c5_24.err || exit 1
python -c "import json; d=json.loads(open('$O/c5_24.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
