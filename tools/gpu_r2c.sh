set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2c; mkdir -p $O
timeout -k 10 300 python bench.py --workload c5 --path panel_gemm_i8_24 --cpu-budget 0 --steps 3 --warmup 1 > $O/c5_24.json 2> $O/c5_24.err || { echo fail24; tail -20 $O/c5_24.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --path panel_gemm_i8 --cpu-budget 0 --steps 3 --warmup 1 > $O/c5_32.json 2> $O/c5_32.err || { echo fail32; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace24 -o t --output-format csv -- python3 bench.py --workload c5 --spectra 16 --path panel_gemm_i8_24 --cpu-budget 0 --steps 2 --warmup 1 > $O/tr24.json 2>/dev/null || exit 1
python - <<'PY'
import json
for f in ("c5_24","c5_32"):
    d=json.loads(open(f"gpurun_out/r2c/{f}.json").read().strip().splitlines()[-1])
    print(f, "%.4g"%d["value"], d["ms_per_step"], d["checks_ok"])
PY
