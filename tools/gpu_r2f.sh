set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2f; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_baseline_configs.py::test_config4_panel_gemm_i8_k50_100k tests/test_gpu_i8.py tests/test_gpu_panel_gemm.py > $O/t.log 2>&1; r=$?; tail -3 $O/t.log; grep "vs fp64" $O/t.log | head -20
[ $r -eq 0 ] || exit 1
bash tools/ab_variants.sh --workload c5 --path panel_gemm_i8_24 && bash tools/trace_variants.sh --workload c5 --spectra 16 --path panel_gemm_i8_24
