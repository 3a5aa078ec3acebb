# r5d: the folded headline kernel (window ring, batched reciprocals, 128-entry exp, 6-deep B reads):
# whole GPU suite + smoke, bench lines, rocprof summaries of c2; GEMM store-policy / XCD-split A/B on c5.
set -uo pipefail
bash tools/gpu_run.sh r5d tests smoke bench=bench_c2 "bench=bench_c5=--workload c5 --cpu-budget 0" \
  "ab=2=head,g_ntg,g_ex4,g_ex1=--workload c5" "prof=c2" || exit $?
for v in g_ntg g_ex4; do
  GPDLA_LIB=$PWD/tools/variants/$v.so timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r5d/tcc_$v -o tcc --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-budget 0 --no-alt > gpurun_out/r5d/tcc_$v.json 2>gpurun_out/r5d/tcc_$v.err || exit $?
done
echo tcc-done
timeout -k 10 120 rocprofv3 -L > gpurun_out/r5d/avail.txt 2>&1 || true
