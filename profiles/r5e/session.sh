# r5e: head with prep's exact unit scaling (fixes prod-d under/overflow for noise far from 1): whole GPU
# suite + smoke, bench lines, rocprof summaries of c2; GEMM store-policy / XCD-split and weights-kernel
# exp-table A/B on c5.
set -uo pipefail
bash tools/gpu_run.sh r5e tests smoke bench=bench_c2 "bench=bench_c5=--workload c5 --cpu-budget 0" \
  "ab=2=head,g_ntg,g_ex4,g_ex1,w128=--workload c5" "ab=2=head,f128=--path fused_i8" "prof=c2" || exit $?
for v in g_ntg g_ex4; do
  GPDLA_LIB=$PWD/tools/variants/$v.so timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r5e/tcc_$v -o tcc --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-budget 0 --no-alt > gpurun_out/r5e/tcc_$v.json 2>gpurun_out/r5e/tcc_$v.err || exit $?
done
echo tcc-done
timeout -k 10 120 rocprofv3 -L > gpurun_out/r5e/avail.txt 2>&1 || true
