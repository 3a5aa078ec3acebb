# r5i: B-stationary int8 Gram GEMM (gemm_i8_bst_kernel, 12 waves; bst8 = 8 waves; nobst = the
# previous gemm_i8_kernel<3>): bitwise check against nobst on every path, the panel / int8 GPU tests,
# configs[4] A/B and L2 counters.
set -uo pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 300 python tools/bitwise_ab.py run $O/head.npz > $O/bw_head.log 2>&1 || exit 1
GPDLA_LIB=$PWD/tools/variants/nobst.so timeout -k 10 300 python tools/bitwise_ab.py run $O/nobst.npz > $O/bw_nobst.log 2>&1 || exit 1
python tools/bitwise_ab.py compare $O/head.npz $O/nobst.npz | tee $O/bitwise.txt
bash tools/gpu_run.sh r5i "tests=panel or i8 or config4 or extremes or line_centres" \
  "ab=2=head,nobst,bst8=--workload c5" || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/tcc -o tcc --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-budget 0 --no-alt > $O/tcc.json 2>$O/tcc.err && echo tcc-done
