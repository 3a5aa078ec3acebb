set -uo pipefail
mkdir -p gpurun_out/r5a
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probe_rcp > gpurun_out/r5a/probe_rcp.txt 2>&1 && cat gpurun_out/r5a/probe_rcp.txt && \
bash tools/gpu_run.sh r5a "ab=2=base,x_nobar,x_nofix,x_noepi,x_rcp4" lib=tools/variants/x_rcp4.so testfile=tests/test_gpu_parity.py testfile=tests/test_gpu_line_centres.py lib=head && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r5a/tcc -o tcc --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-budget 0 --no-alt > gpurun_out/r5a/tcc_bench.json 2>gpurun_out/r5a/tcc.err && echo tcc-done
