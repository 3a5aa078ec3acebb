set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-r2c}
for v in ${VARIANTS:-ldl_mfma1 ldl_mfma0}; do
  GPDLA_LIB=$PWD/tools/variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r2c}/$v -o t --output-format csv -- python3 bench.py --workload c5 --no-alt --cpu-budget 0 --steps 2 --warmup 1 > gpurun_out/${TAG:-r2c}/$v.json 2> gpurun_out/${TAG:-r2c}/$v.err || exit 1
done
echo done
