mkdir -p gpurun_out/r15d && export TMPDIR=/tmp
for v in base os1 os2 os4 os8 os16 os31; do
  if [ "$v" = base ]; then L=gp_dla_detection_amd/libgpdla.so; else L=tools/variants/$v.so; fi
  GPDLA_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r15d/$v -o obj -- python tools/bench_objective.py 5000 1217 20 > gpurun_out/r15d/$v.json 2>gpurun_out/r15d/$v.err || exit 1
done
