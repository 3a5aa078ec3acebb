# r5p: weights_i8_kernel at 5 and 6 waves per SIMD (GPDLA_WI8_OCC; head = 4, 128 VGPRs): configs[4]
# A/B, interleaved.
set -uo pipefail
bash tools/gpu_run.sh r5p "ab=3=head,wi8_o5,wi8_o6=--workload c5"
