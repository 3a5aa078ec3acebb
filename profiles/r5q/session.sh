# r5q: ldl_mfma_kernel<13, float> (configs[4]'s LDL^T) at 3 waves per SIMD (168 VGPRs, spilling) with
# all rows or 2 rows of Gram tiles loaded ahead, and at 2 waves with 3 rows ahead: configs[4] A/B.
set -uo pipefail
bash tools/gpu_run.sh r5q "ab=2=head,ldl_w3a2,ldl_w3a64,ldl_w2a3=--workload c5"
