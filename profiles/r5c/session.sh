# r5c: headline A/B -- base (HEAD~) vs u5+rcp4+e128 (fixed prologue exp) and with the chunk's B-operand
# LDS reads software-pipelined 4 / 6 / 8 deep; GPU suite on the two leading candidates.
set -uo pipefail
bash tools/gpu_run.sh r5c "ab=3=base,u5_rcp4_e128,h_d4,h_d6,h_d8" lib=tools/variants/u5_rcp4_e128.so "tests=parity or line_centres or config1 or i8_equals or panel_gemm_equals_fused" lib=tools/variants/h_d6.so "testfile=tests/test_gpu_parity.py" lib=head
