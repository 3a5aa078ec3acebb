# r5l: prep_kernel with 2 or 4 blocks per spectrum on the fused layout (GPDLA_PREP_Y; head = 1):
# configs[1] A/B, interleaved.
set -uo pipefail
bash tools/gpu_run.sh r5l "ab=3=head,prep_y2,prep_y4"
