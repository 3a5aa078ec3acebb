# r5b: headline A/B -- base (HEAD~) vs chunk loop unrolled x5 (u5), + batched reciprocals (rcp4),
# + 128-entry exp table without clamp on the main path (e128); then the whole GPU suite on the last.
set -uo pipefail
bash tools/gpu_run.sh r5b "ab=3=base,u5,u5_rcp4,u5_rcp4_e128" lib=tools/variants/u5_rcp4_e128.so tests lib=head
