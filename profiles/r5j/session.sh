# r5j: XCD split of the B-stationary Gram GEMM: EX = 4 (head), 2, 8 entry-tile ranges; configs[4] A/B.
set -uo pipefail
bash tools/gpu_run.sh r5j "ab=3=head,bst_ex2,bst_ex8=--workload c5"
