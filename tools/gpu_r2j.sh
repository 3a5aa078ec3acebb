#!/bin/bash
# Round-2 session j: rocprofv3 profiles of HEAD (c2 fused fp64, c5 int8 panel-GEMM 24-bit).
set -uo pipefail
export TMPDIR=/tmp
bash tools/profile.sh r2j || exit 1
bash tools/profile.sh r2j_c5 --workload c5 || exit 1
echo session-done
