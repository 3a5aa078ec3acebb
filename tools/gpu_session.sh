#!/bin/bash
# One GPU-box session: the -m gpu suite, then optional extra steps, each under its own time limit.
# Usage: tools/gpu_session.sh <tag> [extra command ...]   (outputs under gpurun_out/<tag>/)
# A test failure (pytest rc 1) still lets the extra steps run; a timeout, abort or crash stops here.
set -uo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -5 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
for step in "$@"; do
  echo "== $step"
  bash -c "$step"
  r=$?
  if [ $r -ne 0 ]; then echo "step rc=$r: stopping"; exit $r; fi
done
exit $rc
