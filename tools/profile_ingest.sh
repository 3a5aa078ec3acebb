#!/bin/bash
# rocprofv3 passes over tools/bench_ingest.py (GPU box, repo root): kernel trace, then FETCH_SIZE and
# WRITE_SIZE in passes of their own (MI355X_MICROARCH.md, HBM section).  Summarise with
#   python3 tools/summarize_ingest.py <out dir> > profiles/<round>/<tag>_ingest.md
set -euo pipefail
OUT=${1:-gpurun_out/ingest}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 tools/bench_ingest.py "$OUT/bench_trace.json" > "$OUT/trace.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 tools/bench_ingest.py > "$OUT/fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 tools/bench_ingest.py > "$OUT/write.log" 2>&1
