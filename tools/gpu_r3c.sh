#!/bin/bash
# rocprofv3 passes (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ mix) of both bench workloads on HEAD.
set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 900 bash tools/profile.sh r3c > gpurun_out/prof_r3c.log 2>&1 || { echo prof c2 failed; tail -5 gpurun_out/prof_r3c.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh r3c_c5 --workload c5 > gpurun_out/prof_r3c_c5.log 2>&1 || { echo prof c5 failed; tail -5 gpurun_out/prof_r3c_c5.log; exit 1; }
echo all-done
