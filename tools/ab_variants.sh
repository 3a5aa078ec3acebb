#!/bin/bash
# A/B: run the bench (no CPU baseline) against each tools/variants/*.so, interleaved rounds.
set -uo pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for so in tools/variants/*.so; do
    n=$(basename $so .so)
    GPDLA_LIB=$PWD/$so timeout -k 10 300 python bench.py --cpu-budget 0 "$@" > gpurun_out/ab_${n}_${round}.json 2>gpurun_out/ab_${n}_${round}.err || { echo "FAIL $n"; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${n}_${round}.json').read().strip().splitlines()[-1]); print('$n', $round, round(d['value']/1e6,2), 'Mevals/s', round(d['kernel_ms']['likelihood'],2), 'ms', d['checks_ok'])"
  done
done
