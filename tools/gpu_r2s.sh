#!/bin/bash
# configs[3] rehearsal on files: the full-DR12Q end-to-end run (run_process_qsos, 13 GB v7.3 out)
# with 2 and 4 ranks sharing the one leased GPU (each rank decodes, evaluates and writes its shard).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2s; mkdir -p $O
for n in 2 4; do
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --workload e2e > $O/e2e_n$n.json 2> $O/e2e_n$n.err || { echo "e2e n=$n failed"; tail -20 $O/e2e_n$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/e2e_n$n.json'));print($n, d['e2e'])"
done
echo all-done
