#!/bin/bash
# Final tree: default bench line (N = 1), then the multi-rank bench path rehearsed with 2 and 4 ranks
# sharing the one leased GPU (launcher started before any GPU call; weak scaling, so the total rate
# should equal the 1-rank rate on a shared device).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_c2_n1.json 2> $O/n1.err || { echo n1 failed; tail -5 $O/n1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2_n1.json'));print('n1', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload c2 --steps 5 --warmup 2 --cpu-budget 0 > $O/bench_c2_n2_shared_gpu.json 2> $O/n2.err || { echo n2 failed; tail -5 $O/n2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2_n2_shared_gpu.json'));print('n2', d['value'], d['ms_per_step'], d['n_gpus'])"
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --workload c2 --steps 3 --warmup 1 --cpu-budget 0 > $O/bench_c2_n4_shared_gpu.json 2> $O/n4.err || { echo n4 failed; tail -5 $O/n4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2_n4_shared_gpu.json'));print('n4', d['value'], d['ms_per_step'], d['n_gpus'])"
echo all-done
