set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r2n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s -k standalone --timeout 200 --timeout-method thread > $O/standalone.log 2>&1; tail -2 $O/standalone.log
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload c2 --steps 5 --warmup 2 --cpu-budget 0 > $O/c2_n2.json 2> $O/c2_n2.err || { echo c2n2 failed; exit 1; }
tail -c 300 $O/c2_n2.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload c4 --steps 1 --warmup 1 --cpu-budget 0 > $O/c4_n2.json 2> $O/c4_n2.err || { echo c4n2 failed; exit 1; }
tail -c 300 $O/c4_n2.json
timeout -k 10 700 python bench.py --workload e2e > $O/e2e.json 2> $O/e2e.err || { echo e2e failed; exit 1; }
cat $O/e2e.json
