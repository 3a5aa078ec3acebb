"""bench.py's multi-rank machinery on CPU (gloo, world size 2): the timed region's barriers and
max-over-ranks reduction (timed_steps) and the configs[3] LPT spectrum split (dr12q_shard)."""
import importlib.util
import os
import socket
import time
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _bench()
        syncs = []
        el = bench.timed_steps(lambda: time.sleep(0.05 * (rank + 1)), lambda: syncs.append(1), 3, dist)
        q.put((rank, el, len(syncs)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_timed_steps_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (el, ns) for r, el, ns in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 1 sleeps 3 x 0.10 s: both ranks report its time (the max), and each synced twice
    assert got[0][0] == got[1][0]
    assert 0.29 < got[0][0] < 2.0
    assert got[0][1] == got[1][1] == 2


def test_dr12q_lpt_shards_cover_and_balance():
    bench = _bench()
    rng = np.random.default_rng(0)
    pixels = rng.integers(270, 1251, 4096)
    total = 162861
    for world in (2, 3, 8):
        shards = [bench.dr12q_shard(pixels, total, r, world, split=True) for r in range(world)]
        # every spectrum exactly once (pool index i % 4096 counted per position)
        counts = np.bincount(np.concatenate(shards), minlength=4096)
        np.testing.assert_array_equal(counts, np.bincount(np.arange(total) % 4096, minlength=4096))
        loads = np.array([pixels[s].sum() for s in shards], dtype=np.float64)
        assert loads.max() / loads.mean() < 1.001
    np.testing.assert_array_equal(bench.dr12q_shard(pixels, total, 0, 8, split=False), np.arange(total) % 4096)
