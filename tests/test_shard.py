"""Multi-process sharding on CPU (gloo, world size 2): partition, per-rank compute, gather, merge.

The per-spectrum compute here is a deterministic stand-in (a function of the spectrum's own
pixels only, like the real hot path); the GPU-side equivalence of sharded vs unsharded engine runs
is covered by tests/test_gpu_parity.py::test_engine_batching_and_sharding_bitwise."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gp_dla_detection_amd import synthetic as syn
from gp_dla_detection_amd.shard import (block_lpt_shards, contiguous_shards, expected_pixels, lpt_shards, merge_shards,
                                        process_sharded, subset_packed)


def _compute(p):
    off = p["offsets"]
    Q = off.size - 1
    s = np.array([np.sum(p["flux"][off[q]:off[q + 1]] * p["noise_variance"][off[q]:off[q + 1]]) for q in range(Q)])
    return dict(stat=s, sample=np.outer(s, np.arange(3.0)), n=np.diff(off).astype(np.int32))


def _packed():
    model = syn.make_model(k=4, seed=1)
    return syn.pack_spectra(syn.make_dr12q_like_spectra(model, 9, seed=2))


def test_partitions_cover_exactly_once():
    for Q, W in ((10, 3), (7, 8), (1024, 8)):
        parts = contiguous_shards(Q, W)
        assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(Q))
    costs = np.random.default_rng(0).integers(269, 1250, 100)
    parts = lpt_shards(costs, 8)
    assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(100))
    loads = [costs[p].sum() for p in parts]
    assert max(loads) - min(loads) <= costs.max()


def test_block_lpt_shards_whole_blocks_balanced():
    """Chunk-aligned shards (run_process_qsos, world > 1): every rank holds whole blocks of
    consecutive spectra, together exactly once; with DR12Q's count and ~4 MB chunks (56 rows at
    S = 10^4) the expected-pixel load is balanced to within one block (< 0.3%)."""
    rng = np.random.default_rng(3)
    for Q, block, W in ((10, 3, 3), (7, 2, 8), (162861, 56, 8)):
        costs = expected_pixels(rng.uniform(2.15, 6.0, Q))
        shards = block_lpt_shards(costs, block, W)
        allidx = np.sort(np.concatenate(shards))
        assert np.array_equal(allidx, np.arange(Q))
        for sh in shards:
            assert np.all(np.diff(sh) > 0)
            for b in np.unique(sh // block):    # whole blocks only
                assert np.array_equal(sh[sh // block == b], np.arange(b * block, min(Q, (b + 1) * block)))
        if Q > 1000:
            loads = [costs[sh].sum() for sh in shards]
            assert max(loads) / np.mean(loads) < 1.003     # LPT: within about one block of the mean
    assert all(sh.size == 0 for sh in block_lpt_shards(np.zeros(0), 4, 3))


def test_expected_pixels_matches_synthetic_spectra():
    """The sweep-cost proxy against the in-range pixel count of DR12Q-shaped synthetic spectra
    (BOSS 3600 A blue edge): within 2 pixels."""
    model = syn.make_model(k=4, seed=1)
    sp = syn.make_dr12q_like_spectra(model, 40, seed=5, mask_fraction=0.0)
    from gp_dla_detection_amd import parameters as P
    n = [int(np.sum((s["wavelengths"] / (1 + s["z_qso"]) >= P.MIN_LAMBDA)
                    & (s["wavelengths"] / (1 + s["z_qso"]) <= P.MAX_LAMBDA))) for s in sp]
    est = expected_pixels([s["z_qso"] for s in sp])
    assert np.max(np.abs(est - np.array(n))) <= 2


def test_subset_and_merge_roundtrip():
    p = _packed()
    full = _compute(p)
    shards = lpt_shards(np.diff(p["offsets"]), 3)
    merged = merge_shards(9, shards, [_compute(subset_packed(p, s)) for s in shards])
    for k in full:
        np.testing.assert_array_equal(merged[k], full[k])


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = _packed()
    out = process_sharded(p, _compute, rank, world, gather=True, costs=np.diff(p["offsets"]))
    if rank == 0:
        q.put({k: v for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_gloo_world2_gather_equals_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    full = _compute(_packed())
    for k in full:
        np.testing.assert_array_equal(got[k], full[k])
