"""Spectrum sharding across GPUs.

The hot path has no exchange step: every spectrum's null evaluation, S sample evaluations and
log-mean-exp depend only on that spectrum plus the replicated model and samples
(process_qsos.m:88-220).  So N GPUs = N independent processes, each owning a disjoint set of
spectra, no collective on the data path.  Results can stay sharded (one output per rank) or be
gathered to rank 0 on the host.
"""
from __future__ import annotations

import heapq

import numpy as np


def contiguous_shards(num_spectra: int, world: int) -> list[np.ndarray]:
    """Balanced contiguous index ranges (fixed-n workloads)."""
    bounds = np.linspace(0, num_spectra, world + 1).round().astype(np.int64)
    return [np.arange(bounds[r], bounds[r + 1], dtype=np.int64) for r in range(world)]


def lpt_shards(costs, world: int) -> list[np.ndarray]:
    """Longest-processing-time assignment by per-spectrum cost (e.g. pixel count n, which sets the
    sweep length; real DR12Q spectra span n = 269..1250).  Each shard is returned sorted."""
    costs = np.asarray(costs, dtype=np.float64)
    order = np.argsort(-costs, kind="stable")
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    owner = np.empty(costs.size, dtype=np.int64)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + costs[i], r))
    return [np.flatnonzero(owner == r) for r in range(world)]


def block_lpt_shards(costs, block: int, world: int) -> list[np.ndarray]:
    """LPT over blocks of ``block`` consecutive spectra (the last block may be short): each rank
    gets whole blocks, so with ``block`` = the output file's chunk rows (matv73.auto_chunk_rows) every
    rank writes whole chunks of the Q x S sample array and no two ranks share a file range.  Each
    shard is returned sorted."""
    costs = np.asarray(costs, dtype=np.float64)
    n = costs.size
    if n == 0:
        return [np.zeros(0, np.int64) for _ in range(world)]
    starts = np.arange(0, n, block)
    owners = lpt_shards(np.add.reduceat(costs, starts), world)
    return [np.concatenate([np.arange(starts[b], min(n, starts[b] + block)) for b in blk]).astype(np.int64)
            if blk.size else np.zeros(0, np.int64) for blk in owners]


def expected_pixels(z_qsos, blue_limit: float = 3600.0) -> np.ndarray:
    """Sweep-cost proxy before any spectrum is decoded: the 1e-4 dex pixels a spectrum at z_QSO has
    in the modelled rest range (set_parameters.m:33-35, 59-60), observed-frame clipped at the
    spectrograph's blue edge (BOSS: 3600 A).  Only balances shards; it never changes a result."""
    from .parameters import MAX_LAMBDA, MIN_LAMBDA, PIXEL_SPACING
    z = np.asarray(z_qsos, dtype=np.float64)
    top = np.log10(MAX_LAMBDA * (1 + z))
    bottom = np.maximum(np.log10(MIN_LAMBDA * (1 + z)), np.log10(blue_limit))
    return np.maximum((top - bottom) / PIXEL_SPACING, 1.0)


def subset_packed(packed: dict, idx: np.ndarray) -> dict:
    """CSR subset of packed spectra (see synthetic.pack_spectra)."""
    off = packed["offsets"]
    lens = off[idx + 1] - off[idx]
    new_off = np.zeros(idx.size + 1, dtype=np.int64)
    np.cumsum(lens, out=new_off[1:])
    take = np.concatenate([np.arange(off[q], off[q + 1]) for q in idx]) if idx.size else np.zeros(0, np.int64)
    return dict(offsets=new_off, wavelengths=packed["wavelengths"][take], flux=packed["flux"][take],
                noise_variance=packed["noise_variance"][take], pixel_mask=packed["pixel_mask"][take],
                z_qsos=packed["z_qsos"][idx])


def merge_shards(num_spectra: int, shards: list[np.ndarray], results: list[dict]) -> dict:
    """Scatter per-shard result dicts back into spectrum order."""
    out = {}
    for idx, res in zip(shards, results):
        for key, val in res.items():
            if not isinstance(val, np.ndarray) or val.shape[:1] != (idx.size,):
                continue
            if key not in out:
                out[key] = np.empty((num_spectra,) + val.shape[1:], dtype=val.dtype)
            out[key][idx] = val
    return out


def process_sharded(packed: dict, compute, rank: int, world: int, gather: bool = True,
                    costs=None):
    """Run ``compute(packed_subset) -> dict of per-spectrum arrays`` on this rank's shard.

    With ``gather`` the shards are collected on rank 0 over torch.distributed (host objects,
    any backend; gloo suffices because the data never leaves the host path) and merged into
    spectrum order; other ranks return their local result."""
    Q = packed["z_qsos"].size
    shards = lpt_shards(costs, world) if costs is not None else contiguous_shards(Q, world)
    local = compute(subset_packed(packed, shards[rank]))
    if not gather or world == 1:
        return merge_shards(Q, shards, [local]) if world == 1 else local
    import torch.distributed as dist
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(local, gathered, dst=0)
    if rank != 0:
        return local
    return merge_shards(Q, shards, gathered)
