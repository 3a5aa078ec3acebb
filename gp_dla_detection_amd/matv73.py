"""MATLAB v7.3 ``.mat`` files (HDF5 behind a 512-byte MATLAB user block), in numpy only.

The reference saves its result with ``save(filename, variables_to_save{:}, '-v7.3')``
(process_qsos.m:249) and loads its inputs with ``load`` from v7.3 files written by the same
pipeline (process_qsos.m:4,30-50).  ``sample_log_likelihoods_dla`` is Q x S doubles: 13.0 GB at
full DR12Q, far over the 2 GB per-variable limit of MATLAB v5 files, and h5py is
not installed on the GPU box.  So this module writes and reads the HDF5 subset MATLAB uses,
directly:

writer (``savemat73``)
  superblock v0 at file offset 512 (base address 512, the layout libhdf5 itself writes for a
  user block), old-style groups (v1 B-tree + symbol-table nodes + local heap), v1 object
  headers, contiguous datasets -- and chunked ones (v1 B-tree index) for large 2-D arrays, as
  MATLAB's own v7.3 saves are chunked: a chunk is a block of whole MATLAB rows (all S columns of
  ``chunk_rows`` spectra), so one process per GPU writes whole chunks of its own spectra with
  one ``pwrite`` each instead of pieces of every file row.  Every variable carries MATLAB's
  ``MATLAB_class`` attribute
  (plus ``MATLAB_int_decode`` for logical/char, ``MATLAB_empty`` for empties); cell arrays are
  object-reference datasets into ``#refs#`` as MATLAB writes them.  Array data is laid out
  MATLAB-style: a MATLAB r x c matrix is HDF5 dims (c, r), column-major bytes.  A variable may be
  a ``LazyArray`` whose bytes are streamed into a memory map of the file after the metadata is
  written (how process.save_processed_qsos writes the 13 GB sample array straight from the
  spectrum-major engine output without a second host copy of it transposed).

reader (``loadmat73``)
  superblock v0-v3, object headers v1/v2 with continuations, symbol-table and compact link
  groups, contiguous / compact / chunked (v1 B-tree) layouts with the deflate, shuffle and
  fletcher32 filters (MATLAB compresses v7.3 variables by default), fixed/float/string/
  reference/compound(complex) types, attributes, and MATLAB class decoding (double, single,
  integers, logical, char, cell, struct, empty).

What h5py sees in a file written here matches what it sees in MATLAB's: a Q-vector is (1, Q),
``sample_log_likelihoods_dla`` is (S, Q) (calc_cddf.py:61-64,92,98).
"""
from __future__ import annotations

import math
import mmap
import os
import struct
import time
import zlib
from dataclasses import dataclass
from typing import Callable

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIGNATURE = b"\x89HDF\r\n\x1a\n"
USERBLOCK = 512
LEAF_K = 4          # group leaf node K: a symbol-table node holds 2K entries (libhdf5 default)
INTERNAL_K = 16     # group internal node K: a B-tree node holds 2K children (libhdf5 default)
CHUNK_K = 32        # chunk B-tree K (indexed-storage K; a v0 superblock implies libhdf5's default 32)
CHUNK_TARGET = 4 << 20   # bytes per chunk of a large 2-D array (auto_chunk_rows)
_STREAM_BYTES = 1 << 26  # arrays at least this large are streamed into the file map

_MATLAB_CLASS = {np.dtype(np.float64): "double", np.dtype(np.float32): "single",
                 np.dtype(np.int8): "int8", np.dtype(np.uint8): "uint8",
                 np.dtype(np.int16): "int16", np.dtype(np.uint16): "uint16",
                 np.dtype(np.int32): "int32", np.dtype(np.uint32): "uint32",
                 np.dtype(np.int64): "int64", np.dtype(np.uint64): "uint64"}
_CLASS_DTYPE = {v: k for k, v in _MATLAB_CLASS.items()}


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


# ============================================================================ writer
@dataclass
class LazyArray:
    """A numeric variable whose bytes are produced after the file layout is fixed.

    ``shape`` is the MATLAB shape (e.g. (Q, S)); ``fill(view)`` receives a writable
    array of that MATLAB shape and dtype (a Fortran-ordered view of the file's bytes) and must
    assign every element.  ``fill=None`` defers the bytes to other writers (``open_region`` for a
    contiguous variable, ``write_chunks`` for a chunked one).  ``chunk_rows`` makes the 2-D
    variable chunked: HDF5 chunks of (columns, chunk_rows), i.e. blocks of whole MATLAB rows."""
    shape: tuple
    dtype: np.dtype
    fill: Callable[[np.ndarray], None] | None = None
    src: np.ndarray | None = None   # set instead of fill: written by write_chunks / write_transposed
    chunk_rows: int | None = None


def auto_chunk_rows(cols: int, itemsize: int = 8, rows: int | None = None) -> int:
    """MATLAB rows per chunk of a large R x ``cols`` array: ~CHUNK_TARGET bytes, a multiple of 8
    rows, at most ``rows``.  It depends on the column count only, so every rank can shard its
    spectra chunk-aligned before the file exists."""
    row_bytes = max(cols * itemsize, 1)
    r = max(8, int(round(CHUNK_TARGET / row_bytes / 8)) * 8)
    r = min(r, max(1, 0xFFFFFFFF // row_bytes))            # chunk bytes < 4 GiB (32-bit B-tree key)
    return max(1, min(r, rows)) if rows else r


def _dt_message(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "f":
        if dt.itemsize == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            bits = (0x20, 63, 0)
        elif dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            bits = (0x20, 31, 0)
        else:
            raise TypeError(f"unsupported float width {dt.itemsize}")
        return bytes([0x11, *bits]) + struct.pack("<I", dt.itemsize) + props
    if dt.kind in "iub":
        signed = 0x08 if dt.kind == "i" else 0
        return bytes([0x10, signed, 0, 0]) + struct.pack("<IHH", dt.itemsize, 0, 8 * dt.itemsize)
    raise TypeError(f"unsupported dtype {dt}")


def _dt_string(n: int) -> bytes:
    return bytes([0x13, 0x00, 0, 0]) + struct.pack("<I", n)      # fixed, null-terminated ASCII


_DT_OBJREF = bytes([0x17, 0x00, 0, 0]) + struct.pack("<I", 8)


def _dataspace(dims) -> bytes:
    return bytes([1, len(dims), 0, 0, 0, 0, 0, 0]) + b"".join(struct.pack("<Q", int(d)) for d in dims)


def _attr_message(name: str, value) -> bytes:
    nm = name.encode() + b"\0"
    if isinstance(value, str):
        raw = value.encode("ascii")
        dt, ds, data = _dt_string(len(raw)), _dataspace(()), raw
    else:
        arr = np.asarray(value)
        dt, ds, data = _dt_message(arr.dtype), _dataspace(()), arr.astype(arr.dtype.newbyteorder("<")).tobytes()
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds)) + _pad8(nm) + _pad8(dt) + _pad8(ds) + data
    return _pad8(body)


def _object_header(messages: list[tuple[int, bytes]]) -> bytes:
    body = b"".join(struct.pack("<HHB3x", t, len(m), 0) + m for t, m in messages)
    return struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body)) + body


class _Node:
    """One object to lay out: a dataset (data bytes or lazy) or a group (children)."""

    def __init__(self, name, kind, **kw):
        self.name, self.kind = name, kind
        self.chunk = None
        self.__dict__.update(kw)
        self.addr = None


def _matlab_node(name: str, value, refs: list) -> _Node:
    """Map a Python/numpy value to MATLAB's HDF5 representation."""
    attrs: list = []
    if isinstance(value, LazyArray):
        dt = np.dtype(value.dtype)
        return _Node(name, "dataset", dims=tuple(reversed(value.shape)), dtype=dt, data=None,
                     lazy=value, chunk=_chunk_dims(value), attrs=[("MATLAB_class", _MATLAB_CLASS[dt])])
    if isinstance(value, dict):
        # MATLAB scalar struct: a group with MATLAB_class "struct", one member per field (this is
        # also the side format for the catalogue's containers.Map variables, SURVEY.md 7 viii)
        kids = [_matlab_node(k, v, refs) for k, v in value.items()]
        return _Node(name, "group", entries=kids, attrs=[("MATLAB_class", "struct")])
    if isinstance(value, str):
        codes = np.frombuffer(value.encode("utf-16-le"), dtype="<u2") if value else np.zeros(0, "<u2")
        arr, cls = codes.reshape(1, -1), "char"
        attrs.append(("MATLAB_int_decode", np.int32(2)))
    elif isinstance(value, (list, tuple)) or (isinstance(value, np.ndarray) and value.dtype == object):
        if isinstance(value, (list, tuple)):
            cells = np.empty(len(value), dtype=object)
            for i, v in enumerate(value):
                cells[i] = v
        else:
            cells = value
        if cells.ndim == 1:
            cells = cells.reshape(-1, 1)                    # MATLAB n x 1 cell (like preload_qsos)
        targets = []
        for v in cells.ravel(order="F"):
            idx = len(refs)
            refs.append(None)                               # reserve the name before recursing
            refs[idx] = child = _matlab_node(_refname(idx), v, refs)
            targets.append(child)
        if not targets:
            return _empty_node(name, cells.shape, "cell")
        return _Node(name, "dataset", dims=tuple(reversed(cells.shape)), dtype=None, ref_targets=targets,
                     data=None, lazy=None, attrs=[("MATLAB_class", "cell")])
    else:
        arr = np.asarray(value)
        if arr.dtype == bool:
            arr, cls = arr.astype(np.uint8), "logical"
            attrs.append(("MATLAB_int_decode", np.int32(1)))
        elif arr.dtype.kind in "iuf" and arr.dtype in _MATLAB_CLASS:
            cls = _MATLAB_CLASS[arr.dtype]
        elif arr.dtype.kind in "iu":
            arr, cls = arr.astype(np.int64), "int64"
        else:
            raise TypeError(f"{name}: cannot store dtype {arr.dtype} in a MATLAB file")
        if arr.ndim == 0:
            arr = arr.reshape(1, 1)
        elif arr.ndim == 1:
            arr = arr.reshape(-1, 1)                          # MATLAB column vector (oned_as column)
    if arr.size == 0:
        return _empty_node(name, arr.shape, cls, extra=attrs)
    if arr.nbytes >= _STREAM_BYTES and arr.ndim == 2:
        # large: chunked (blocks of whole rows), each chunk transposed and pwritten (write_chunks)
        lazy = LazyArray(arr.shape, arr.dtype, src=arr,
                         chunk_rows=auto_chunk_rows(arr.shape[1], arr.dtype.itemsize, arr.shape[0]))
        return _Node(name, "dataset", dims=tuple(reversed(arr.shape)), dtype=arr.dtype, data=None,
                     lazy=lazy, chunk=_chunk_dims(lazy), attrs=[("MATLAB_class", cls)] + attrs)
    data = np.asfortranarray(arr)
    return _Node(name, "dataset", dims=tuple(reversed(arr.shape)), dtype=data.dtype, data=data, lazy=None,
                 attrs=[("MATLAB_class", cls)] + attrs)


def _chunk_dims(lazy: LazyArray):
    """HDF5 chunk dims (C order: columns, rows) of a chunked LazyArray, or None."""
    if not lazy.chunk_rows:
        return None
    if len(lazy.shape) != 2:
        raise ValueError("a chunked LazyArray must be 2-D")
    R, C = (int(d) for d in lazy.shape)
    return (C, int(min(lazy.chunk_rows, max(R, 1))))


def fill_transposed(view, src, tile_rows: int = 512, tile_cols: int = 2048, threads: int | None = None):
    """``view[:] = src`` for a 2-D MATLAB-shaped ``view`` that is the transpose of a C-order file map
    (open_region): the copy is a transpose in memory, done in cache-sized tiles (each tile row is a
    contiguous 4 KiB run of the file) on a thread pool (numpy copies release the GIL).  A
    row-at-a-time strided copy ran at ~0.8 GB/s; the 13 GB full-DR12Q sample array needs better."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    if view.ndim != 2:
        view[...] = src
        return
    R, Cn = src.shape
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1))

    def band(r0):
        r1 = min(R, r0 + tile_rows)
        for c0 in range(0, Cn, tile_cols):
            view[r0:r1, c0:c0 + tile_cols] = src[r0:r1, c0:c0 + tile_cols]

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(band, range(0, R, tile_rows)))


def write_transposed(path: str, offset: int, src: np.ndarray, row0: int = 0, rows_total: int | None = None,
                     band: int = 32, threads: int | None = None):
    """Write the MATLAB-shaped 2-D array ``src`` (R x C) in column-major order -- the file's C-order
    (C, rows_total) dataset at byte ``offset``, rows row0 .. row0 + R of the MATLAB array (one rank's
    spectra; all of them by default) -- band by band: each thread transposes src[:, c0:c0+band] into its
    own buffer and pwrite()s it (one write per band when the rows are all of the file's, else one per
    file row).  No memory map of the output: a first-touch page fault per 4 KiB of a 13 GB map cost
    more than the copy (the map-based fill ran at ~1.4 GB/s on the full-DR12Q sample array)."""
    from concurrent.futures import ThreadPoolExecutor
    R, C = src.shape
    Rt = R if rows_total is None else rows_total
    dt = np.dtype(src.dtype).newbyteorder("<")
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1))
    fd = os.open(path, os.O_WRONLY)
    try:
        def run(c0):
            c1 = min(C, c0 + band)
            buf = np.empty((c1 - c0, R), dtype=dt)
            buf[...] = src[:, c0:c1].T
            runs = [(memoryview(buf).cast("B"), offset + c0 * Rt * dt.itemsize)] if Rt == R else \
                   [(memoryview(buf[c - c0]).cast("B"), offset + (c * Rt + row0) * dt.itemsize) for c in range(c0, c1)]
            for mv, pos in runs:
                while len(mv):
                    n = os.pwrite(fd, mv, pos)
                    mv, pos = mv[n:], pos + n

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(run, range(0, C, band)))
    finally:
        os.close(fd)


def write_chunks(path: str, region: "Region", src: np.ndarray, row0: int = 0, threads: int | None = None):
    """Write MATLAB rows row0 .. row0 + R of a chunked region (savemat73 with a ``chunk_rows``
    LazyArray).  ``src`` is R x C, spectrum-major like the engine's output, and must cover whole
    chunks: row0 a multiple of chunk_rows, and R too unless the block ends at the last row.  Each
    chunk is transposed into its own buffer (the chunk's C-order (C, chunk_rows) bytes, the last one
    zero-padded) and written with one ``pwrite``.  Chunks are disjoint 4 KiB-aligned file ranges,
    so processes can write their own chunks concurrently."""
    from concurrent.futures import ThreadPoolExecutor
    cr, stride = region.chunk_rows, region.chunk_stride
    C, Rt = region.dims
    R = src.shape[0]
    if not cr:
        raise ValueError("region is not chunked (use write_transposed)")
    if src.ndim != 2 or src.shape[1] != C or row0 % cr or row0 + R > Rt or (R % cr and row0 + R != Rt):
        raise ValueError(f"rows {row0}..{row0 + R} of a {Rt} x {C} array are not whole {cr}-row chunks")
    dt = np.dtype(region.dtype)
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1))
    fd = os.open(path, os.O_WRONLY)
    try:
        def run(r0):
            r1 = min(R, r0 + cr)
            buf = np.zeros((C, cr), dtype=dt)
            buf[:, : r1 - r0] = src[r0:r1].T
            mv, pos = memoryview(buf).cast("B"), region.offset + (row0 + r0) // cr * stride
            while len(mv):
                n = os.pwrite(fd, mv, pos)
                mv, pos = mv[n:], pos + n

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(run, range(0, R, cr)))
    finally:
        os.close(fd)


def _empty_node(name, shape, cls, extra=()):
    # MATLAB stores an empty array as its dimensions (uint64) plus MATLAB_empty = 1
    dims = np.array(shape if len(shape) >= 2 else (0, 0), dtype=np.uint64)
    return _Node(name, "dataset", dims=(dims.size,), dtype=np.dtype(np.uint64), data=dims, lazy=None,
                 attrs=[("MATLAB_class", cls), ("MATLAB_empty", np.uint8(1))] + list(extra))


def _refname(i: int) -> str:
    """MATLAB's #refs# naming: a, b, ..., z, ba, bb, ... (base 26 on the letters a-z)."""
    s = ""
    while True:
        s = chr(ord("a") + i % 26) + s
        i //= 26
        if i == 0:
            return s


def _dataset_header(node: _Node, data_addr: int) -> bytes:
    """v1 object header of a dataset.  ``data_addr`` is the data (contiguous layout) or the root
    node of the chunk B-tree (chunked: layout message v3 class 2, the chunk dims + element size)."""
    if getattr(node, "ref_targets", None) is not None:
        dt, nbytes = _DT_OBJREF, 8 * len(node.ref_targets)
    else:
        dt = _dt_message(node.dtype)
        nbytes = int(np.prod(node.dims)) * node.dtype.itemsize
    if node.chunk is not None:
        layout = bytes([3, 2, len(node.chunk) + 1]) + struct.pack("<Q", data_addr) \
            + struct.pack(f"<{len(node.chunk) + 1}I", *node.chunk, node.dtype.itemsize)
    else:
        layout = bytes([3, 1]) + struct.pack("<QQ", data_addr, nbytes)
    msgs = [(0x0001, _pad8(_dataspace(node.dims))), (0x0003, _pad8(dt)), (0x0008, _pad8(layout))]
    msgs += [(0x000C, _attr_message(k, v)) for k, v in node.attrs]
    return _object_header(msgs)


def _group_header(node: _Node, btree: int, heap: int) -> bytes:
    msgs = [(0x0011, struct.pack("<QQ", btree, heap))]
    msgs += [(0x000C, _attr_message(k, v)) for k, v in node.attrs]
    return _object_header(msgs)


def _group_blocks(entries: list[_Node]):
    """Heap + symbol-table nodes + B-tree for a group; returns sizes so the layout can be fixed
    before addresses are known, and an emitter that encodes them once they are."""
    entries = sorted(entries, key=lambda e: e.name.encode())
    heap_data = bytearray(b"\0" * 8)                              # offset 0: the empty name
    name_off = {}
    for e in entries:
        name_off[e.name] = len(heap_data)
        heap_data += _pad8(e.name.encode() + b"\0")
    snods = [entries[i:i + 2 * LEAF_K] for i in range(0, len(entries), 2 * LEAF_K)] or [[]]
    snod_size = 8 + 2 * LEAF_K * 40
    node_size = 24 + 2 * INTERNAL_K * 8 + (2 * INTERNAL_K + 1) * 8
    # B-tree levels: level 0 over the SNODs, higher levels over nodes, until one root
    levels = []
    count = len(snods)
    while True:
        n_nodes = -(-count // (2 * INTERNAL_K))
        levels.append(n_nodes)
        if n_nodes == 1:
            break
        count = n_nodes
    return entries, bytes(heap_data), name_off, snods, snod_size, node_size, levels


def _chunk_plan(node: _Node) -> dict:
    """Sizes of a chunked 2-D dataset: its chunks (whole blocks of rows, each at a 4 KiB-aligned
    stride) and its v1 B-tree (type 1, raw-data chunks): 2K children per node, levels until one
    root.  Node size as libhdf5 computes it from K, so its reader finds every key."""
    C, Rt = node.dims
    cr = node.chunk[1]
    nchunks = max(1, -(-Rt // cr))
    chunk_bytes = C * cr * node.dtype.itemsize
    key_size = 8 + 8 * (len(node.chunk) + 1)
    levels, count = [], nchunks
    while True:
        count = -(-count // (2 * CHUNK_K))
        levels.append(count)
        if count == 1:
            break
    return dict(nchunks=nchunks, rows=cr, chunk_bytes=chunk_bytes, stride=-(-chunk_bytes // 4096) * 4096,
                key_size=key_size, node_size=24 + 2 * CHUNK_K * 8 + (2 * CHUNK_K + 1) * key_size, levels=levels)


def _chunk_btree(node: _Node, plan: dict, node_addrs: list, chunk_base: int) -> list[tuple[int, bytes]]:
    """Encode the chunk B-tree: key i = (chunk bytes, filter mask 0, offsets (0, i * rows, 0)) in
    front of child i; the key after the last chunk is the right bound libhdf5 writes (every scaled
    coordinate + 1, zero size).  Internal nodes carry their children's first keys and the right key
    of their last child."""
    C = node.dims[0]
    n, cr, isz = plan["nchunks"], plan["rows"], node.dtype.itemsize

    def key(i):
        if i < n:
            return struct.pack("<II3Q", plan["chunk_bytes"], 0, 0, i * cr, 0)
        return struct.pack("<II3Q", 0, 0, C, n * cr, isz)

    out = []
    per = 2 * CHUNK_K
    # spans[j] = (first chunk, end chunk) under child j of the current level
    children = [chunk_base + i * plan["stride"] for i in range(n)]
    spans = [(i, i + 1) for i in range(n)]
    for level, addrs in enumerate(node_addrs):
        new_spans = []
        for j, addr in enumerate(addrs):
            ch, sp = children[j * per:(j + 1) * per], spans[j * per:(j + 1) * per]
            left = addrs[j - 1] if j > 0 else UNDEF
            right = addrs[j + 1] if j + 1 < len(addrs) else UNDEF
            b = b"TREE" + bytes([1, level]) + struct.pack("<HQQ", len(ch), left, right)
            for c, (lo, _) in zip(ch, sp):
                b += key(lo) + struct.pack("<Q", c)
            b += key(sp[-1][1])
            out.append((addr, b.ljust(plan["node_size"], b"\0")))
            new_spans.append((sp[0][0], sp[-1][1]))
        children, spans = addrs, new_spans
    return out


class _Layout:
    def __init__(self):
        self.pos = 0
        self.blobs: list[tuple[int, bytes]] = []

    def alloc(self, size: int, align: int = 8) -> int:
        self.pos += -self.pos % align
        a = self.pos
        self.pos += size
        return a


def savemat73(path: str, variables: dict, created: str | None = None) -> dict:
    """Write ``variables`` (name -> numpy array / scalar / str / list(cell) / LazyArray) as a
    MATLAB v7.3 file.  1-D arrays become MATLAB column vectors (process_qsos.m's nan(Q, 1)).
    Returns {name: Region} for the LazyArray variables."""
    refs: list = []
    top = [_matlab_node(name, val, refs) for name, val in variables.items()]
    root = _Node("/", "group", entries=list(top), attrs=[])
    if refs:
        root.entries.append(_Node("#refs#", "group", entries=refs, attrs=[]))
    groups, datasets = [], []

    def collect(g):
        groups.append(g)
        for e in g.entries:
            (collect(e) if e.kind == "group" else datasets.append(e))

    collect(root)
    L = _Layout()
    sb_addr = L.alloc(96)
    # pass 1: addresses of every metadata structure (sizes do not depend on addresses)
    gmeta = []
    for gnode in groups:
        entries_sorted, heap_data, name_off, snods, snod_size, node_size, levels = _group_blocks(gnode.entries)
        g = dict(entries=entries_sorted, heap_data=heap_data, name_off=name_off, snods=snods)
        g["ohdr"] = L.alloc(len(_group_header(gnode, 0, 0)))
        g["heap"] = L.alloc(32)
        g["heap_data_addr"] = L.alloc(len(heap_data))
        g["snod_addr"] = [L.alloc(snod_size) for _ in snods]
        g["levels"] = [[L.alloc(node_size) for _ in range(n)] for n in levels]
        gnode.addr, gnode.g, g["node"] = g["ohdr"], g, gnode
        gmeta.append(g)
    rg = gmeta[0]
    for n in datasets:
        n.addr = L.alloc(len(_dataset_header(n, 0)))
    for n in datasets:                      # chunk B-trees (metadata; the chunks go with the lazy data)
        if n.chunk is not None:
            n.plan = _chunk_plan(n)
            n.tree = [[L.alloc(n.plan["node_size"]) for _ in range(cnt)] for cnt in n.plan["levels"]]
    data_addr = {}

    def nbytes(n):
        if getattr(n, "ref_targets", None) is not None:
            return 8 * len(n.ref_targets)
        return int(np.prod(n.dims)) * n.dtype.itemsize

    for n in datasets:                      # eager data first, lazy (large) regions last
        if n.lazy is None:
            data_addr[id(n)] = L.alloc(max(nbytes(n), 1))
    meta_end = L.pos
    for n in datasets:
        if n.lazy is not None:
            size = n.plan["nchunks"] * n.plan["stride"] if n.chunk is not None else max(nbytes(n), 1)
            data_addr[id(n)] = L.alloc(size, align=4096)
    eof = L.pos
    # pass 2: encode the metadata and the eager data
    img = bytearray(meta_end)

    def put(addr, b):
        img[addr:addr + len(b)] = b

    sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", LEAF_K, INTERNAL_K, 0)
    sb += struct.pack("<QQQQ", USERBLOCK, UNDEF, USERBLOCK + eof, UNDEF)
    sb += struct.pack("<QQII", 0, rg["ohdr"], 1, 0) + struct.pack("<QQ", rg["levels"][-1][0], rg["heap"])
    put(sb_addr, sb)
    for g in gmeta:
        put(g["ohdr"], _group_header(g["node"], g["levels"][-1][0], g["heap"]))
        # free-list head 1 = H5HL_FREE_NULL (no free block)
        put(g["heap"], b"HEAP" + bytes(4) + struct.pack("<QQQ", len(g["heap_data"]), 1, g["heap_data_addr"]))
        put(g["heap_data_addr"], g["heap_data"])
        for sn_addr, sn in zip(g["snod_addr"], g["snods"]):
            b = b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(sn))
            for e in sn:
                if e.kind == "group":
                    b += struct.pack("<QQII", g["name_off"][e.name], e.addr, 1, 0)
                    b += struct.pack("<QQ", e.g["levels"][-1][0], e.g["heap"])
                else:
                    b += struct.pack("<QQII", g["name_off"][e.name], e.addr, 0, 0) + bytes(16)
            put(sn_addr, b)
        # B-tree: level-0 children are the SNODs; key i+1 = heap offset of the last name under child i
        children = g["snod_addr"]
        child_last = [g["name_off"][sn[-1].name] if sn else 0 for sn in g["snods"]]
        per = 2 * INTERNAL_K
        for level, nodes in enumerate(g["levels"]):
            new_last = []
            for j, node_addr in enumerate(nodes):
                ch = children[j * per:(j + 1) * per]
                lk = child_last[j * per:(j + 1) * per]
                b = b"TREE" + bytes([0, level]) + struct.pack("<H", len(ch)) + struct.pack("<QQ", UNDEF, UNDEF)
                b += struct.pack("<Q", 0)
                for c, k in zip(ch, lk):
                    b += struct.pack("<QQ", c, k)
                put(node_addr, b)
                new_last.append(lk[-1])
            children, child_last = nodes, new_last
    for n in datasets:
        if n.chunk is not None:
            put(n.addr, _dataset_header(n, n.tree[-1][0]))
            for addr, b in _chunk_btree(n, n.plan, n.tree, data_addr[id(n)]):
                put(addr, b)
            continue
        put(n.addr, _dataset_header(n, data_addr[id(n)]))
        if getattr(n, "ref_targets", None) is not None:
            put(data_addr[id(n)], np.array([t.addr for t in n.ref_targets], dtype="<u8").tobytes())
        elif n.data is not None:
            put(data_addr[id(n)], np.ascontiguousarray(n.data.ravel(order="F")).astype(
                n.data.dtype.newbyteorder("<"), copy=False).tobytes())
    hdr = (f"MATLAB 7.3 MAT-file, Platform: GLNXA64, Created on: "
           f"{created or time.strftime('%a %b %d %H:%M:%S %Y')} HDF5 schema 1.00 .").encode()
    ub = hdr.ljust(116, b" ")[:116] + bytes(8) + struct.pack("<H", 0x0200) + b"IM"
    ub = ub.ljust(USERBLOCK, b"\0")
    lazies = [n for n in datasets if n.lazy is not None]
    with open(path, "wb") as f:
        f.write(ub)
        f.write(bytes(img))
        f.truncate(USERBLOCK + eof)     # lazy regions: sparse until filled through the memory map
    regions = {}
    for n in lazies:
        chunked = n.chunk is not None
        reg = Region(USERBLOCK + data_addr[id(n)], tuple(int(d) for d in n.dims), np.dtype(n.dtype).str,
                     n.plan["rows"] if chunked else 0, n.plan["stride"] if chunked else 0)
        regions[n.name] = reg
        if n.lazy.src is not None:
            if chunked:
                write_chunks(path, reg, n.lazy.src)
            else:
                write_transposed(path, reg.offset, n.lazy.src)
            continue
        if n.lazy.fill is None:
            continue                          # deferred: filled later via open_region / write_chunks
        if chunked:
            raise ValueError(f"{n.name}: a chunked LazyArray takes src= or is deferred, not fill=")
        mm = open_region(path, reg)
        n.lazy.fill(mm)
        # no msync: like MATLAB's save (plain writes), the data is in the page cache and visible
        # to every reader when this returns; the kernel writes it back in the background
        del mm
    return regions


@dataclass(frozen=True)
class Region:
    """Where a variable's bytes live in a written file: absolute byte offset, HDF5 (C-order) dims
    and numpy dtype string; for a chunked variable, MATLAB rows per chunk and the byte stride
    between chunks (``offset`` is then the first chunk).  A ``LazyArray`` with ``fill=None`` is
    left for other writers (e.g. one process per GPU, each writing its own spectra) to fill
    through ``open_region`` (contiguous) or ``write_chunks`` (chunked)."""
    offset: int
    dims: tuple
    dtype: str
    chunk_rows: int = 0
    chunk_stride: int = 0


def open_region(path: str, region: Region, mode: str = "r+") -> np.ndarray:
    """A writable view of a contiguous variable's data in MATLAB shape (the transpose of a memory
    map of the HDF5 C-order dims).  Several processes may fill disjoint parts of it concurrently."""
    if region.chunk_rows:
        raise ValueError("chunked region: write it with write_chunks")
    mm = np.memmap(path, dtype=np.dtype(region.dtype).newbyteorder("<"), mode=mode,
                   offset=region.offset, shape=region.dims)
    return mm.T


# ============================================================================ reader
class _Reader:
    def __init__(self, path: str):
        self.f = open(path, "rb")
        # a plain mmap: slicing it returns bytes without numpy-subclass overhead (4 x 162,861 cell
        # headers are parsed at full DR12Q); self.mm is a uint8 view of it for the superblock scan
        self.buf = mmap.mmap(self.f.fileno(), 0, access=mmap.ACCESS_READ)
        self.mm = np.frombuffer(self.buf, dtype=np.uint8)
        self.base = self._find_superblock()

    def close(self):
        del self.mm
        try:
            self.buf.close()
        except BufferError:  # arrays decoded without a copy still view the map; it closes with them
            pass
        self.f.close()

    def read(self, addr: int, n: int, absolute: bool = False) -> bytes:
        a = addr if absolute else self.base + addr
        return self.buf[a:a + n]

    def _find_superblock(self) -> int:
        off = 0
        while off + 8 <= self.mm.size:
            if self.mm[off:off + 8].tobytes() == SIGNATURE:
                ver = int(self.mm[off + 8])
                if ver in (0, 1):
                    so, sl = int(self.mm[off + 13]), int(self.mm[off + 14])
                    if (so, sl) != (8, 8):
                        raise ValueError("only 8-byte offsets/lengths are supported")
                    # addresses are relative to the superblock (libhdf5 moves the base there)
                    p = off + 24 + (4 if ver == 1 else 0)
                    ent = self.mm[p + 32:p + 72].tobytes()        # root symbol-table entry
                    self.root_ohdr = struct.unpack("<Q", ent[8:16])[0]
                    return off
                if ver in (2, 3):
                    p = off + 12
                    self.root_ohdr = struct.unpack("<QQQQ", self.mm[p:p + 32].tobytes())[3]
                    return off
                raise ValueError(f"unsupported superblock version {ver}")
            off = 512 if off == 0 else off * 2
        raise ValueError("not an HDF5 file")

    # ------------------------------------------------------------------ object headers
    def messages(self, addr: int) -> list[tuple[int, bytes]]:
        head = self.read(addr, 16)
        out = []
        if head[:4] == b"OHDR":
            ver, flags = head[4], head[5]
            p = 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            sz_bytes = 1 << (flags & 3)
            hdr = self.read(addr, p + sz_bytes)
            chunk0 = int.from_bytes(hdr[p:p + sz_bytes], "little")
            start = addr + p + sz_bytes
            chunks = [(start, chunk0, True)]
            track = bool(flags & 0x04)
            while chunks:
                a, n, first = chunks.pop(0)
                buf = self.read(a, n)
                q = 0 if first else 4  # continuation chunks start with "OCHK"
                end = n - 4            # checksum
                while q + 4 <= end:
                    t = buf[q]
                    size = struct.unpack("<H", buf[q + 1:q + 3])[0]
                    q += 4 + (2 if track else 0)
                    body = buf[q:q + size]
                    q += size
                    if t == 0x10:
                        ca, cl = struct.unpack("<QQ", body[:16])
                        chunks.append((ca, cl, False))
                    elif t != 0:
                        out.append((t, body))
            return out
        ver, _, nmsg, _rc, size = struct.unpack("<BBHII", head[:12])
        if ver != 1:
            raise ValueError(f"unsupported object header version {ver}")
        chunks = [(addr + 16, size)]
        remaining = nmsg
        while chunks and remaining > 0:
            a, n = chunks.pop(0)
            buf = self.read(a, n)
            q = 0
            while q + 8 <= n and remaining > 0:
                t, size_m, _flags = struct.unpack("<HHB", buf[q:q + 5])
                body = buf[q + 8:q + 8 + size_m]
                q += 8 + size_m
                remaining -= 1
                if t == 0x10:
                    ca, cl = struct.unpack("<QQ", body[:16])
                    chunks.append((ca, cl))
                elif t != 0:
                    out.append((t, body))
        return out

    # ------------------------------------------------------------------ groups
    def group_links(self, addr: int) -> dict:
        links = {}
        for t, body in self.messages(addr):
            if t == 0x11:
                btree, heap = struct.unpack("<QQ", body[:16])
                hh = self.read(heap, 32)
                dsize, _free, daddr = struct.unpack("<QQQ", hh[8:32])
                heap_data = self.read(daddr, dsize)
                for name_off, obj in self._walk_group_btree(btree):
                    end = heap_data.index(b"\0", name_off)
                    links[heap_data[name_off:end].decode()] = obj
            elif t == 0x06:
                name, obj = self._link_message(body)
                if obj is not None:
                    links[name] = obj
            elif t == 0x02:
                p = 2 + (8 if body[1] & 1 else 0)
                if struct.unpack("<Q", body[p:p + 8])[0] != UNDEF:
                    raise NotImplementedError("dense (fractal-heap) link storage is not supported")
        return links

    def _walk_group_btree(self, addr):
        h = self.read(addr, 24)
        if h[:4] != b"TREE":
            raise ValueError("bad group B-tree node")
        level, used = h[5], struct.unpack("<H", h[6:8])[0]
        buf = self.read(addr + 24, 8 + used * 16)
        children = [struct.unpack("<Q", buf[8 + 16 * i:16 + 16 * i])[0] for i in range(used)]
        for c in children:
            if level > 0:
                yield from self._walk_group_btree(c)
            else:
                sh = self.read(c, 8)
                if sh[:4] != b"SNOD":
                    raise ValueError("bad symbol table node")
                n = struct.unpack("<H", sh[6:8])[0]
                ents = self.read(c + 8, 40 * n)
                for i in range(n):
                    name_off, obj = struct.unpack("<QQ", ents[40 * i:40 * i + 16])
                    yield name_off, obj

    @staticmethod
    def _link_message(body):
        ver, flags = body[0], body[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = body[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nlen_sz = 1 << (flags & 3)
        nlen = int.from_bytes(body[p:p + nlen_sz], "little")
        p += nlen_sz
        name = body[p:p + nlen].decode()
        p += nlen
        if ltype != 0:
            return name, None
        return name, struct.unpack("<Q", body[p:p + 8])[0]

    # ------------------------------------------------------------------ datasets
    @staticmethod
    def _dataspace(body):
        ver, rank = body[0], body[1]
        flags = body[2]
        if ver == 1:
            p = 8
        else:
            if body[3] == 2:  # null dataspace
                return None
            p = 4
        dims = struct.unpack(f"<{rank}Q", body[p:p + 8 * rank]) if rank else ()
        return tuple(dims)

    @staticmethod
    def _datatype(body):
        cls, ver = body[0] & 0x0F, body[0] >> 4
        bits = body[1:4]
        size = struct.unpack("<I", body[4:8])[0]
        if cls == 0:
            signed = bool(bits[0] & 0x08)
            order = ">" if bits[0] & 1 else "<"
            return np.dtype(f"{order}{'i' if signed else 'u'}{size}"), "int"
        if cls == 1:
            order = ">" if bits[0] & 1 else "<"
            return np.dtype(f"{order}f{size}"), "float"
        if cls == 3:
            return np.dtype(f"S{size}"), "string"
        if cls == 7:
            if bits[0] & 0x0F != 0:
                raise NotImplementedError("region references are not supported")
            return np.dtype("<u8"), "ref"
        if cls == 6:
            nmembers = struct.unpack("<H", bits[:2])[0]
            fields = []
            p = 8
            for _ in range(nmembers):
                end = body.index(b"\0", p)
                name = body[p:end].decode()
                # names are padded to a multiple of 8 bytes before version 3
                p = p + ((end - p + 8) // 8) * 8 if ver < 3 else end + 1
                if ver == 1:
                    off = struct.unpack("<I", body[p:p + 4])[0]
                    p += 4 + 1 + 3 + 4 + 4 + 16
                elif ver == 2:
                    off = struct.unpack("<I", body[p:p + 4])[0]
                    p += 4
                else:
                    nb = max(1, (size.bit_length() + 7) // 8)
                    off = int.from_bytes(body[p:p + nb], "little")
                    p += nb
                mdt, _ = _Reader._datatype(body[p:])
                p += _Reader._datatype_size(body[p:])
                fields.append((name, mdt, off))
            return np.dtype({"names": [f[0] for f in fields], "formats": [f[1] for f in fields],
                             "offsets": [f[2] for f in fields], "itemsize": size}), "compound"
        raise NotImplementedError(f"datatype class {cls}")

    @staticmethod
    def _datatype_size(body):
        cls = body[0] & 0x0F
        return 8 + {0: 4, 1: 12, 3: 0, 7: 0}.get(cls, 0) if cls != 6 else len(body)

    def _attributes(self, msgs) -> dict:
        attrs = {}
        for t, body in msgs:
            if t != 0x0C:
                continue
            ver = body[0]
            if ver == 1:
                nlen, dtlen, dslen = struct.unpack("<HHH", body[2:8])
                p = 8
                name = body[p:p + nlen].rstrip(b"\0").decode()
                p += nlen + (-nlen % 8)
                dtb = body[p:p + dtlen]
                p += dtlen + (-dtlen % 8)
                dsb = body[p:p + dslen]
                p += dslen + (-dslen % 8)
            else:
                nlen, dtlen, dslen = struct.unpack("<HHH", body[2:8])
                p = 8 + (1 if ver == 3 else 0)
                name = body[p:p + nlen].rstrip(b"\0").decode()
                p += nlen
                dtb = body[p:p + dtlen]
                p += dtlen
                dsb = body[p:p + dslen]
                p += dslen
            dt, kind = self._datatype(dtb)
            dims = self._dataspace(dsb)
            n = math.prod(dims) if dims else 1
            raw = body[p:p + n * dt.itemsize]
            val = np.frombuffer(raw, dtype=dt, count=n)
            if kind == "string":
                attrs[name] = val[0].split(b"\0")[0].decode() if n == 1 else [v.decode() for v in val]
            else:
                attrs[name] = val[0] if not dims else val.reshape(dims)
        return attrs

    def dataset(self, addr: int, msgs=None):
        if msgs is None:
            msgs = self.messages(addr)
        dims = dt = layout = None
        filters = []
        kind = None
        for t, body in msgs:
            if t == 0x01:
                dims = self._dataspace(body)
            elif t == 0x03:
                dt, kind = self._datatype(body)
            elif t == 0x08:
                layout = body
            elif t == 0x0B:
                filters = self._filters(body)
        attrs = self._attributes(msgs)
        if dims is None:
            return np.zeros(0, dtype=dt), attrs, kind
        n = math.prod(dims) if dims else 1
        raw = self._read_layout(layout, dims, dt, filters)
        arr = np.frombuffer(raw, dtype=dt, count=n).reshape(dims if dims else ())
        return arr, attrs, kind

    @staticmethod
    def _filters(body):
        ver, nf = body[0], body[1]
        p = 8 if ver == 1 else 2
        out = []
        for _ in range(nf):
            fid = struct.unpack("<H", body[p:p + 2])[0]
            if ver == 1 or fid >= 256:
                nlen = struct.unpack("<H", body[p + 2:p + 4])[0]
                flags, ncd = struct.unpack("<HH", body[p + 4:p + 8])
                p += 8 + nlen + (-nlen % 8 if ver == 1 else 0)
            else:
                flags, ncd = struct.unpack("<HH", body[p + 2:p + 6])
                p += 6
            cd = struct.unpack(f"<{ncd}I", body[p:p + 4 * ncd])
            p += 4 * ncd
            if ver == 1 and ncd % 2:
                p += 4
            out.append((fid, cd))
        return out

    def _read_layout(self, body, dims, dt, filters) -> bytes:
        ver = body[0]
        if ver not in (3, 4):
            raise NotImplementedError(f"data layout version {ver}")
        cls = body[1]
        nbytes = (math.prod(dims) if dims else 1) * dt.itemsize
        if cls == 0:
            size = struct.unpack("<H", body[2:4])[0]
            return body[4:4 + size]
        if cls == 1:
            addr, size = struct.unpack("<QQ", body[2:18])
            if addr == UNDEF:
                return bytes(nbytes)
            return self.read(addr, size)
        if cls == 2 and ver == 3:
            ndims = body[2]
            btree = struct.unpack("<Q", body[3:11])[0]
            cdims = struct.unpack(f"<{ndims}I", body[11:11 + 4 * ndims])
            chunk = cdims[:-1]
            out = np.zeros(dims, dtype=np.dtype(f"V{dt.itemsize}")) if dims else None
            if btree == UNDEF:
                return bytes(nbytes)
            for offs, caddr, csize, fmask in self._walk_chunk_btree(btree, ndims):
                raw = self.read(caddr, csize)
                raw = self._unfilter(raw, filters, fmask, dt.itemsize)
                block = np.frombuffer(raw, dtype=out.dtype, count=math.prod(chunk)).reshape(chunk)
                sl = tuple(slice(o, min(o + c, d)) for o, c, d in zip(offs, chunk, dims))
                out[sl] = block[tuple(slice(0, s.stop - s.start) for s in sl)]
            return out.tobytes()
        raise NotImplementedError(f"layout class {cls} (version {ver})")

    def _walk_chunk_btree(self, addr, ndims):
        h = self.read(addr, 24)
        if h[:4] != b"TREE" or h[4] != 1:
            raise ValueError("bad chunk B-tree node")
        level, used = h[5], struct.unpack("<H", h[6:8])[0]
        ksize = 8 + 8 * ndims
        buf = self.read(addr + 24, (used + 1) * ksize + used * 8)
        p = 0
        for _ in range(used):
            csize, fmask = struct.unpack("<II", buf[p:p + 8])
            offs = struct.unpack(f"<{ndims}Q", buf[p + 8:p + ksize])[:-1]
            child = struct.unpack("<Q", buf[p + ksize:p + ksize + 8])[0]
            p += ksize + 8
            if level > 0:
                yield from self._walk_chunk_btree(child, ndims)
            else:
                yield offs, child, csize, fmask

    @staticmethod
    def _unfilter(raw, filters, fmask, itemsize):
        for i, (fid, cd) in reversed(list(enumerate(filters))):
            if fmask & (1 << i):
                continue
            if fid == 1:
                raw = zlib.decompress(raw)
            elif fid == 2:
                a = np.frombuffer(raw, dtype=np.uint8)
                n = a.size // itemsize
                raw = a[: n * itemsize].reshape(itemsize, n).T.tobytes() + a[n * itemsize:].tobytes()
            elif fid == 3:
                raw = raw[:-4]
            else:
                raise NotImplementedError(f"HDF5 filter {fid}")
        return raw

    def is_group(self, addr: int, msgs=None) -> bool:
        return any(t in (0x11, 0x06, 0x02) for t, _ in (self.messages(addr) if msgs is None else msgs))


def _decode(r: _Reader, addr: int):
    """An HDF5 object in MATLAB terms."""
    msgs = r.messages(addr)  # parsed once for both checks
    if r.is_group(addr, msgs):
        # MATLAB struct: a group whose members are the fields
        return {name: _decode(r, a) for name, a in r.group_links(addr).items() if not name.startswith("#")}
    arr, attrs, kind = r.dataset(addr, msgs)
    cls = attrs.get("MATLAB_class", None)
    if isinstance(cls, bytes):
        cls = cls.decode()
    if attrs.get("MATLAB_empty", 0):
        mshape = tuple(int(x) for x in np.asarray(arr).ravel())
        if cls == "char":
            return ""
        if cls == "cell":
            return np.empty(mshape, dtype=object)
        return np.zeros(mshape, dtype=_CLASS_DTYPE.get(cls, np.float64) if cls != "logical" else bool)
    mshape = tuple(reversed(arr.shape))
    if kind == "ref":
        flat = arr.ravel()                       # C order over HDF5 dims == MATLAB column-major
        cells = np.empty(flat.size, dtype=object)
        for i, c in enumerate(_decode_cells(r, flat.astype(np.int64))):
            cells[i] = c
        return cells.reshape(mshape, order="F")
    if kind == "compound":
        names = arr.dtype.names
        if names and set(names) >= {"real", "imag"}:
            arr = arr["real"] + 1j * arr["imag"]
        else:
            raise NotImplementedError("compound dataset that is not a MATLAB complex array")
    out = np.asarray(arr).T.astype(arr.dtype.newbyteorder("="), copy=False)   # MATLAB shape
    if cls == "char":
        rows = ["".join(chr(c) for c in row) for row in np.atleast_2d(out).astype(np.uint32)]
        return rows[0] if len(rows) == 1 else rows
    if cls == "logical":
        return out.astype(bool)
    return out


# ------------------------------------------------------------------ batched cells
@dataclass
class _CellTemplate:
    """One cell's v1 object header as a byte pattern: the cells of a cell array written by one
    writer differ only in their dims and data address / size (MATLAB and savemat73 alike), so the
    others are matched against it in bulk instead of parsed one by one.  ``fixed`` marks the bytes
    that must be equal; ``dims`` / ``layout`` are the offsets of the dataspace dims and of the
    contiguous layout's address and size in the header."""
    raw: np.ndarray
    fixed: np.ndarray
    dims: int
    rank: int
    layout: int
    dtype: np.dtype
    cls: str
    empty: bool


_FAST_CLASSES = set(_CLASS_DTYPE) | {"logical"}


def _cell_template(r: _Reader, addr: int) -> _CellTemplate | None:
    """The byte pattern of the cell at ``addr``, or None for headers the bulk path does not
    take (v2 headers, continuations, non-contiguous data, char / cell / struct cells)."""
    head = r.read(addr, 16)
    if len(head) < 16 or head[:4] == b"OHDR" or head[0] != 1:
        return None
    nmsg, size = struct.unpack("<HxxxxI", head[2:12])
    span = 16 + size
    if span > 4096 or addr + span + r.base > len(r.buf):
        return None
    raw = r.read(addr, span)
    var = np.zeros(span, dtype=bool)
    dims = layout = None
    q = 16
    for _ in range(nmsg):
        if q + 8 > span:
            return None
        t, sz = struct.unpack("<HH", raw[q:q + 4])
        b = q + 8
        if t == 0x10:
            return None
        if t == 0x01:
            ver, rank, flags = raw[b], raw[b + 1], raw[b + 2]
            if ver == 2 and raw[b + 3] != 1:
                return None
            p = b + (8 if ver == 1 else 4)
            dims = (p, rank)
            var[p:p + 16 * rank if flags & 1 else p + 8 * rank] = True
        elif t == 0x08:
            if raw[b] not in (3, 4) or raw[b + 1] != 1:
                return None
            layout = b + 2
            var[b + 2:b + 18] = True
        elif t in (0x0E, 0x12):   # modification times (libhdf5 tracks them per object by default)
            var[b:b + sz] = True
        q = b + sz
    if dims is None or layout is None or q > span:
        return None
    msgs = r.messages(addr)
    attrs = r._attributes(msgs)
    cls = attrs.get("MATLAB_class", None)
    cls = cls.decode() if isinstance(cls, bytes) else cls
    if cls not in _FAST_CLASSES:
        return None
    empty = bool(attrs.get("MATLAB_empty", 0))
    dt = None
    for t, body in msgs:
        if t == 0x03:
            dt, kind = r._datatype(body)
            if kind not in ("int", "float"):
                return None
    if dt is None:
        return None
    return _CellTemplate(np.frombuffer(raw, dtype=np.uint8), ~var, dims[0], dims[1], layout, dt, cls, empty)


def _match_cells(r: _Reader, tpl: _CellTemplate, addrs: np.ndarray):
    """Which of ``addrs`` have ``tpl``'s header (every fixed byte equal, data contiguous, in the
    file and of the size its dims give); for those, their HDF5 dims and data addresses / sizes."""
    span = tpl.raw.size
    a = addrs.astype(np.int64) + r.base
    inb = (a >= 0) & (a + span <= len(r.buf))
    ok = np.zeros(addrs.size, dtype=bool)
    dims = np.zeros((addrs.size, tpl.rank), dtype=np.uint64)
    dadr = np.zeros(addrs.size, dtype=np.uint64)
    dsz = np.zeros(addrs.size, dtype=np.uint64)
    sel = np.flatnonzero(inb)
    al = int(a[sel[0]]) % 8 if sel.size else 0
    if span % 8 == 0 and sel.size and np.all(a[sel] % 8 == al):
        # 8-byte aligned headers (v1 header messages are): gather words, not bytes
        words = np.frombuffer(r.buf, dtype="<u8", offset=al, count=(len(r.buf) - al) // 8)
        gather = lambda part: words[((a[part] - al) // 8)[:, None] + np.arange(span // 8)].view(np.uint8)
    else:
        gather = lambda part: r.mm[a[part][:, None] + np.arange(span)]
    for s0 in range(0, sel.size, 1 << 15):
        part = sel[s0:s0 + (1 << 15)]
        h = gather(part)
        good = ~np.any(h[:, tpl.fixed] != tpl.raw[tpl.fixed], axis=1)
        d = np.ascontiguousarray(h[:, tpl.dims:tpl.dims + 8 * tpl.rank]).view("<u8")
        lay = np.ascontiguousarray(h[:, tpl.layout:tpl.layout + 16]).view("<u8")
        ok[part], dims[part], dadr[part], dsz[part] = good, d, lay[:, 0], lay[:, 1]
    nel = np.prod(dims, axis=1, dtype=np.uint64) if tpl.rank else np.ones(addrs.size, np.uint64)
    ok &= (dadr != UNDEF) & (dsz == nel * np.uint64(tpl.dtype.itemsize)) & (nel > 0)
    ok &= dadr.astype(np.float64) + dsz.astype(np.float64) + r.base <= len(r.buf)
    return ok, dims, dadr.astype(np.int64) + r.base, dsz.astype(np.int64)


def _bulk_cells(r: _Reader, addrs: np.ndarray):
    """Yield (indices, template, dims, data addresses, sizes) for the cells of ``addrs`` that
    match a template taken from the first cell not yet matched (at most 8 tries), and finally
    (indices, None, ...) for the rest, which are decoded one by one."""
    rest = np.arange(addrs.size)
    single = []
    for _ in range(8):
        if rest.size == 0:
            break
        tpl = _cell_template(r, int(addrs[rest[0]]))
        ok = _match_cells(r, tpl, addrs[rest]) if tpl is not None else None
        if ok is None or not ok[0][0]:
            single.append(int(rest[0]))
            rest = rest[1:]
            continue
        good, dims, dadr, dsz = ok
        yield rest[good], tpl, dims[good], dadr[good], dsz[good]
        rest = rest[~good]
    if single or rest.size:
        yield np.concatenate([np.asarray(single, dtype=np.int64), rest]), None, None, None, None


def _decode_cells(r: _Reader, addrs: np.ndarray) -> list:
    """``[_decode(r, a) for a in addrs]``, with numeric / logical cells read in bulk."""
    out = [None] * addrs.size
    buf = r.buf
    for idx, tpl, dims, dadr, dsz in _bulk_cells(r, addrs):
        if tpl is None:
            for i in idx.tolist():
                out[i] = _decode(r, int(addrs[i]))
            continue
        dt, native = tpl.dtype, tpl.dtype.newbyteorder("=")
        if tpl.empty:
            zdt = bool if tpl.cls == "logical" else _CLASS_DTYPE[tpl.cls]
            for i, a, n in zip(idx.tolist(), dadr.tolist(), dsz.tolist()):
                raw = np.frombuffer(buf[a:a + n], dtype=dt)
                out[i] = np.zeros(tuple(int(x) for x in raw), dtype=zdt)
            continue
        logical = tpl.cls == "logical"
        for i, d, a, n in zip(idx.tolist(), dims.tolist(), dadr.tolist(), dsz.tolist()):
            x = np.frombuffer(buf[a:a + n], dtype=dt).reshape(d).T.astype(native, copy=False)
            out[i] = x.astype(bool) if logical else x
    return out


class MatFile:
    """Random access to a v7.3 file: ``names()``, ``load(name)`` and ``cell_elements(name,
    indices)``, which decodes only the selected cells of a cell array (preloaded_qsos.mat at full
    DR12Q holds 4 x 162,861 cells; a process working on one shard needs its own)."""

    def __init__(self, path: str):
        self._r = _Reader(path)
        self._links = self._r.group_links(self._r.root_ohdr)

    def names(self):
        return [n for n in self._links if not n.startswith("#")]

    def load(self, name: str):
        return _decode(self._r, self._links[name])

    def cell_elements(self, name: str, indices) -> list:
        arr, attrs, kind = self._r.dataset(self._links[name])
        if kind != "ref":
            raise TypeError(f"{name} is not a cell array")
        flat = arr.ravel()                  # MATLAB column-major order
        return _decode_cells(self._r, flat[np.asarray(indices, dtype=np.int64)].astype(np.int64))

    def cell_vectors(self, name: str, indices, dtype) -> tuple[np.ndarray, np.ndarray]:
        """The selected cells of a cell array of vectors, ravelled and concatenated in ``dtype``:
        (values, per-cell lengths) -- ``np.concatenate([c.ravel() for c in cell_elements(...)])``
        without a Python object per cell where the cells match a header template (logical cells
        come back as 0 / 1).  A matrix cell is ravelled in MATLAB (column-major) order.  Cells
        that follow each other in the selection and in the file (writers lay a cell array's data
        out in order, at most a few alignment bytes apart) are copied as one run."""
        arr, _, kind = self._r.dataset(self._links[name])
        if kind != "ref":
            raise TypeError(f"{name} is not a cell array")
        addrs = arr.ravel()[np.asarray(indices, dtype=np.int64)].astype(np.int64)
        dtype = np.dtype(dtype)
        lengths = np.zeros(addrs.size, dtype=np.int64)
        slow, groups = {}, []
        for idx, tpl, dims, dadr, dsz in _bulk_cells(self._r, addrs):
            if tpl is None or tpl.empty:
                for i in idx.tolist():
                    c = np.asarray(_decode(self._r, int(addrs[i])))
                    if c.dtype.kind not in "biuf":
                        raise TypeError(f"{name}: cell {i} is not a real numeric or logical array")
                    slow[i] = c.ravel(order="F")
                    lengths[i] = slow[i].size
            else:
                lengths[idx] = dsz // tpl.dtype.itemsize
                groups.append((idx, tpl, dadr, dsz))
        offs = np.zeros(addrs.size + 1, dtype=np.int64)
        np.cumsum(lengths, out=offs[1:])
        vals = np.empty(int(offs[-1]), dtype=dtype)
        for i, c in slow.items():
            vals[offs[i]:offs[i + 1]] = c
        for idx, tpl, dadr, dsz in groups:
            self._copy_runs(vals, offs, idx, tpl, dadr, dsz)
        return vals, lengths

    def _copy_runs(self, vals, offs, idx, tpl, dadr, dsz):
        """vals[offs[i]:offs[i+1]] = cell i's data for the cells ``idx`` of one template, one
        numpy copy per run of cells adjacent in the selection and in the file."""
        src, logical = tpl.dtype, tpl.cls == "logical"
        end = dadr + dsz
        gap = dadr[1:] - end[:-1]
        brk = np.flatnonzero((idx[1:] != idx[:-1] + 1) | (gap < 0) | (gap >= 64)) + 1
        starts = np.concatenate([[0], brk]).tolist()
        stops = np.concatenate([brk, [idx.size]]).tolist()
        u8 = self._r.mm
        direct = not logical and src == vals.dtype
        for j0, j1 in zip(starts, stops):
            lo, hi = int(dadr[j0]), int(end[j1 - 1])
            o0, o1 = int(offs[idx[j0]]), int(offs[idx[j1 - 1] + 1])
            if direct and hi - lo == (o1 - o0) * src.itemsize:
                # one read straight into the output (no faults on the file map)
                if os.preadv(self._r.f.fileno(), [vals[o0:o1].view(np.uint8)], lo) != hi - lo:
                    raise ValueError(f"{self._r.f.name}: short read at {lo}")
                continue
            span = u8[lo:hi]                                  # a view of the file map
            if hi - lo != int(dsz[j0:j1].sum()):              # alignment gaps between the cells
                runs = np.empty(2 * (j1 - j0) - 1, dtype=np.int64)
                runs[0::2], runs[1::2] = dsz[j0:j1], gap[j0:j1 - 1]
                keep = np.repeat(np.arange(runs.size) % 2 == 0, runs)
                span = span[keep]
            x = span.view(src)
            vals[o0:o1] = x != 0 if logical else x

    def cell_count(self, name: str) -> int:
        arr, _, kind = self._r.dataset(self._links[name])
        return int(arr.size)

    def close(self):
        self._r.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class LazyMat(dict):
    """``loadmat73(path)`` that decodes each variable on first access: a dict whose ``[]``,
    ``get`` and ``in`` see every variable of the file, while iteration, ``len`` and ``items``
    decode the rest first.  ``close()`` (or a ``with`` block) releases the file; values decoded
    by then stay valid."""

    def __init__(self, path: str):
        super().__init__()
        self._mf = MatFile(path)
        self._names = [n for n in self._mf.names()]

    def __missing__(self, key):
        if self._mf is None or key not in self._names:
            raise KeyError(key)
        val = self._mf.load(key)
        self[key] = val
        return val

    def __contains__(self, key):
        return dict.__contains__(self, key) or key in self._names

    def get(self, key, default=None):
        return self[key] if key in self else default

    def _load_all(self):
        for n in self._names:
            if not dict.__contains__(self, n):
                self[n]                                            # noqa: B018 (decodes it)

    def keys(self):
        self._load_all()
        return super().keys()

    def values(self):
        self._load_all()
        return super().values()

    def items(self):
        self._load_all()
        return super().items()

    def __iter__(self):
        self._load_all()
        return super().__iter__()

    def __len__(self):
        self._load_all()
        return super().__len__()

    def close(self):
        if self._mf is not None:
            self._mf.close()
            self._mf = None
            self._names = [n for n in self._names if dict.__contains__(self, n)]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def loadmat73(path: str, variable_names=None) -> dict:
    """Read a MATLAB v7.3 file into {name: value} with MATLAB shapes (a Q x 1 vector comes back
    as a (Q, 1) array; ``squeeze`` it as scipy's ``squeeze_me`` would)."""
    r = _Reader(path)
    try:
        links = r.group_links(r.root_ohdr)
        out = {}
        for name, addr in links.items():
            if name.startswith("#"):
                continue
            if variable_names is not None and name not in variable_names:
                continue
            out[name] = _decode(r, addr)
        return out
    finally:
        r.close()


_KNOWN_CLASSES = set(_MATLAB_CLASS.values()) | {"char", "logical", "cell", "struct", "double"}


def rewrite_blockers(path: str) -> list[str]:
    """Why a load + ``savemat73`` round trip of this v7.3 file would lose data: MATLAB objects
    (``containers.Map`` and other MCOS classes are stored as opaque uint32 handles into the
    ``#subsystem#`` group, which this reader does not decode) or classes it does not know.
    Empty if every top-level variable decodes to what was written."""
    r = _Reader(path)
    try:
        links = r.group_links(r.root_ohdr)
        out = []
        if "#subsystem#" in links:
            out.append("#subsystem# group (MATLAB objects)")
        for name, addr in links.items():
            if name.startswith("#") or r.is_group(addr):
                continue
            attrs = r._attributes(r.messages(addr))
            cls = attrs.get("MATLAB_class")
            cls = cls.decode() if isinstance(cls, bytes) else cls
            if "MATLAB_object_decode" in attrs or (cls is not None and cls not in _KNOWN_CLASSES):
                out.append(f"{name}: MATLAB_class {cls!r}")
        return out
    finally:
        r.close()


def update_variable(path: str, name: str, value) -> bool:
    """``save(path, name, '-append')`` for a numeric variable that already exists with the same
    class and element count in contiguous, unfiltered storage: the new values are written over
    the old bytes in place and nothing else in the file changes.  Returns False (file untouched)
    when that is not possible."""
    r = _Reader(path)
    try:
        links = r.group_links(r.root_ohdr)
        if name not in links or r.is_group(links[name]):
            return False
        msgs = r.messages(links[name])
        dims = dt = layout = None
        for t, body in msgs:
            if t == 0x01:
                dims = r._dataspace(body)
            elif t == 0x03:
                dt, kind = r._datatype(body)
                if kind not in ("int", "float"):
                    return False
            elif t == 0x08:
                layout = body
            elif t == 0x0B:
                return False                      # filtered (compressed) storage
        if layout is None or dims is None or dt is None or layout[0] not in (3, 4) or layout[1] != 1:
            return False
        addr, size = struct.unpack("<QQ", layout[2:18])
        val = np.asarray(value)
        n = math.prod(dims) if dims else 1
        if addr == UNDEF or val.size != n or size != n * dt.itemsize:
            return False
        # the MATLAB shape must match the stored one (a 1-D value is a Q x 1 column, like savemat73's
        # vectors): a same-size value of another shape would land in the wrong column-major order
        mshape = val.shape if val.ndim >= 2 else ((val.size, 1) if val.ndim == 1 else (1, 1))
        if tuple(int(d) for d in reversed(mshape)) != tuple(int(d) for d in dims):
            return False
        conv = val.astype(dt.newbyteorder("="))
        if not np.array_equal(conv, val):         # would not survive the class conversion
            return False
        off = r.base + addr
    finally:
        r.close()
    mm = np.memmap(path, dtype=dt, mode="r+", offset=off, shape=(n,))
    mm[:] = conv.ravel(order="F")                 # MATLAB column-major == C order over HDF5 dims
    mm.flush()
    del mm
    return True


def is_matv73(path: str) -> bool:
    with open(path, "rb") as f:
        head = f.read(128)
        if len(head) < 128:
            return False
        f.seek(USERBLOCK)
        return head[124:126] == struct.pack("<H", 0x0200) and f.read(8) == SIGNATURE


def loadmat(path: str, variable_names=None) -> dict:
    """``load`` for either MATLAB format: v7.3 via this module, v5/v7 via scipy."""
    if is_matv73(path):
        return loadmat73(path, variable_names)
    from scipy.io import loadmat as _lm
    d = _lm(path, variable_names=variable_names)
    return {k: v for k, v in d.items() if not k.startswith("__")}


__all__ = ["LazyArray", "Region", "MatFile", "savemat73", "open_region", "loadmat73", "loadmat", "is_matv73",
           "update_variable", "rewrite_blockers"]
