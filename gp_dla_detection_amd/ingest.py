"""Spectrum ingest: read_spec.m and preload_qsos.m.

``read_spec_columns`` loads an SDSS DR12Q coadded "speclite" FITS file -- binary-table HDU 1,
columns 1-4 = flux, loglam, ivar, and_mask (read_spec.m:11-25) -- on the host: the FITS reader is a
numpy implementation of the binary-table subset these files use (no astropy on the GPU box).
Everything numeric runs on the GPU (csrc/ingest.hip): ``read_spec`` derives wavelengths, noise
variance and the bad-pixel mask (read_spec.m:27-38, ``gpdla_read_spec_f32``); ``preload_qsos``
sends a batch of catalogue spectra as one CSR of their fitsread columns, and the device applies
read_spec's rules, normalises each spectrum by its median flux in the 1310-1325 A rest window,
sets the filter-flag bits and keeps the 910-1217 A rest range plus one unmasked pixel on either
side (preload_qsos.m:18-67, ``gpdla_preload_qsos_f32``), producing the cells process_qsos reads
(preloaded_qsos.mat).

MATLAB's fitsread returns an 'E' column as single precision, and read_spec / preload_qsos keep
computing in single (10.^loglam, 1./ivar, the normalisation); the device does the same (float32
arithmetic, float32 cells, widened to float64 only when packed for the engine), with 10.^loglam
correctly rounded to single.  There is no CPU path: without a HIP device the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib as L
from . import parameters as P

BRIGHTSKY = 24  # read_spec.m:9 (1-based bit of the and_mask)

_TFORM = {"L": ("i1", 1), "X": ("u1", 1), "B": ("u1", 1), "I": (">i2", 2), "J": (">i4", 4),
          "K": (">i8", 8), "A": ("S1", 1), "E": (">f4", 4), "D": (">f8", 8)}


def _cards(block: bytes):
    for i in range(0, len(block), 80):
        card = block[i:i + 80].decode("ascii", errors="replace")
        key = card[:8].strip()
        if card[8:10] == "= ":
            val = card[10:].split("/")[0].strip() if not card[10:].strip().startswith("'") else card[10:]
            yield key, val
        else:
            yield key, None


def _value(v: str):
    v = v.strip()
    if v.startswith("'"):
        end = v.find("'", 1)
        while end != -1 and end + 1 < len(v) and v[end + 1] == "'":   # '' escapes a quote
            end = v.find("'", end + 2)
        return v[1:end].replace("''", "'").rstrip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        return float(v.replace("D", "E"))


def _read_header(f):
    hdr = {}
    while True:
        block = f.read(2880)
        if len(block) < 2880:
            raise ValueError("truncated FITS header")
        done = False
        for key, val in _cards(block):
            if key == "END":
                done = True
                break
            if val is not None and key:
                hdr[key] = _value(val)
        if done:
            return hdr


def _data_bytes(hdr) -> int:
    naxis = hdr.get("NAXIS", 0)
    if naxis == 0:
        return 0
    n = 1
    for i in range(1, naxis + 1):
        n *= hdr[f"NAXIS{i}"]
    return abs(hdr["BITPIX"]) // 8 * hdr.get("GCOUNT", 1) * (hdr.get("PCOUNT", 0) + n)


def read_bintable(path: str, hdu: int = 1, columns=None) -> list:
    """fitsread(path, 'binarytable', hdu, 'tablecolumns', columns): a list of column arrays
    (1-based column numbers; scalar columns as 1-D arrays, vector columns as (rows, repeat)).
    TSCAL/TZERO are applied; 'E' stays float32 and 'D' float64 like MATLAB's single/double."""
    with open(path, "rb") as f:
        for _ in range(hdu):
            hdr = _read_header(f)
            nbytes = _data_bytes(hdr)
            f.seek(nbytes + (-nbytes % 2880), os.SEEK_CUR)
        hdr = _read_header(f)
        if hdr.get("XTENSION") != "BINTABLE":
            raise ValueError(f"HDU {hdu} of {path} is not a binary table")
        row_bytes, nrows, nfields = hdr["NAXIS1"], hdr["NAXIS2"], hdr["TFIELDS"]
        raw = np.frombuffer(f.read(row_bytes * nrows), dtype=np.uint8)
    if raw.size < row_bytes * nrows:
        raise ValueError("truncated FITS table")
    raw = raw.reshape(nrows, row_bytes)
    cols, off = [], 0
    for j in range(1, nfields + 1):
        tform = str(hdr[f"TFORM{j}"]).strip()
        i = 0
        while i < len(tform) and tform[i].isdigit():
            i += 1
        repeat = int(tform[:i]) if i else 1
        code = tform[i]
        if code not in _TFORM:
            raise NotImplementedError(f"TFORM {tform}")
        dt, size = _TFORM[code]
        width = repeat * size if code != "X" else (repeat + 7) // 8
        cols.append((j, code, dt, repeat, off, width))
        off += width
    want = range(1, nfields + 1) if columns is None else columns
    out = []
    for j in want:
        _, code, dt, repeat, o, width = cols[j - 1]
        block = np.ascontiguousarray(raw[:, o:o + width])
        if code == "A":
            arr = block.view(f"S{width}").ravel()
        elif code == "X":
            arr = np.unpackbits(block, axis=1)[:, :repeat].astype(bool)
        else:
            arr = block.view(dt).reshape(nrows, repeat) if repeat != 1 else block.view(dt).ravel()
            arr = arr.astype(np.dtype(dt).newbyteorder("="))
            if code == "L":
                arr = arr == ord("T")
            scale, zero = hdr.get(f"TSCAL{j}", 1), hdr.get(f"TZERO{j}", 0)
            if (scale, zero) != (1, 0):
                if code in "BIJK" and scale == 1 and float(zero).is_integer():
                    arr = arr.astype(np.int64) + int(zero)    # unsigned-int convention
                else:
                    arr = arr * scale + zero
        out.append(arr)
    return out


def read_spec_columns(filename: str):
    """fitsread(filename, 'binarytable', 1, 'tablecolumns', 1:4) (read_spec.m:11-25): flux, loglam and
    ivar as single, and_mask as int32 (host)."""
    flux, log_wavelengths, ivar, and_mask = read_bintable(filename, 1, [1, 2, 3, 4])
    return (np.ascontiguousarray(flux, dtype=np.float32), np.ascontiguousarray(log_wavelengths, dtype=np.float32),
            np.ascontiguousarray(ivar, dtype=np.float32), np.ascontiguousarray(and_mask, dtype=np.int32))


def read_spec(filename: str, device: int = 0):
    """[wavelengths, flux, noise_variance, pixel_mask] = read_spec(filename) (read_spec.m): the columns
    read on the host, read_spec.m:27-38 on the device."""
    flux, loglam, ivar, and_mask = read_spec_columns(filename)
    n = flux.size
    w, nv, pm = np.empty(n, np.float32), np.empty(n, np.float32), np.empty(n, np.uint8)
    L.check(L.load().gpdla_read_spec_f32(device, n, L.ptr(loglam, C.c_float), L.ptr(ivar, C.c_float),
                                         L.ptr(and_mask, C.c_int32), L.ptr(w, C.c_float), L.ptr(nv, C.c_float),
                                         L.ptr(pm, C.c_uint8)))
    return w, flux, nv, pm.astype(bool)


def preload_params() -> "L.PreloadParams":
    """set_parameters.m:21-30's ingest constants and read_spec.m:9's BRIGHTSKY bit."""
    return L.PreloadParams(P.NORMALIZATION_MIN_LAMBDA, P.NORMALIZATION_MAX_LAMBDA, P.MIN_LAMBDA, P.MAX_LAMBDA,
                           P.LOADING_MIN_LAMBDA, P.LOADING_MAX_LAMBDA, P.MIN_NUM_PIXELS, BRIGHTSKY)


def preload_batch(z_qsos, filter_flags, columns, device: int = 0) -> dict:
    """preload_qsos.m:18-67 for one batch on the device.  ``columns[i]``: spectrum i's fitsread columns
    (flux, loglam, ivar, and_mask), or None where filter_flags[i] > 0 (not read, :19-21).  Returns the
    cells (lists of single / logical arrays), normalisers, updated flags and the single medians."""
    z = np.ascontiguousarray(z_qsos, dtype=np.float64)
    flags = np.array(filter_flags, dtype=np.uint8).ravel().copy()
    Q = z.size
    lens = np.array([0 if c is None else np.asarray(c[0]).size for c in columns], dtype=np.int64)
    off = np.zeros(Q + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    N = int(off[-1])
    cat = lambda k, dt: (np.concatenate([np.asarray(c[k], dt) for c in columns if c is not None])   # noqa: E731
                         if N else np.zeros(1, dt))
    fl, ll, iv, am = cat(0, np.float32), cat(1, np.float32), cat(2, np.float32), cat(3, np.int32)
    cap = max(N, 1)
    ooff = np.zeros(Q + 1, np.int64)
    w_o, f_o, nv_o = np.empty(cap, np.float32), np.empty(cap, np.float32), np.empty(cap, np.float32)
    m_o = np.empty(cap, np.uint8)
    norm, med = np.zeros(Q), np.empty(Q, np.float32)
    params = preload_params()
    L.check(L.load().gpdla_preload_qsos_f32(device, Q, L.ptr(off, C.c_int64), L.ptr(fl, C.c_float),
                                            L.ptr(ll, C.c_float), L.ptr(iv, C.c_float), L.ptr(am, C.c_int32),
                                            L.ptr(z), C.byref(params), L.ptr(flags, C.c_uint8),
                                            L.ptr(ooff, C.c_int64), L.ptr(w_o, C.c_float), L.ptr(f_o, C.c_float),
                                            L.ptr(nv_o, C.c_float), L.ptr(m_o, C.c_uint8), L.ptr(norm),
                                            L.ptr(med, C.c_float)))
    cells = lambda a: [a[ooff[i]:ooff[i + 1]].copy() for i in range(Q)]   # noqa: E731
    return dict(all_wavelengths=cells(w_o), all_flux=cells(f_o), all_noise_variance=cells(nv_o),
                all_pixel_mask=[c.astype(bool) for c in cells(m_o)], all_normalizers=norm, filter_flags=flags,
                medians=med)


def spec_filename(spectra_directory: str, plate: int, mjd: int, fiber_id: int) -> str:
    """The DR12Q layout file_loader reads: <spectra>/<plate>/spec-<plate>-<mjd>-<fiber>.fits."""
    return f"{spectra_directory}/{int(plate)}/spec-{int(plate)}-{int(mjd)}-{int(fiber_id):04d}.fits"


def preload_qsos(z_qsos, plates, mjds, fiber_ids, filter_flags, file_loader, log=None, device: int = 0,
                 batch: int = 8192) -> dict:
    """preload_qsos.m:10-71.  ``file_loader(plate, mjd, fiber_id)`` returns the spectrum's fitsread
    columns (flux, loglam, ivar, and_mask; ``read_spec_columns``): the files are read on the host, and
    read_spec.m:27-38 with preload_qsos.m:26-67 run on the device, ``batch`` spectra per launch.
    Returns the saved variables (cells as lists, filter_flags updated with bits 3 and 4)."""
    z_qsos = np.asarray(z_qsos, dtype=np.float64).ravel()
    filter_flags = np.array(filter_flags, dtype=np.uint8).ravel().copy()
    Q = z_qsos.size
    keys = ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask")
    out = {k: [] for k in keys}
    all_normalizers = np.zeros(Q)
    for b0 in range(0, Q, batch):
        sl = slice(b0, min(Q, b0 + batch))
        cols = [None if filter_flags[i] > 0 else file_loader(plates[i], mjds[i], fiber_ids[i])   # :19-24
                for i in range(sl.start, sl.stop)]
        res = preload_batch(z_qsos[sl], filter_flags[sl], cols, device=device)
        for k in keys:
            out[k].extend(res[k])
        all_normalizers[sl] = res["all_normalizers"]
        filter_flags[sl] = res["filter_flags"]
        if log:
            for i in range(sl.start, sl.stop):
                if res["all_wavelengths"][i - sl.start].size:
                    log(f"loaded quasar {i + 1} of {Q} ({plates[i]}/{mjds[i]}/{int(fiber_ids[i]):04d})")
    return dict(loading_min_lambda=P.LOADING_MIN_LAMBDA, loading_max_lambda=P.LOADING_MAX_LAMBDA,
                normalization_min_lambda=P.NORMALIZATION_MIN_LAMBDA,
                normalization_max_lambda=P.NORMALIZATION_MAX_LAMBDA, min_num_pixels=P.MIN_NUM_PIXELS,
                **out, all_normalizers=all_normalizers, filter_flags=filter_flags)


def run_preload_qsos(base_directory: str, release: str) -> dict:
    """The script on files: catalog.mat (z_qsos, plates, mjds, fiber_ids, filter_flags) and the
    spectra under <base>/<release>/spectra -> preloaded_qsos.mat; filter_flags saved back into
    catalog.mat with ``'-append'`` (preload_qsos.m:77-83), i.e. only that variable changes.

    The existing filter_flags dataset is overwritten in place when its storage allows it
    (matv73.update_variable).  Otherwise catalog.mat is rewritten only if a load + save round trip
    is lossless (no MATLAB objects such as the containers.Map variables build_catalogs.m writes,
    no classes the reader does not know); if it is not, catalog.mat is left untouched, the flags
    go to ``catalog_filter_flags.mat`` beside it and a warning names the file."""
    import warnings

    from .matv73 import loadmat, rewrite_blockers, savemat73, update_variable
    from .process import processed_directory
    d = processed_directory(base_directory, release)
    cat = loadmat(f"{d}/catalog.mat")
    spectra_dir = f"{base_directory}/{release}/spectra"
    out = preload_qsos(np.ravel(cat["z_qsos"]), np.ravel(cat["plates"]), np.ravel(cat["mjds"]),
                       np.ravel(cat["fiber_ids"]), np.ravel(cat["filter_flags"]),
                       lambda p, m, f: read_spec_columns(spec_filename(spectra_dir, p, m, f)))
    flags = out.pop("filter_flags")
    savemat73(f"{d}/preloaded_qsos.mat", {k: (np.float64(v) if np.isscalar(v) else v) for k, v in out.items()})
    cpath = f"{d}/catalog.mat"
    out["filter_flags"] = flags
    out["filter_flags_path"] = cpath
    if update_variable(cpath, "filter_flags", flags):                                    # '-append'
        return out
    blockers = rewrite_blockers(cpath)
    if not blockers:
        cat["filter_flags"] = flags.reshape(-1, 1)
        savemat73(cpath, cat)
        return out
    side = f"{d}/catalog_filter_flags.mat"
    savemat73(side, {"filter_flags": flags.reshape(-1, 1)})
    warnings.warn(f"catalog.mat not rewritten ({'; '.join(blockers)}): filter_flags saved to {side}")
    out["filter_flags_path"] = side
    return out
