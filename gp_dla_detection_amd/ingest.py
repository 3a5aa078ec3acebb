"""Spectrum ingest: read_spec.m and preload_qsos.m.

``read_spec`` loads an SDSS DR12Q coadded "speclite" FITS file -- binary-table HDU 1, columns
1-4 = flux, loglam, ivar, and_mask (read_spec.m:11-25) -- and derives wavelengths, noise
variance and the bad-pixel mask (read_spec.m:27-38).  ``preload_qsos`` normalises each
catalogue spectrum by its median flux in the 1310-1325 A rest window, applies the filter-flag
rules and keeps the 910-1217 A rest range plus one unmasked pixel on either side
(preload_qsos.m:13-70), producing the cells process_qsos reads (preloaded_qsos.mat).

The FITS reader is a numpy implementation of the binary-table subset these files use (no
astropy on the GPU box).  MATLAB's fitsread returns a 'E' column as single precision, and
read_spec/preload_qsos keep computing in single (10.^loglam, 1./ivar, the normalisation); that
is reproduced here (float32 arithmetic, float32 cells, widened to float64 only when packed for
the engine) so the preloaded cells hold the values and the class the reference's cells hold.
"""
from __future__ import annotations

import os

import numpy as np

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


def read_spec(filename: str):
    """[wavelengths, flux, noise_variance, pixel_mask] = read_spec(filename) (read_spec.m)."""
    flux, log_wavelengths, ivar, and_mask = read_bintable(filename, 1, [1, 2, 3, 4])     # :11-25
    flux = np.asarray(flux, dtype=np.float32)
    log_wavelengths = np.asarray(log_wavelengths, dtype=np.float32)
    ivar = np.asarray(ivar, dtype=np.float32)
    wavelengths = np.power(np.float32(10), log_wavelengths)                              # :28
    with np.errstate(divide="ignore"):
        noise_variance = np.float32(1) / ivar                                            # :31
    and_mask = np.asarray(and_mask).astype(np.int64)
    pixel_mask = (ivar == 0) | (((and_mask >> (BRIGHTSKY - 1)) & 1) == 1)                # :36-38
    return wavelengths, flux, noise_variance, pixel_mask


def nanmedian(v: np.ndarray):
    """MATLAB's nanmedian (preload_qsos.m:33) in the array's own class: NaNs dropped, the middle
    element, or for an even count median.m's meanof(a, b) = a + (b - a) / 2 when a and b are finite
    with the same sign, else (a + b) / 2 -- numpy's (a + b) / 2 can differ from it in the last bit."""
    v = np.sort(v[~np.isnan(v)])
    n = v.size
    if n == 0:
        return v.dtype.type(np.nan)
    if n % 2:
        return v[n // 2]
    a, b = v[n // 2 - 1], v[n // 2]
    two = v.dtype.type(2)
    if np.isfinite(a) and np.isfinite(b) and np.sign(a) == np.sign(b):
        return a + (b - a) / two
    return (a + b) / two


def spec_filename(spectra_directory: str, plate: int, mjd: int, fiber_id: int) -> str:
    """The DR12Q layout file_loader reads: <spectra>/<plate>/spec-<plate>-<mjd>-<fiber>.fits."""
    return f"{spectra_directory}/{int(plate)}/spec-{int(plate)}-{int(mjd)}-{int(fiber_id):04d}.fits"


def preload_qsos(z_qsos, plates, mjds, fiber_ids, filter_flags, file_loader, log=None) -> dict:
    """preload_qsos.m:10-71.  ``file_loader(plate, mjd, fiber_id)`` returns read_spec's tuple.
    Returns the saved variables (cells as lists, filter_flags updated with bits 3 and 4)."""
    z_qsos = np.asarray(z_qsos, dtype=np.float64).ravel()
    filter_flags = np.array(filter_flags, dtype=np.uint8).ravel().copy()
    Q = z_qsos.size
    all_w, all_f, all_n, all_m = ([np.zeros(0) for _ in range(Q)] for _ in range(4))
    all_normalizers = np.zeros(Q)
    for i in range(Q):
        if filter_flags[i] > 0:                                                           # :19-21
            continue
        w, fl, nv, pm = file_loader(plates[i], mjds[i], fiber_ids[i])                     # :23-24
        # emitted_wavelengths (:26); single-precision cells stay single as in MATLAB
        rest = w / (np.float32(1 + z_qsos[i]) if w.dtype == np.float32 else 1 + z_qsos[i])
        ind = (rest >= P.NORMALIZATION_MIN_LAMBDA) & (rest <= P.NORMALIZATION_MAX_LAMBDA) & ~pm  # :29-31
        med = nanmedian(fl[ind])                                                          # :33
        if np.isnan(med):                                                                 # :36-39
            filter_flags[i] |= 1 << 2
            continue
        ind = (rest >= P.MIN_LAMBDA) & (rest <= P.MAX_LAMBDA) & ~pm                       # :41-43
        if np.count_nonzero(ind) < P.MIN_NUM_PIXELS:                                       # :46-49
            filter_flags[i] |= 1 << 3
            continue
        all_normalizers[i] = med                                                          # :51
        fl = fl / med                                                                     # :53
        nv = nv / (med * med)                                                             # :54
        ind = (rest >= P.LOADING_MIN_LAMBDA) & (rest <= P.LOADING_MAX_LAMBDA)             # :56-57
        avail = np.flatnonzero(~ind & ~pm)                                                # :60
        if ind.any():
            first, last = np.flatnonzero(ind)[0], np.flatnonzero(ind)[-1]
            after, before = avail[avail > last], avail[avail < first]
            if after.size:
                ind[after.min()] = True                                                  # :61
            if before.size:
                ind[before.max()] = True                                                 # :62
        # the cells keep fitsread's single class, as the reference's preloaded_qsos.mat holds them;
        # pack_spectra widens them (exactly) to the engine's fp64
        all_w[i], all_f[i] = w[ind], fl[ind]                                               # :64-67
        all_n[i], all_m[i] = nv[ind], pm[ind].astype(bool)
        if log:
            log(f"loaded quasar {i + 1} of {Q} ({plates[i]}/{mjds[i]}/{int(fiber_ids[i]):04d})")
    return dict(loading_min_lambda=P.LOADING_MIN_LAMBDA, loading_max_lambda=P.LOADING_MAX_LAMBDA,
                normalization_min_lambda=P.NORMALIZATION_MIN_LAMBDA,
                normalization_max_lambda=P.NORMALIZATION_MAX_LAMBDA, min_num_pixels=P.MIN_NUM_PIXELS,
                all_wavelengths=all_w, all_flux=all_f, all_noise_variance=all_n, all_pixel_mask=all_m,
                all_normalizers=all_normalizers, filter_flags=filter_flags)


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
                       lambda p, m, f: read_spec(spec_filename(spectra_dir, p, m, f)))
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
