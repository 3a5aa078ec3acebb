"""CPU oracle for read_spec.m and preload_qsos.m -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` runs this module, as the checker of gp_dla_detection_amd/ingest.py and its device
kernels (csrc/ingest.hip).  Its FITS path needs astropy (a reader independent of the product's own
numpy one) and is executed with the interpreter that has it (/opt/conda/bin/python3.9 in the build
container; absent on the GPU box):

    python3.9 oracle/ingest_oracle.py <job.npz> <out.npz>

job.npz holds the catalogue columns (z_qsos, plates, mjds, fiber_ids, filter_flags) and the
spectra directory; out.npz receives every variable preload_qsos.m saves, cells flattened.

Restated, in MATLAB's order and classes:
* read_spec.m:11-38   fitsread(..., 'binarytable', 1, 'tablecolumns', 1:4) -- astropy.io.fits,
  columns kept in their FITS class ('E' -> single, like fitsread); wavelengths = 10.^loglam and
  noise_variance = 1 ./ ivar computed in single; pixel_mask = (ivar == 0) | bitget(and_mask, 24).
* preload_qsos.m:18-71  per catalogue entry, skipping filter_flags > 0 (:19-21):
  - rest = wavelengths / (1 + z): single / double is single in MATLAB (:26; emitted_wavelengths,
    set_parameters.m:14-15);
  - nanmedian of the flux in the 1310-1325 A window over unmasked pixels (:29-33), with MATLAB's
    median for an even count, meanof(a, b) = a + (b - a) / 2 (same signs, finite), else
    (a + b) / 2;
  - bit 3 when the median is NaN (:36-39), bit 4 when fewer than 200 unmasked pixels fall in
    911.75-1215.75 A (:41-49);
  - flux / median and noise_variance / median^2 in single (:53-54);
  - the 910-1217 A loading range plus one unmasked pixel on either side, the first found after
    the range's last pixel, then the last before its first (:56-62; ``min``/``max`` of an empty
    set index nothing).
10.^x is taken correctly rounded to single (the double power rounded once); MATLAB's single pow may
differ in the last ulp (unpinned).  ``preload_from_columns`` is the same restatement on columns
already read (no astropy: the GPU tests run it on the box against the device kernels).  Parity status: no reference outputs exist (the spectra are downloaded), so the
oracle is pinned by the .m files' semantics as MATLAB documents them, not by executed outputs.
"""
from __future__ import annotations

import sys

import numpy as np

BRIGHTSKY = 24                                     # read_spec.m:9
NORMALIZATION_MIN, NORMALIZATION_MAX = 1310.0, 1325.0   # set_parameters.m:29-30
MIN_LAMBDA, MAX_LAMBDA = 911.75, 1215.75           # set_parameters.m:33-34
LOADING_MIN, LOADING_MAX = 910.0, 1217.0           # set_parameters.m:21-22
MIN_NUM_PIXELS = 200                               # set_parameters.m:26


def read_columns(filename):
    """fitsread(filename, 'binarytable', 1, 'tablecolumns', 1:4) (read_spec.m:11-25), astropy."""
    if not hasattr(np, "asscalar"):          # astropy 4.3 with numpy >= 1.23
        np.asscalar = lambda a: a.item()
    if not hasattr(np, "alen"):
        np.alen = lambda a: len(a)
    from astropy.io import fits
    with fits.open(filename, memmap=False) as h:
        data = h[1].data
        names = h[1].columns.names
        flux = np.array(data[names[0]])                                            # :16
        log_wavelengths = np.array(data[names[1]])                                 # :19
        ivar = np.array(data[names[2]])                                            # :22
        and_mask = np.array(data[names[3]])                                        # :25
    return tuple(a.astype(a.dtype.newbyteorder("=")) for a in (flux, log_wavelengths, ivar, and_mask))


def derive(flux, log_wavelengths, ivar, and_mask):
    """read_spec.m:27-38 on the fitsread columns, in single.  10.^loglam is taken correctly rounded to
    single (the double power rounded once: over every float32 loglam in [3.0, 4.5] that equals the
    extended-precision value rounded to single, tests/test_ingest.py); MATLAB's own single pow is
    unpinned at the last ulp."""
    wavelengths = (10.0 ** np.asarray(log_wavelengths, np.float64)).astype(np.float32)   # :28
    with np.errstate(divide="ignore"):
        noise_variance = np.float32(1.0) / ivar                                    # :31
    bit = (np.asarray(and_mask).astype(np.int64) >> (BRIGHTSKY - 1)) & 1           # bitget(and_mask, 24)
    pixel_mask = (ivar == 0) | (bit == 1)                                          # :36-38
    return wavelengths, flux, noise_variance, pixel_mask


def read_spec(filename):
    return derive(*read_columns(filename))


def matlab_median(v):
    """median.m: middle element, or meanof of the two middle ones."""
    s = np.sort(v)
    n = s.size
    if n == 0:
        return v.dtype.type(np.nan)
    if n % 2:
        return s[n // 2]
    a, b = s[n // 2 - 1], s[n // 2]
    if np.sign(a) == np.sign(b) and np.isfinite(a) and np.isfinite(b):
        return a + (b - a) / v.dtype.type(2)
    return (a + b) / v.dtype.type(2)


def preload_one(w, fl, nv, pm, z):
    """preload_qsos.m:26-67 for one spectrum: (flag bits to set, median, cells or None)."""
    rest = w / np.float32(1.0 + z)                                                 # :26 (single)
    ind = (rest >= NORMALIZATION_MIN) & (rest <= NORMALIZATION_MAX) & ~pm          # :29-31
    vals = fl[ind]
    med = matlab_median(vals[~np.isnan(vals)])                                     # :33 nanmedian
    if np.isnan(med):                                                              # :36-39
        return 1 << 2, med, None
    ind = (rest >= MIN_LAMBDA) & (rest <= MAX_LAMBDA) & ~pm                        # :41-43
    if np.count_nonzero(ind) < MIN_NUM_PIXELS:                                     # :46-49
        return 1 << 3, med, None
    fl = fl / med                                                                  # :53
    nv = nv / (med * med)                                                          # :54 (single)
    ind = (rest >= LOADING_MIN) & (rest <= LOADING_MAX)                            # :56-57
    available = [j for j in range(ind.size) if not ind[j] and not pm[j]]           # :60
    sel = [j for j in range(ind.size) if ind[j]]
    if sel:
        after = [j for j in available if j > sel[-1]]
        if after:
            ind[min(after)] = True                                                 # :61
        sel = [j for j in range(ind.size) if ind[j]]
        before = [j for j in available if j < sel[0]]
        if before:
            ind[max(before)] = True                                                # :62
    return 0, med, (w[ind], fl[ind], nv[ind], pm[ind])                             # :64-67


def preload_from_columns(z_qsos, filter_flags, columns):
    """preload_qsos.m:18-67 over spectra given as their fitsread columns (flux, loglam, ivar,
    and_mask) -- ``columns[i]`` may be None for an entry that is pre-filtered (filter_flags > 0)."""
    Q = len(z_qsos)
    flags = np.array(filter_flags, dtype=np.uint8).copy()
    out = dict(all_wavelengths=[None] * Q, all_flux=[None] * Q, all_noise_variance=[None] * Q,
               all_pixel_mask=[None] * Q, all_normalizers=np.zeros(Q), medians=np.full(Q, np.nan, np.float32))
    for i in range(Q):                                                             # :18
        if flags[i] > 0:                                                           # :19-21
            continue
        bits, med, cells = preload_one(*derive(*columns[i]), z_qsos[i])            # :23-67
        flags[i] |= bits
        out["medians"][i] = med
        if cells is None:
            continue
        out["all_normalizers"][i] = med                                            # :51
        for key, c in zip(("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask"), cells):
            out[key][i] = c
    out["filter_flags"] = flags
    return out


def preload_qsos(z_qsos, plates, mjds, fiber_ids, filter_flags, spectra_dir):
    cols = [None if filter_flags[i] > 0 else
            read_columns(f"{spectra_dir}/{int(plates[i])}/spec-{int(plates[i])}-{int(mjds[i])}-{int(fiber_ids[i]):04d}.fits")
            for i in range(len(z_qsos))]                                           # :23-24
    return preload_from_columns(z_qsos, filter_flags, cols)


def main(job_path, out_path):
    job = np.load(job_path, allow_pickle=False)
    out = preload_qsos(job["z_qsos"], job["plates"], job["mjds"], job["fiber_ids"], job["filter_flags"],
                       str(job["spectra_dir"]))
    flat = dict(filter_flags=out["filter_flags"], all_normalizers=out["all_normalizers"])
    for key in ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask"):
        for i, c in enumerate(out[key]):
            if c is not None:
                flat[f"{key}__{i}"] = c
    np.savez(out_path, **flat)


if __name__ == "__main__":
    sys.dont_write_bytecode = True
    main(sys.argv[1], sys.argv[2])
