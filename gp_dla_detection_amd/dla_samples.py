"""``generate_dla_samples`` mirror (generate_dla_samples.m:1-63): the DLA parameter samples every
spectrum's likelihood sweep is evaluated on, computed on the GPU.

The reference draws a 2-D quasi-random sequence and maps its second coordinate through the inverse CDF
of a column-density prior.  Every numeric step runs in libgpdla (csrc/dla_samples.hip, C-ABI
``gpdla_generate_dla_samples_f64`` / ``gpdla_halton_rr2_f64``):

* ``scramble(haltonset(2), 'rr2')`` (:8-9) -- one device thread per point, RR2-permuted radical-
  inverse digits (Kocis & Whiten 1997), point 0 the origin; bit-exact;
* offsets = the first coordinate (:13);
* ``ksdensity(log_nhis, linspace(fit_min, fit_max, 1000))`` (:32-33) -- a device block per grid point
  at MATLAB's default bandwidth (MAD / 0.6745 (4 / 3n)^(1/5));
* ``polyfit(x, log(kde), 2)`` (:34) -- economy QR on the host, as MATLAB solves it;
* Z = integral of the fit over [fit_min, 25] (:37-38) and the mixture CDF (:42-46) -- an erf difference
  for a concave fit, Gauss-Legendre otherwise;
* ``fzero(cdf - u_i, 20.5)`` (:51-55) -- one device thread per sample, bracketed Newton to full double
  precision (MATLAB's fzero / integral stop at their default tolerances);
* nhi_samples = 10 .^ log_nhi_samples (:57).

There is no CPU path: without a HIP device the calls raise (GpdlaError, GPDLA_EDEVICE).  Checkers:
oracle/dla_samples_oracle.py (MATLAB's order, step by step) and oracle/dla_samples_closed_form.py (the
same closed-form algorithm in numpy), tests/test_gpu_dla_samples.py.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from . import parameters as P

ALPHA = 0.9                 # set_parameters.m:49
FIT_UPPER = 25.0            # generate_dla_samples.m:38 integral(..., fit_min_log_nhi, 25.0)


def catalogue_column_densities(log_nhis) -> np.ndarray:
    """The catalogue's column densities as one vector: a cell of per-sightline vectors with the empty
    cells skipped (generate_dla_samples.m:26-28), or an array."""
    if isinstance(log_nhis, (list, tuple)) or (isinstance(log_nhis, np.ndarray) and log_nhis.dtype == object):
        parts = [np.asarray(c, dtype=np.float64).ravel() for c in np.asarray(log_nhis, dtype=object).ravel()]
        return np.ascontiguousarray(np.concatenate([p for p in parts if p.size] or [np.zeros(0)]))
    return np.ascontiguousarray(np.asarray(log_nhis, dtype=np.float64).ravel())


def halton_rr2(num: int, bases=(2, 3), start: int = 0, stride: int = 1, device: int = 0) -> np.ndarray:
    """Points ``start, start + stride, ...`` (``num`` of them) of the RR2-scrambled Halton sequence on the
    device, shape (num, len(bases)): MATLAB's ``scramble(haltonset(d, 'Skip', start, 'Leap', stride - 1),
    'RR2')`` rows (generate_dla_samples.m:8-9)."""
    b = np.ascontiguousarray(bases, dtype=np.int32)
    out = np.empty((num, b.size), dtype=np.float64)
    L.check(L.load().gpdla_halton_rr2_f64(device, start, stride, num, b.ctypes.data_as(C.POINTER(C.c_int32)), b.size,
                                          L.ptr(out)))
    return out


def generate_dla_samples(log_nhis, num_dla_samples: int = P.NUM_DLA_SAMPLES, alpha: float = ALPHA,
                         device: int = 0) -> dict:
    """The variables generate_dla_samples.m:60-63 saves.  ``log_nhis``: the catalogue's DLA column
    densities (catalog.log_nhis(dla_catalog_name), a cell of per-sightline vectors or one array).
    ``fit`` carries the quadratic's coefficients (highest power first), Z and the KDE bandwidth."""
    data = catalogue_column_densities(log_nhis)
    if data.size < 2:
        raise ValueError("need at least two catalogue column densities for the density fit")
    prior = L.DlaPrior(alpha, P.UNIFORM_MIN_LOG_NHI, P.UNIFORM_MAX_LOG_NHI, P.FIT_MIN_LOG_NHI, P.FIT_MAX_LOG_NHI,
                       FIT_UPPER)
    off = np.empty(num_dla_samples)
    lognhi = np.empty(num_dla_samples)
    nhi = np.empty(num_dla_samples)
    fit = np.empty(5)
    L.check(L.load().gpdla_generate_dla_samples_f64(device, L.ptr(data), data.size, num_dla_samples, C.byref(prior),
                                                    L.ptr(off), L.ptr(lognhi), L.ptr(nhi), L.ptr(fit)))
    return dict(uniform_min_log_nhi=P.UNIFORM_MIN_LOG_NHI, uniform_max_log_nhi=P.UNIFORM_MAX_LOG_NHI,
                fit_min_log_nhi=P.FIT_MIN_LOG_NHI, fit_max_log_nhi=P.FIT_MAX_LOG_NHI, alpha=alpha,
                offset_samples=off, log_nhi_samples=lognhi, nhi_samples=nhi,
                fit=dict(coeffs=fit[:3].copy(), Z=float(fit[3]), bandwidth=float(fit[4])))


def run_generate_dla_samples(base_directory: str, training_release: str, dla_catalog_name: str,
                             num_dla_samples: int = P.NUM_DLA_SAMPLES, device: int = 0) -> dict:
    """The script on files: reads <base>/<training_release>/processed/catalog.mat (log_nhis as a
    struct keyed by catalogue name, see process.run_process_qsos) and writes dla_samples.mat."""
    from .matv73 import loadmat
    from .process import processed_directory, save_dla_samples
    d = processed_directory(base_directory, training_release)
    catalog = loadmat(f"{d}/catalog.mat", ["log_nhis"])
    out = generate_dla_samples(catalog["log_nhis"][dla_catalog_name], num_dla_samples, device=device)
    scalars = {k: np.float64(out[k]) for k in ("uniform_min_log_nhi", "uniform_max_log_nhi",
                                                "fit_min_log_nhi", "fit_max_log_nhi", "alpha")}
    save_dla_samples(f"{d}/dla_samples.mat", {k: v for k, v in out.items() if k != "fit"}, **scalars)
    return out
