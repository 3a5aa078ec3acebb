"""CPU restatement of generate_dla_samples.m in closed form -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  It is the vectorised numpy statement of the algorithm the
device kernels of gp_dla_detection_amd/csrc/dla_samples.hip implement (it was the product's host path
through round 5; round 6 moved the product onto the GPU), and the second checker of those kernels
beside oracle/dla_samples_oracle.py (which follows MATLAB's own order: quadrature integral, Brent
fzero, one sample at a time, too slow for 10^5 samples):

* ``scramble(haltonset(2), 'rr2')`` (generate_dla_samples.m:8-9): the Halton sequence in bases 2
  and 3, point 0 first (MATLAB's default Skip = 0 starts at the origin), each radical-inverse digit
  through the RR2 permutation of Kocis & Whiten (1997): the bit-reversed integers
  0 .. 2^ceil(log2 b) - 1 restricted to those below b.
* offsets = the first coordinate (:13).
* log10 N_HI prior (:17-49): alpha x (a fit to the catalogue's DLA column densities) +
  (1 - alpha) x U(uniform_min_log_nhi, uniform_max_log_nhi).  The fit is exp(quadratic), the
  quadratic a least-squares fit (polyfit, :34) of log ksdensity(log_nhis) on
  linspace(fit_min, fit_max, 1000) (:32-33), normalised over [fit_min, 25] (:37-38).
* log_nhi_samples(i) = fzero(cdf - u_i) (:51-55); nhi_samples = 10 .^ log_nhi_samples (:58).

ksdensity's default bandwidth is MATLAB's normal-reference rule on the median absolute deviation,
sigma = MAD / 0.6745, h = sigma (4 / 3N)^(1/5), Gaussian kernel, no boundary correction.  The fitted
density's integral is an erf difference when the quadratic is concave (any unimodal catalogue) and
adaptive quadrature otherwise; the inverse CDF is solved to full double precision by bracketed Newton
steps, where MATLAB's fzero / integral stop at their default tolerances.

Pins: the RR2 Halton points against MATLAB's own documented output (the haltonset/scramble example:
Skip 1e3, Leap 1e2, RR2, bases 2, 3, 5 -- reproduced to its 4 printed decimals), the density fit and
inverse CDF by their published definitions and against the MATLAB-order oracle
(tests/test_dla_samples.py); not by executed reference outputs (none ship with the reference).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erf

from gp_dla_detection_amd import parameters as P

ALPHA = 0.9                 # set_parameters.m:49
FIT_UPPER = 25.0            # generate_dla_samples.m:38 integral(..., fit_min_log_nhi, 25.0)


def rr2_permutation(base: int) -> np.ndarray:
    """RR2 digit permutation for ``base``: bit-reversed 0 .. 2^m - 1 (m = ceil(log2 base)),
    keeping the values below ``base``."""
    m = max(1, math.ceil(math.log2(base)))
    rev = [int(format(i, f"0{m}b")[::-1], 2) for i in range(1 << m)]
    perm = np.array([r for r in rev if r < base], dtype=np.int64)
    assert perm.size == base
    return perm


def halton_rr2(num: int, bases=(2, 3), start: int = 0) -> np.ndarray:
    """Points ``start .. start+num-1`` of the RR2-scrambled Halton sequence, shape (num, dims)."""
    idx = np.arange(start, start + num, dtype=np.int64)
    out = np.zeros((num, len(bases)))
    for d, b in enumerate(bases):
        perm = rr2_permutation(b)
        i = idx.copy()
        scale = 1.0 / b
        while np.any(i > 0):
            out[:, d] += perm[i % b] * scale
            i //= b
            scale /= b
    return out


def ksdensity_bandwidth(x: np.ndarray) -> float:
    """MATLAB ksdensity default: normal-reference bandwidth on the median absolute deviation."""
    x = np.asarray(x, dtype=np.float64).ravel()
    sig = np.median(np.abs(x - np.median(x))) / 0.6745
    if sig <= 0:
        sig = np.max(x) - np.min(x)
    return float(sig * (4.0 / (3.0 * x.size)) ** 0.2) if sig > 0 else 1.0


def ksdensity(data: np.ndarray, points: np.ndarray, bandwidth: float | None = None) -> np.ndarray:
    """Gaussian-kernel density estimate of ``data`` at ``points`` (ksdensity(data, points))."""
    data = np.asarray(data, dtype=np.float64).ravel()
    points = np.asarray(points, dtype=np.float64).ravel()
    h = ksdensity_bandwidth(data) if bandwidth is None else bandwidth
    out = np.empty(points.size)
    for a in range(0, points.size, 256):
        z = (points[a:a + 256, None] - data[None, :]) / h
        out[a:a + 256] = np.exp(-0.5 * z * z).sum(axis=1)
    return out / (data.size * h * math.sqrt(2 * math.pi))


class ColumnDensityPrior:
    """The log10 N_HI mixture prior of generate_dla_samples.m:17-49."""

    def __init__(self, log_nhis, alpha: float = ALPHA,
                 uniform_min: float = P.UNIFORM_MIN_LOG_NHI, uniform_max: float = P.UNIFORM_MAX_LOG_NHI,
                 fit_min: float = P.FIT_MIN_LOG_NHI, fit_max: float = P.FIT_MAX_LOG_NHI):
        self.alpha, self.umin, self.umax, self.fmin, self.fmax = alpha, uniform_min, uniform_max, fit_min, fit_max
        x = np.linspace(fit_min, fit_max, 1000)                                    # :32
        kde = ksdensity(log_nhis, x)                                               # :33
        self.coeffs = np.polyfit(x, np.log(kde), 2)                                # :34
        self.Z = self._fit_integral(fit_min, FIT_UPPER)                            # :37-38

    # exp(c2 x^2 + c1 x + c0) and its integral
    def _fit_pdf(self, t):
        return np.exp(np.polyval(self.coeffs, t))

    def _fit_integral(self, lo, hi):
        c2, c1, c0 = self.coeffs
        lo, hi = np.asarray(lo, dtype=np.float64), np.asarray(hi, dtype=np.float64)
        if c2 < 0:
            s = math.sqrt(-c2)
            m = -c1 / (2 * c2)
            peak = math.exp(c0 - c1 * c1 / (4 * c2))
            return peak * math.sqrt(math.pi) / (2 * s) * (erf(s * (hi - m)) - erf(s * (lo - m)))
        from scipy.integrate import quad
        f = np.vectorize(lambda a, b: quad(lambda t: float(self._fit_pdf(t)), a, b, epsabs=0, epsrel=1e-13)[0])
        return f(lo, hi)

    def pdf(self, t):
        """normalized_pdf (:42-44)."""
        t = np.asarray(t, dtype=np.float64)
        uni = np.where((t >= self.umin) & (t <= self.umax), 1.0 / (self.umax - self.umin), 0.0)
        return self.alpha * self._fit_pdf(t) / self.Z + (1 - self.alpha) * uni

    def cdf(self, t):
        """cdf(nhi) = integral(normalized_pdf, fit_min_log_nhi, nhi) (:46)."""
        t = np.asarray(t, dtype=np.float64)
        fit = self._fit_integral(self.fmin, t) / self.Z
        lo = max(self.fmin, self.umin)
        uni = (np.clip(t, lo, self.umax) - lo) / (self.umax - self.umin)
        return self.alpha * fit + (1 - self.alpha) * np.where(t >= lo, uni, 0.0)

    def inverse_cdf(self, u) -> np.ndarray:
        """fzero(@(nhi) cdf(nhi) - u, 20.5) (:51-55): bracketed Newton to full precision."""
        u = np.asarray(u, dtype=np.float64)
        lo = np.full(u.shape, self.fmin)
        hi = np.full(u.shape, FIT_UPPER)
        t = np.clip(np.full(u.shape, 20.5), lo, hi)
        for _ in range(200):
            g = self.cdf(t) - u
            lo = np.where(g <= 0, t, lo)
            hi = np.where(g > 0, t, hi)
            d = self.pdf(t)
            with np.errstate(divide="ignore", invalid="ignore"):
                tn = t - g / d
            bad = ~np.isfinite(tn) | (tn <= lo) | (tn >= hi)
            tn = np.where(bad, 0.5 * (lo + hi), tn)
            done = np.abs(tn - t) <= 4 * np.finfo(float).eps * np.abs(t)
            t = tn
            if np.all(done | (hi - lo <= 4 * np.finfo(float).eps * np.abs(hi))):
                break
        return np.where(u <= 0, self.fmin, t)


def generate_dla_samples(log_nhis, num_dla_samples: int = P.NUM_DLA_SAMPLES, alpha: float = ALPHA) -> dict:
    """The variables generate_dla_samples.m:60-63 saves.  ``log_nhis``: the catalogue's DLA column
    densities (catalog.log_nhis(dla_catalog_name), a cell of per-sightline vectors or one array;
    empty cells are skipped like :28-30)."""
    if isinstance(log_nhis, (list, tuple)) or (isinstance(log_nhis, np.ndarray) and log_nhis.dtype == object):
        parts = [np.asarray(c, dtype=np.float64).ravel() for c in np.asarray(log_nhis, dtype=object).ravel()]
        data = np.concatenate([p for p in parts if p.size] or [np.zeros(0)])
    else:
        data = np.asarray(log_nhis, dtype=np.float64).ravel()
    if data.size < 2:
        raise ValueError("need at least two catalogue column densities for the density fit")
    seq = halton_rr2(num_dla_samples)                                              # :8-9
    prior = ColumnDensityPrior(data, alpha=alpha)
    log_nhi = prior.inverse_cdf(seq[:, 1])                                         # :51-55
    return dict(uniform_min_log_nhi=P.UNIFORM_MIN_LOG_NHI, uniform_max_log_nhi=P.UNIFORM_MAX_LOG_NHI,
                fit_min_log_nhi=P.FIT_MIN_LOG_NHI, fit_max_log_nhi=P.FIT_MAX_LOG_NHI, alpha=alpha,
                offset_samples=seq[:, 0].copy(), log_nhi_samples=log_nhi, nhi_samples=10.0 ** log_nhi)
