"""CPU oracle for generate_dla_samples.m -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker of gp_dla_detection_amd/dla_samples.py.
It restates the reference script step by step, in MATLAB's order and with MATLAB's building
blocks as their documentation defines them, written independently of the product module:

* generate_dla_samples.m:8-9   ``scramble(haltonset(2), 'rr2')``: radical inverse of point i in
  base b with each digit mapped through the RR2 permutation (Kocis & Whiten 1997: the bit-reversed
  integers 0 .. 2^ceil(log2 b) - 1 that are below b), one point at a time, digit by digit.
* :13                          offsets = the first coordinate of points 1..S (MATLAB's point 1 is
                               the sequence's index 0, the origin).
* :26-28                       the non-empty cells concatenated in order.
* :32-33                       ``ksdensity(log_nhis, x)`` at 1,000 linspace points: Gaussian kernel,
                               MATLAB's default bandwidth sig (4 / 3n)^(1/5), sig = MAD / 0.6745
                               (median absolute deviation about the median).
* :34                          ``polyfit(x, log(kde), 2)`` as MATLAB computes it: the Vandermonde
                               system by an economy QR, p = R \\ (Q' y).
* :37-38                       Z = integral of exp(polyval(f, t)) over [fit_min, 25]
                               (scipy.integrate.quad standing in for MATLAB's adaptive
                               Gauss-Kronrod ``integral``; tolerances tightened below MATLAB's
                               defaults AbsTol 1e-10 / RelTol 1e-6 so the oracle is the sharper one).
* :42-46                       normalized_pdf = alpha fit / Z + (1 - alpha) U(20, 23);
                               cdf(t) = integral(normalized_pdf, fit_min, t).
* :51-54                       fzero(cdf - u_i, 20.5): a root bracket found by expanding around
                               20.5, then Brent's method to full precision (scipy.optimize.brentq,
                               the algorithm MATLAB's fzero documents).
* :57                          nhi_samples = 10 .^ log_nhi_samples.

Parity status: the reference ships no catalogue or sample file, so this oracle is pinned by
MATLAB's documented algorithms (and the RR2 points by MATLAB's documented haltonset/scramble
output, tests/test_dla_samples.py), not by executed reference outputs.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import integrate, optimize

UNIFORM_MIN, UNIFORM_MAX = 20.0, 23.0      # set_parameters.m:50-51
FIT_MIN, FIT_MAX = 20.0, 22.0              # set_parameters.m:52-53
ALPHA = 0.9                                # set_parameters.m:49


def rr2_digit_map(b: int) -> list[int]:
    m = 1
    while (1 << m) < b:
        m += 1
    out = []
    for i in range(1 << m):
        r = 0
        for bit in range(m):          # reverse the m-bit representation of i
            if i >> bit & 1:
                r |= 1 << (m - 1 - bit)
        if r < b:
            out.append(r)
    return out


def halton_rr2_point(i: int, b: int) -> float:
    perm = rr2_digit_map(b)
    x, f = 0.0, 1.0 / b
    while i > 0:
        x += perm[i % b] * f
        i //= b
        f /= b
    return x


def mad_bandwidth(data: np.ndarray) -> float:
    med = np.median(data)
    sig = np.median(np.abs(data - med)) / 0.6745
    return sig * (4.0 / (3.0 * data.size)) ** (1.0 / 5.0)


def ksdensity(data: np.ndarray, x: np.ndarray) -> np.ndarray:
    h = mad_bandwidth(data)
    out = np.zeros(x.size)
    for j, xj in enumerate(x):
        u = (xj - data) / h
        out[j] = np.sum(np.exp(-0.5 * u * u)) / (data.size * h * math.sqrt(2.0 * math.pi))
    return out


def polyfit_qr(x: np.ndarray, y: np.ndarray, n: int) -> np.ndarray:
    V = np.vander(x, n + 1)
    Q, R = np.linalg.qr(V, mode="reduced")
    return np.linalg.solve(R, Q.T @ y)


def generate_dla_samples(cells, num_dla_samples: int, alpha: float = ALPHA, sample_indices=None) -> dict:
    """``sample_indices`` (optional): solve :51-54 only for these samples (the others are NaN) -- the
    per-sample quadrature and Brent root are slow, so checks at 10^5 samples take a subset."""
    log_nhis = np.concatenate([np.asarray(c, dtype=np.float64).ravel() for c in cells
                               if np.asarray(c).size > 0])                          # :26-28
    x = np.linspace(FIT_MIN, FIT_MAX, 1000)                                        # :32
    kde_pdf = ksdensity(log_nhis, x)                                               # :33
    f = polyfit_qr(x, np.log(kde_pdf), 2)                                          # :34

    def unnormalized_pdf(t):                                                       # :37
        return math.exp((f[0] * t + f[1]) * t + f[2])

    Z = integrate.quad(unnormalized_pdf, FIT_MIN, 25.0, epsabs=1e-15, epsrel=1e-13, limit=200)[0]  # :38

    def normalized_pdf(t):                                                         # :42-44
        uni = 1.0 / (UNIFORM_MAX - UNIFORM_MIN) if UNIFORM_MIN <= t <= UNIFORM_MAX else 0.0
        return alpha * (unnormalized_pdf(t) / Z) + (1 - alpha) * uni

    def cdf(t):                                                                    # :46
        brk = [p for p in (UNIFORM_MIN, UNIFORM_MAX) if FIT_MIN < p < t]
        return integrate.quad(normalized_pdf, FIT_MIN, t, points=brk or None, epsabs=1e-15, epsrel=1e-13,
                              limit=200)[0]

    offsets = np.array([halton_rr2_point(i, 2) for i in range(num_dla_samples)])  # :13
    us = np.array([halton_rr2_point(i, 3) for i in range(num_dla_samples)])
    out = np.full(num_dla_samples, np.nan)
    todo = range(num_dla_samples) if sample_indices is None else sample_indices
    for i in todo:                                                                 # :51-54
        u = us[i]
        g = lambda t: cdf(t) - u                                                   # noqa: E731
        if g(FIT_MIN) >= 0:
            out[i] = FIT_MIN
            continue
        lo, hi, step = 20.5, 20.5, 0.05                                            # fzero's bracket search
        while g(lo) > 0 and lo > FIT_MIN:
            lo = max(FIT_MIN, 20.5 - step)
            step *= 2
        step = 0.05
        while g(hi) < 0:
            hi = 20.5 + step
            step *= 2
        out[i] = optimize.brentq(g, lo, hi, xtol=1e-15, rtol=4 * np.finfo(float).eps, maxiter=200)
    return dict(offset_samples=offsets, log_nhi_samples=out, nhi_samples=10.0 ** out)  # :57
