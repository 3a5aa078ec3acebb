"""Numpy emulation of the 24-bit int8 panel path (panel_gemm_i8_24, gemm_i8.hip) with its weights'
raw Voigt profiles in fp32 (raw_profile3_pair_f32) against the fp64 restatement.

The path quantises the Gram weights to 3 digit planes (24 bits) and keeps the 6 digit pairs of level
<= 2, the u weights to 4 planes (levels <= 3), and hands the Gram to the LDL^T in fp32.  On the
device the raw profiles exp(N sum_j -lc_j V_j) are evaluated in packed fp32 from an fp64 x_j (the
subtraction of the line centre cancels), and the 7-tap instrument broadening runs in fp32; the
pixel terms r, d, 1/d, sum r^2/d and sum log d stay fp64.  This module emulates both profile
precisions (the fp32 one: profile values and their sum rounded to fp32, N tot and the exp in fp32,
the broadening in fp32) so the error added by the fp32 profile can be compared with the scheme's
own.  Test infrastructure (imports the oracle as the checker; lives under tests/ for that reason).
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from oracle import gpdla_oracle as O  # noqa: E402

from support.emulate_i8 import digits_balanced  # noqa: E402


def contract(wt, Pt, nd_a, nd_b, maxlevel, signed):
    """sum_slot wt[slot] Pt[slot, e] as gemm_i8.hip computes it with nd_a weight and nd_b panel
    digit planes and the digit pairs of level i + j <= maxlevel (emulate_i8.contract, generalised)."""
    mx = np.abs(Pt).max(axis=0)
    mx = np.where(mx > 0, mx, 1.0)
    se = mx / (127 * 2.0 ** 24)
    XB = np.rint(Pt / se).astype(np.int64)
    sc = (2.0 ** 31 - 256) if signed else (2.0 ** 32 - 256)
    U = np.rint(wt * sc).astype(np.int64) + (2 ** 31 if signed else 0)
    dA = [((U >> (8 * (3 - i))) & 255) - 128 for i in range(4)]
    dB = digits_balanced(XB)
    tot = np.zeros(Pt.shape[1])
    for i in range(nd_a):
        for j in range(nd_b):
            if i + j <= maxlevel:
                tot += (2.0 ** (8 * (6 - i - j))) * (dA[i][:, None] * dB[j]).sum(axis=0)
    tot += (8421504.0 if signed else 2155905152.0) * XB.sum(axis=0)
    return tot * se / sc


def voigt_f32(lambdas, z, N, num_lines=3):
    """voigt.c:253-304 with the device's fp32 profile: x_j in fp64, each line's value rounded to
    fp32 and summed in fp32, exp(N total) in fp32, the instrument broadening in fp32."""
    lambdas = np.asarray(lambdas, dtype=np.float64)
    mult = O.C_CGS / (O.TRANSITION_WAVELENGTHS[:num_lines] * (1 + z)) / 1e8
    total = np.zeros(lambdas.size, dtype=np.float32)
    for j in range(num_lines):
        vel = lambdas * mult[j] - O.C_CGS
        f = (O.LEADING_CONSTANTS[j] * O.libcerf_voigt(vel, O.SIGMA, O.LORENTZ_GAMMAS[j])).astype(np.float32)
        total = (total - f).astype(np.float32)
    raw = np.exp(np.float32(N) * total).astype(np.float32)
    n_out = lambdas.size - 2 * O.VOIGT_WIDTH
    prof = np.zeros(n_out, dtype=np.float32)
    for k in range(2 * O.VOIGT_WIDTH + 1):
        prof = (prof + raw[k:k + n_out] * np.float32(O.INSTRUMENT_PROFILE[k])).astype(np.float32)
    return prof.astype(np.float64)


def ll_24(prep, a):
    """The 24-bit path's sample log-likelihood for broadened absorption a (process_qsos.m:191-197,
    log_mvnpdf_low_rank.m:11-32): 3 x 3 Gram digits (level <= 2) rounded to fp32, 4 x 4 u digits."""
    y, mu, M, om2, noise = prep["y"], prep["mu"], prep["M"], prep["omega2"], prep["noise"]
    r = y - mu * a
    d = om2 * a * a + noise
    wg, wu = a * a / d, a * r / d
    k = M.shape[1]
    iu = np.triu_indices(k)
    P = M[:, iu[0]] * M[:, iu[1]]
    G = contract(wg * (om2 + noise), P / (om2 + noise)[:, None], 3, 3, 2, False)
    G = G.astype(np.float32).astype(np.float64)
    f = np.abs(y - mu)
    av = np.where(mu != 0, y / (2 * np.where(mu != 0, mu, 1)), -1)
    f = np.where((av > 0) & (av < 1), np.maximum(f, np.abs(y * av - mu * av * av)), f)
    beta = 1.125 * f / noise
    beta = np.where((beta > 0) & np.isfinite(beta), beta, 1.0)
    u = contract(wu / beta, M * beta[:, None], 4, 4, 3, True)
    B = np.eye(k)
    B[iu] += G
    B = np.triu(B) + np.triu(B, 1).T
    Lc = np.linalg.cholesky(B)
    t = np.linalg.solve(Lc, u)
    q = np.sum(r * r / d) - t @ t
    logdet = np.sum(np.log(d)) + 2 * np.sum(np.log(np.diag(Lc)))
    return -0.5 * (q + logdet + y.size * 1.83787706640934534)


def worst_errors(model, spectra, samples, picks):
    """Max relative log-likelihood error vs the fp64 oracle of the 24-bit scheme with fp64 and with
    fp32 raw profiles over the (spectrum, sample) pairs ``picks``."""
    worst = {"f64": 0.0, "f32": 0.0}
    for q, s in picks:
        spec = spectra[q]
        prep = O.prepare_spectrum(spec["wavelengths"], spec["flux"], spec["noise_variance"],
                                  spec["pixel_mask"], spec["z_qso"], model)
        z = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * samples["offset_samples"][s]
        N = samples["nhi_samples"][s]
        ref = O.sample_log_likelihood(prep, z, N, 3)
        idx = prep["absorption_index"]
        for key, a in (("f64", O.voigt_mex(prep["padded"], z, N, 3)[idx]),
                       ("f32", voigt_f32(prep["padded"], z, N)[idx])):
            worst[key] = max(worst[key], abs(ll_24(prep, a) - ref) / max(abs(ref), 1.0))
    return worst


if __name__ == "__main__":
    from gp_dla_detection_amd import synthetic as syn
    model = syn.make_model(k=50)
    samples = syn.make_samples(100000)
    rng = np.random.default_rng(3)
    spectra = [syn.make_spectrum(model, q) for q in range(8)]
    picks = [(q, int(s)) for q in range(8) for s in rng.choice(100000, 24, replace=False)]
    print(worst_errors(model, spectra, samples, picks))
