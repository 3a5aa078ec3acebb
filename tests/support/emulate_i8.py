"""Numpy emulation of the int8 Ozaki contraction (kernels_i8.hip) against the fp64 likelihood.

Quantises the per-slot weights and panel entries exactly as convert_i8_kernel / likelihood_i8_kernel
do, forms the digit-pair level sums in int64 (exact, like the int32 MFMA accumulators), and reports
the log-likelihood error vs the fp64 restatement for the kept levels (<= 3 or <= 4).
Test infrastructure (imports the oracle as the checker; lives under tests/ for that reason)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from oracle import gpdla_oracle as O
from gp_dla_detection_amd import synthetic as syn


def digits_balanced(X):
    X = X.astype(np.int64).copy()
    ds = []
    for _ in range(3):
        d = ((X + 128) & 255) - 128
        ds.append(d)
        X = (X - d) >> 8
    ds.append(X)
    return ds[::-1]  # d0 (most significant) .. d3


def contract(wt, Pt, maxlevel, signed):
    """sum_slot wt[slot] Pt[slot, e] as kernels_i8.hip computes it: weights quantised to
    X_A = rint(w (2^32 - 256)) (Gram, w in [0, 1]) or rint(w (2^31 - 256)) + 2^31 (u, w in [-1, 1])
    read as 4 offset bytes; panel entries X_B = rint(P / s_e), s_e = max|P_e| / (127 2^24), in 4
    balanced base-256 digits; digit pairs of level i + j <= maxlevel summed exactly (int64 here,
    int32 on the GPU); + the offset term c * colsum_e."""
    mx = np.abs(Pt).max(axis=0)
    mx = np.where(mx > 0, mx, 1.0)
    se = mx / (127 * 2.0 ** 24)
    XB = np.rint(Pt / se).astype(np.int64)
    sc = (2.0 ** 31 - 256) if signed else (2.0 ** 32 - 256)
    U = np.rint(wt * sc).astype(np.int64) + (2 ** 31 if signed else 0)
    dA = [((U >> (8 * (3 - i))) & 255) - 128 for i in range(4)]
    dB = digits_balanced(XB)
    tot = np.zeros(Pt.shape[1])
    for i in range(4):
        for j in range(4):
            if i + j <= maxlevel:
                tot += (2.0 ** (8 * (6 - i - j))) * (dA[i][:, None] * dB[j]).sum(axis=0)
    tot += (8421504.0 if signed else 2155905152.0) * XB.sum(axis=0)
    return tot * se / sc


def ll_i8(prep, z, nhi, maxlevel):
    a = O.voigt_mex(prep["padded"], z, nhi, 3)[prep["absorption_index"]]
    y, mu, M, om2, noise = prep["y"], prep["mu"], prep["M"], prep["omega2"], prep["noise"]
    r = y - mu * a
    d = om2 * a * a + noise
    wg = a * a / d
    wu = a * r / d
    k = M.shape[1]
    iu = np.triu_indices(k)
    P = (M[:, iu[0]] * M[:, iu[1]])
    wt = wg * (om2 + noise)
    G = contract(wt, P / (om2 + noise)[:, None], maxlevel, False)
    f = np.abs(y - mu)
    av = np.where(mu != 0, y / (2 * np.where(mu != 0, mu, 1)), -1)
    f = np.where((av > 0) & (av < 1), np.maximum(f, np.abs(y * av - mu * av * av)), f)
    beta = 1.125 * f / noise
    beta = np.where((beta > 0) & np.isfinite(beta), beta, 1.0)
    u = contract(wu / beta, M * beta[:, None], maxlevel, True)
    B = np.eye(k)
    B[iu] += G
    B = np.triu(B) + np.triu(B, 1).T
    Lc = np.linalg.cholesky(B)
    t = np.linalg.solve(Lc, u)
    q = np.sum(r * r / d) - t @ t
    logdet = np.sum(np.log(d)) + 2 * np.sum(np.log(np.diag(Lc)))
    return -0.5 * (q + logdet + y.size * 1.83787706640934534)


if __name__ == "__main__":
    model = syn.make_model(k=20)
    samples = syn.make_samples(10000)
    rng = np.random.default_rng(3)
    worst = {3: 0.0, 4: 0.0}
    for q in range(6):
        spec = syn.make_spectrum(model, q) if q < 3 else syn.make_dr12q_like_spectra(model, 8, seed=q)[q]
        prep = O.prepare_spectrum(spec["wavelengths"], spec["flux"], spec["noise_variance"],
                                  spec["pixel_mask"], spec["z_qso"], model)
        for s in rng.choice(10000, 12, replace=False):
            z = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * samples["offset_samples"][s]
            N = samples["nhi_samples"][s]
            ref = O.sample_log_likelihood(prep, z, N, 3)
            for lv in (3, 4):
                err = abs(ll_i8(prep, z, N, lv) - ref) / max(abs(ref), 1)
                worst[lv] = max(worst[lv], err)
    print("max rel err  level<=3: %.3e   level<=4: %.3e" % (worst[3], worst[4]))
