"""Generate the committed golden fixtures from the CPU oracle (oracle/gpdla_oracle.py).

Run from the repo root:  python tests/golden/make_golden.py
The oracle is a restatement of process_qsos.m / voigt.c / log_mvnpdf_low_rank.m with
scipy.special.voigt_profile standing in for libcerf (see the oracle's header for how it is
pinned).  Only these data files travel to the GPU box.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from oracle import gpdla_oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent


def golden_voigt():
    rng = np.random.default_rng(7)
    cases = []
    for z_qso, nl in ((2.56, 3), (3.3, 1), (2.2, 31), (4.1, 3)):
        lo = np.log10(911.75 * (1 + z_qso)) + 0.003
        hi = np.log10(1215.75 * (1 + z_qso))
        lam = 10 ** np.arange(lo, hi, 1e-4)
        zmax = lam.max() / O.LYA_WAVELENGTH - 1 - O.MAX_Z_CUT
        zmin = lam.min() / O.LYA_WAVELENGTH - 1
        for z, N in ((rng.uniform(zmin, zmax), 10 ** 20.0), (rng.uniform(zmin, zmax), 10 ** 22.7),
                     (zmax, 10 ** 21.3), (zmin, 1e23)):
            cases.append((lam, z, N, nl, O.voigt_mex(lam, z, N, nl)))
    arrays = dict(z=np.array([c[1] for c in cases]), N=np.array([c[2] for c in cases]),
                  num_lines=np.array([c[3] for c in cases]))
    for i, c in enumerate(cases):
        arrays[f"lam_{i}"] = c[0]
        arrays[f"out_{i}"] = c[4]
    np.savez_compressed(OUT / "voigt.npz", **arrays)


def golden_mvn():
    rng = np.random.default_rng(11)
    rows = []
    for n, k in ((800, 20), (37, 4), (269, 20), (1250, 8)):
        M = 0.05 * rng.standard_normal((n, k))
        mu = 1 + 0.1 * rng.standard_normal(n)
        d = rng.uniform(0.01, 0.2, n)
        y = mu + M @ rng.standard_normal(k) + np.sqrt(d) * rng.standard_normal(n)
        rows.append(dict(y=y, mu=mu, M=M, d=d, out=O.log_mvnpdf_low_rank(y, mu, M, d)))
    np.savez_compressed(OUT / "mvn.npz", **{f"{key}_{i}": r[key] for i, r in enumerate(rows) for key in r})


def golden_process():
    model = syn.make_model(k=20)
    samples = syn.make_samples(96)
    # force coverage of the column-density range and both ends of the redshift range
    samples["offset_samples"][:4] = [0.0, 1.0, 0.5, 0.999]
    lognhi = np.log10(samples["nhi_samples"])
    lognhi[:4] = [20.0, 23.0, 21.7, 22.9]
    samples["nhi_samples"] = 10.0 ** lognhi
    samples["log_nhi_samples"] = lognhi
    spectra = syn.make_dr12q_like_spectra(model, 6, seed=5, mask_fraction=0.05)
    spectra += syn.make_spectra(model, 2, dla_fraction=1.0)
    packed = syn.pack_spectra(spectra)
    res = {}
    for mode in ("reference", "unmasked"):
        outs = [O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                   s["z_qso"], model, samples["offset_samples"], samples["nhi_samples"],
                                   num_lines=3, absorption_mode=mode) for s in spectra]
        res[mode] = outs
    np.savez_compressed(
        OUT / "process.npz",
        rest_wavelengths=model["rest_wavelengths"], mu=model["mu"], M=np.asarray(model["M"]),
        log_omega=model["log_omega"], log_c_0=model["log_c_0"], log_tau_0=model["log_tau_0"],
        log_beta=model["log_beta"], offset_samples=samples["offset_samples"],
        nhi_samples=samples["nhi_samples"], offsets=packed["offsets"],
        wavelengths=packed["wavelengths"], flux=packed["flux"], noise_variance=packed["noise_variance"],
        pixel_mask=packed["pixel_mask"], z_qsos=packed["z_qsos"],
        **{f"{mode}_{key}": np.array([o[key] for o in res[mode]])
           for mode in res for key in ("log_likelihood_no_dla", "sample_log_likelihoods_dla",
                                       "log_likelihood_dla", "min_z_dla", "max_z_dla", "n", "m")})


if __name__ == "__main__":
    golden_voigt()
    golden_mvn()
    golden_process()
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)
