"""Seeded synthetic inputs for the hot path.

No catalogue, spectra or trained model ships with the reference (it downloads 35 GB of SDSS
data, README.md:54), so tests and the benchmark use inputs of the reference's shapes:

* model    -- the four arrays of ``learned_qso_model_*.mat`` (learn_qso_model.m:103-123):
              rest grid 911.75:0.25:1215.75 (1,217 points, set_parameters.m:33-35), ``mu``,
              ``M`` (1217 x k), ``log_omega`` and the three absorption-noise scalars.
* samples  -- ``dla_samples.mat`` (generate_dla_samples.m:13,57): offsets and N_HI from an
              unscrambled 2-D Halton sequence (the uniform-prior component; the KDE part needs
              catalogue data that is not available).
* spectra  -- ``preloaded_qsos.mat`` cells (preload_qsos.m:64-67): observed wavelengths on a
              1e-4 dex grid, normalised flux, noise variance and pixel mask, plus z_QSO.
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import gaussian_filter1d
from scipy.special import voigt_profile

from . import parameters as P


def make_model(k: int = 20, seed: int = 1605) -> dict:
    rng = np.random.default_rng(seed)
    lam = np.arange(P.MIN_LAMBDA, P.MAX_LAMBDA + P.DLAMBDA / 2, P.DLAMBDA)
    assert lam.size == 1217
    mu = (1.0 + 0.5 * np.exp(-((lam - 1215.67) / 5.0) ** 2)
          + 0.2 * np.exp(-((lam - 1025.72) / 4.0) ** 2))
    M = 0.05 * gaussian_filter1d(rng.standard_normal((lam.size, k)), 4.0, axis=0)
    M = M / np.std(M) * 0.05
    log_omega = np.log(0.2) + 0.1 * gaussian_filter1d(rng.standard_normal(lam.size), 4.0)
    return dict(rest_wavelengths=lam, mu=mu, M=np.asfortranarray(M), log_omega=log_omega,
                log_c_0=np.log(P.INITIAL_C_0), log_tau_0=np.log(P.INITIAL_TAU_0),
                log_beta=np.log(P.INITIAL_BETA))


def halton(n: int, base: int) -> np.ndarray:
    """Radical-inverse sequence, points 1..n (point 0 = 0 is dropped)."""
    out = np.zeros(n)
    idx = np.arange(1, n + 1)
    f = 1.0 / base
    i = idx.copy()
    while np.any(i > 0):
        out += f * (i % base)
        i //= base
        f /= base
    return out


def make_samples(num_samples: int = P.NUM_DLA_SAMPLES) -> dict:
    offset = halton(num_samples, 2)
    log_nhi = P.UNIFORM_MIN_LOG_NHI + (P.UNIFORM_MAX_LOG_NHI - P.UNIFORM_MIN_LOG_NHI) * halton(num_samples, 3)
    return dict(offset_samples=offset, log_nhi_samples=log_nhi, nhi_samples=10.0 ** log_nhi)


def _voigt_absorption(lam, z, nhi, num_lines=3):
    """Absorption of one DLA on an observed grid (Voigt per Lyman line, voigt.c physics)."""
    from . import voigt_tables as VT
    tau = np.zeros_like(lam)
    for j in range(num_lines):
        v = lam * (VT.C_CGS / (VT.TRANSITION_WAVELENGTHS[j] * (1 + z)) / 1e8) - VT.C_CGS
        tau += VT.LEADING_CONSTANTS[j] * voigt_profile(v, VT.SIGMA, VT.LORENTZ_GAMMAS[j])
    return np.exp(-nhi * tau)


def make_spectrum(model: dict, q: int, z_qso: float | None = None, n_target: int | None = 800,
                  mask_fraction: float = 0.0, dla_fraction: float = 0.1,
                  blue_limit: float = 3600.0, seed_base: int = 416) -> dict:
    """One preloaded spectrum.  With ``n_target`` the in-range pixel count is exactly n_target
    (z_QSO = 2.56 and the BOSS 3600 A blue edge give 800)."""
    rng = np.random.default_rng(seed_base + q)
    if z_qso is None:
        z_qso = 2.56
    top = np.log10(P.MAX_LAMBDA * (1 + z_qso))
    if n_target is None:
        bottom = max(np.log10(P.MIN_LAMBDA * (1 + z_qso)), np.log10(blue_limit))
        n_target = int(np.floor((top - bottom) / P.PIXEL_SPACING))
    # pixel centres strictly inside the modelled range, plus one pixel redward (out of range)
    log_lam = top - P.PIXEL_SPACING * (np.arange(n_target, -1, -1) + 0.5)
    log_lam[-1] = top + 0.5 * P.PIXEL_SPACING
    lam = 10.0 ** log_lam
    rest = lam / (1 + z_qso)
    k = model["M"].shape[1]
    mu = np.interp(rest, model["rest_wavelengths"], model["mu"])
    Mi = np.stack([np.interp(rest, model["rest_wavelengths"], model["M"][:, j]) for j in range(k)], 1)
    om = np.exp(np.interp(rest, model["rest_wavelengths"], model["log_omega"]))
    noise = rng.uniform(0.01, 0.09, lam.size)
    cont = mu + Mi @ rng.standard_normal(k) + om * rng.standard_normal(lam.size)
    absorption = np.ones_like(lam)
    if rng.uniform() < dla_fraction:
        inr = (rest >= P.MIN_LAMBDA) & (rest <= P.MAX_LAMBDA)
        zmin = max(lam[inr].min() / P.LYA_WAVELENGTH - 1,
                   P.LYMAN_LIMIT * (1 + z_qso) / P.LYA_WAVELENGTH - 1 + P.MIN_Z_CUT)
        zmax = lam[inr].max() / P.LYA_WAVELENGTH - 1 - P.MAX_Z_CUT
        absorption = _voigt_absorption(lam, rng.uniform(zmin, zmax), 10 ** rng.uniform(20.3, 21.5))
    flux = absorption * cont + np.sqrt(noise) * rng.standard_normal(lam.size)
    mask = np.zeros(lam.size, dtype=bool)
    if mask_fraction > 0:
        mask = rng.uniform(size=lam.size) < mask_fraction
    return dict(wavelengths=lam, flux=flux, noise_variance=noise, pixel_mask=mask, z_qso=float(z_qso))


def make_spectra(model: dict, num: int, **kw) -> list[dict]:
    return [make_spectrum(model, q, **kw) for q in range(num)]


def make_dr12q_like_spectra(model: dict, num: int, seed: int = 12, mask_fraction: float = 0.05) -> list[dict]:
    """Variable z_QSO (so n ranges ~270-1250) and random in-range masks (parity set)."""
    rng = np.random.default_rng(seed)
    zs = rng.uniform(2.15, 4.5, num)
    return [make_spectrum(model, q, z_qso=float(z), n_target=None, mask_fraction=mask_fraction,
                          seed_base=9000) for q, z in enumerate(zs)]


def pack_spectra(spectra: list[dict]) -> dict:
    """Ragged list -> CSR arrays (the engine's input layout)."""
    lengths = np.array([s["wavelengths"].size for s in spectra], dtype=np.int64)
    offsets = np.zeros(len(spectra) + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    cat = lambda key, dt: np.ascontiguousarray(np.concatenate([np.asarray(s[key], dtype=dt) for s in spectra]))
    return dict(offsets=offsets, wavelengths=cat("wavelengths", np.float64), flux=cat("flux", np.float64),
                noise_variance=cat("noise_variance", np.float64), pixel_mask=cat("pixel_mask", np.uint8),
                z_qsos=np.array([s["z_qso"] for s in spectra], dtype=np.float64))


def write_processed_tree(base: str, model: dict, samples: dict, spectra: list, release: str = "dr12q",
                         training_set_name: str = "dr9q_minus_concordance",
                         dla_catalog_name: str = "dr9q_concordance", seed: int = 3) -> dict:
    """The reference's ``<base>/<release>/processed/`` directory (set_parameters.m:79-86) with every
    file process_qsos.m reads, for synthetic inputs: catalog.mat (z_qsos, filter_flags, in_dr9 and
    the containers.Map variables los_inds / dla_inds / z_dlas as structs keyed by catalogue name,
    build_catalogs.m:50-53), learned_qso_model_<set>.mat (learn_qso_model.m:113-123),
    dla_samples.mat (generate_dla_samples.m:59-63) and preloaded_qsos.mat (the four cell arrays of
    preload_qsos.m:77-80).  The catalogue doubles as the prior catalogue (release ==
    training_release).  Returns the index strings for ``process.run_process_qsos``."""
    from pathlib import Path

    from .matv73 import savemat73
    from .process import save_dla_samples
    rng = np.random.default_rng(seed)
    d = Path(base) / release / "processed"
    d.mkdir(parents=True, exist_ok=True)
    Q = len(spectra)
    z = np.array([s["z_qso"] for s in spectra], dtype=np.float64)
    dla = rng.uniform(size=Q) < 0.1
    z_dlas = [np.array([zq - rng.uniform(0.05, 0.5)]) if f else np.zeros(0) for zq, f in zip(z, dla)]
    savemat73(str(d / "catalog.mat"), dict(
        z_qsos=z, filter_flags=np.zeros(Q, np.uint8), in_dr9=rng.uniform(size=Q) < 0.8,
        los_inds={dla_catalog_name: np.ones(Q, bool)}, dla_inds={dla_catalog_name: dla},
        z_dlas={dla_catalog_name: z_dlas}))
    savemat73(str(d / f"learned_qso_model_{training_set_name}.mat"),
              {k: model[k] for k in ("rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0", "log_beta")})
    save_dla_samples(str(d / "dla_samples.mat"), samples)
    savemat73(str(d / "preloaded_qsos.mat"), dict(
        all_wavelengths=[s["wavelengths"] for s in spectra], all_flux=[s["flux"] for s in spectra],
        all_noise_variance=[s["noise_variance"] for s in spectra],
        all_pixel_mask=[np.asarray(s["pixel_mask"], dtype=bool) for s in spectra]))
    return dict(training_release=release, training_set_name=training_set_name,
                dla_catalog_name=dla_catalog_name,
                prior_ind=" prior_catalog.in_dr9 & prior_catalog.los_inds(dla_catalog_name) & "
                          "(prior_catalog.filter_flags == 0)",
                release=release, test_set_name=release, test_ind="(catalog.filter_flags == 0)")


def make_boss_coadd_columns(rng, z_qso: float, n_pixels: int = 4607):
    """fitsread columns (flux, loglam, ivar, and_mask) of a synthetic full BOSS coadd (3600-10400 A at
    1e-4 dex, read_spec.m:11-25's classes) for the ingest path: ~4% zero-ivar and ~3% BRIGHTSKY pixels,
    2% of spectra with a masked 1310-1325 A normalisation window (preload_qsos.m bit 3), 2% with no
    usable pixel in 911.75-1215.75 A (bit 4), 6% with NaN fluxes in the window."""
    ll = (np.log10(3600.0) + 1e-4 * np.arange(n_pixels)).astype(np.float32)
    f = rng.normal(2.0, 0.5, ll.size).astype(np.float32)
    iv = rng.uniform(1, 50, ll.size).astype(np.float32)
    iv[rng.uniform(size=ll.size) < 0.04] = 0
    am = np.where(rng.uniform(size=ll.size) < 0.03, 1 << 23, 0).astype(np.int32)
    rest = (10.0 ** ll.astype(np.float64)).astype(np.float32) / np.float32(1 + z_qso)
    win = np.flatnonzero((rest >= 1310) & (rest <= 1325))
    u = rng.uniform()
    if u < 0.02:
        iv[win] = 0
    elif u < 0.04:
        iv[(rest >= 911.75) & (rest <= 1215.75)] = 0
    elif u < 0.10 and win.size:
        f[win[::5]] = np.nan
    return f, ll, iv, am
