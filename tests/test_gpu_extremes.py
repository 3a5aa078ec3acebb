"""Extreme inputs on the fast paths of the batched sweeps, against the oracle.

The fused fp64 sweep (kernels.hip likelihood_kernel) evaluates exp(N tot) with a 128-entry table and
no clamp on its main path: only a core-zone lane can take N tot below the table's index range, and
its fix-up clamps there; a wave holding an N_HI whose wings alone could get there clamps every lane
through a wave-uniform branch.  Its per-pixel reciprocals 1/d are batched over a chunk's 4 steps
(one v_rcp_f64 of the product of the d's), with a fallback to 4 reciprocals when that product
leaves [2^-1000, 2^1000].  These tests drive both rare branches:

* column densities up to 1e30 (the reference's samples stop at 1e23; generate_dla_samples.m:20-53
  takes any prior), on some sample blocks only, so clamped and unclamped waves run side by side;
* noise variances and model variances scaled by 1e-80 and 1e+80, so the product of four d's
  under- or overflows on every chunk.

Every kernel path is compared with oracle/gpdla_oracle.py (process_qsos.m:184-197, voigt.c:282-299,
log_mvnpdf_low_rank.m:5-33): 1e-9 relative for the fp64 paths, 1e-8 for the 32-bit int8 contraction
and 5e-7 for the 24-bit one (their regression bars elsewhere in the suite).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402

PATHS = (("auto", 1e-9), ("panel_gemm", 1e-9), ("fused_i8", 1e-8), ("panel_gemm_i8", 1e-8),
         ("panel_gemm_i8_24", 5e-7))


@pytest.fixture(scope="module", autouse=True)
def require_device():
    lib = L.load()
    assert lib.gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _rel_err(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))


def _check(model, spectra, samples, paths=PATHS):
    from oracle import gpdla_oracle as O
    refs = [O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"], s["z_qso"],
                               model, samples["offset_samples"], samples["nhi_samples"]) for s in spectra]
    packed = syn.pack_spectra(spectra)
    for path, tol in paths:
        with Engine(model, samples, set_parameters(k=model["M"].shape[1]), path=path) as eng:
            out = eng.process(packed)
        for q, ref in enumerate(refs):
            sll = out["sample_log_likelihoods_dla"][q]
            assert np.isfinite(sll).all(), path
            assert _rel_err(sll, ref["sample_log_likelihoods_dla"]) < tol, (path, q)
            assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < tol, (path, q)
            assert _rel_err(out["log_likelihoods_dla"][q], ref["log_likelihood_dla"]) < tol, (path, q)


def test_huge_column_densities_clamp_wave_uniformly():
    """log N_HI 27..30 on the samples with offsets in [0.4, 0.7) (a few 64-sample blocks, sorted by
    offset in the engine), the reference's 20..23 elsewhere."""
    model = syn.make_model(k=20, seed=5)
    spectra = [syn.make_spectrum(model, q, z_qso=z, n_target=None, mask_fraction=0.05)
               for q, z in enumerate((2.6, 3.4))]
    base = syn.make_samples(320)
    off = base["offset_samples"]
    log_nhi = base["log_nhi_samples"].copy()
    big = (off >= 0.4) & (off < 0.7)
    log_nhi[big] = 27.0 + 3.0 * ((np.arange(big.sum()) * 0.618) % 1.0)
    samples = dict(offset_samples=off, log_nhi_samples=log_nhi, nhi_samples=10.0 ** log_nhi)
    _check(model, spectra, samples)


@pytest.mark.parametrize("scale", [1e-80, 1e80])
def test_variances_out_of_the_batched_reciprocal_range(scale):
    """The whole problem in other units: flux, mu and M times sqrt(scale), sigma^2 and omega^2 times
    scale.  Then d = omega^2 a^2 + sigma^2 ~ 1e-80 (or 1e80), the product of a chunk's four d's is not
    a normal double and every wave takes the per-step reciprocals."""
    base = syn.make_model(k=20, seed=6)
    model = dict(base, log_omega=base["log_omega"] + 0.5 * np.log(scale), mu=base["mu"] * np.sqrt(scale),
                 M=np.asfortranarray(base["M"] * np.sqrt(scale)))
    spectra = []
    for q, z in enumerate((2.7, 3.1)):
        s = syn.make_spectrum(base, q, z_qso=z, n_target=None, mask_fraction=0.05)
        s["noise_variance"] = s["noise_variance"] * scale
        s["flux"] = s["flux"] * np.sqrt(scale)
        spectra.append(s)
    samples = syn.make_samples(192)
    _check(model, spectra, samples)


@pytest.mark.parametrize("e", [-266, 266])
def test_power_of_two_units_are_exact(e):
    """The same problem with sigma^2, omega^2 times 2^e and flux, mu, M times 2^(e/2): prep_kernel
    (kernels.hip) evaluates it in the original units again (its exponents leave +-60), so every
    sample log-likelihood is the unscaled one plus -n e ln2 / 2 (log det D shifts by n e ln 2).  Exact
    but for omega^2, which the model carries as log omega (exp(2 log omega) of the shifted log is within
    3e-14 of 2^e omega^2), hence rtol 1e-11 rather than rounding level."""
    base = syn.make_model(k=20, seed=7)
    scaled = dict(base, log_omega=base["log_omega"] + 0.5 * e * np.log(2.0), mu=np.ldexp(base["mu"], e // 2),
                  M=np.asfortranarray(np.ldexp(base["M"], e // 2)))
    spectra = [syn.make_spectrum(base, q, z_qso=z, n_target=None, mask_fraction=0.05)
               for q, z in enumerate((2.5, 3.3))]
    spectra_s = [dict(s, flux=np.ldexp(s["flux"], e // 2), noise_variance=np.ldexp(s["noise_variance"], e))
                 for s in spectra]
    samples = syn.make_samples(130)
    for path, _ in PATHS:
        outs = []
        for model, sp in ((base, spectra), (scaled, spectra_s)):
            with Engine(model, samples, set_parameters(k=20), path=path) as eng:
                outs.append(eng.process(syn.pack_spectra(sp)))
        n = outs[0]["num_pixels"].astype(float)
        shift = -0.5 * n * e * np.log(2.0)
        np.testing.assert_allclose(outs[1]["sample_log_likelihoods_dla"],
                                   outs[0]["sample_log_likelihoods_dla"] + shift[:, None], rtol=1e-11, atol=0)
        np.testing.assert_allclose(outs[1]["log_likelihoods_no_dla"], outs[0]["log_likelihoods_no_dla"] + shift,
                                   rtol=1e-11, atol=0)


def test_invalid_column_densities_rejected():
    """Negative, NaN and infinite N_HI are refused at engine creation (GPDLA_EINVAL), before any kernel
    runs: the sweeps' exp relies on N >= 0 and finite."""
    model = syn.make_model(k=20, seed=8)
    base = syn.make_samples(16)
    for bad in (-1e20, np.nan, np.inf):
        nhi = base["nhi_samples"].copy()
        nhi[5] = bad
        samples = dict(base, nhi_samples=nhi)
        with pytest.raises(L.GpdlaError, match="column densities"):
            Engine(model, samples, set_parameters(k=20))


def test_scaled_and_unscaled_spectra_in_one_batch():
    """prep_kernel picks the unit exponent per spectrum, from its sigma^2 and the model's largest
    omega^2: a batch with one spectrum whose noise variances are 2^-100 times the usual (flux and model
    unchanged, so d spans ~2^100 within it and r'D^-1 r ~ 1e30) beside ordinary ones, every path against
    the oracle on the same inputs.  At 2^-200 (d spanning ~2^200) only the fused fp64 sweep keeps prod d
    in range (one factor at a time when four leave it); the panel paths' weights kernels renormalise
    once per 16 pixels and support a span of ~2^120.  fp64 paths only: with d
    spanning 2^100, r'D^-1 r and u'B^-1 u are ~1e44 and cancel to ~1e30, far below the int8
    contraction's error bound (relative to each slot's static scale)."""
    model = syn.make_model(k=20, seed=9)
    spectra = [syn.make_spectrum(model, q, z_qso=z, n_target=None, mask_fraction=0.05)
               for q, z in enumerate((2.4, 2.9, 3.5))]
    for e, paths in ((-100, (("auto", 1e-9), ("panel_gemm", 1e-9))), (-200, (("auto", 1e-9),))):
        sp = list(spectra)
        sp[1] = dict(sp[1], noise_variance=np.ldexp(sp[1]["noise_variance"], e))
        _check(model, sp, syn.make_samples(100), paths)
