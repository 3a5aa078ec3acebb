"""The oracle itself: pinned against independent implementations of the same mathematics
(no reference golden vectors exist -- SURVEY.md section 4) and against the committed fixtures."""
import numpy as np
import pytest
from scipy.special import voigt_profile, wofz
from scipy.stats import multivariate_normal

from oracle import gpdla_oracle as O


def test_libcerf_voigt_definition():
    # libcerf voigt(x, sigma, gamma) = Re w((x + i gamma)/(sigma sqrt 2)) / (sigma sqrt(2 pi))
    x = np.linspace(-3e7, 3e7, 101)
    for g in O.LORENTZ_GAMMAS[:5]:
        ref = np.real(wofz((x + 1j * g) / (O.SIGMA * np.sqrt(2)))) / (O.SIGMA * np.sqrt(2 * np.pi))
        np.testing.assert_allclose(O.libcerf_voigt(x, O.SIGMA, g), ref, rtol=1e-13, atol=0)
    assert abs(voigt_profile(1, 1, 0.5) - 0.20017963759083915) < 1e-15  # SURVEY.md 8c probe


def test_voigt_tables_reproduce_their_formulas():
    # voigt.c:141-240 comments: b = sqrt(2kT/m_p), sigma = b/sqrt 2,
    # leading = pi e^2 f lambda / (m_e c), gammas = Gamma lambda / (4 pi), profile normalised
    kB, mp, me, e = 1.38064852e-16, 1.672621898e-24, 9.10938356e-28, 4.803204672997660e-10
    sigma = np.sqrt(2 * kB * 1e4 / mp) / np.sqrt(2)
    assert abs(sigma / O.SIGMA - 1) < 1e-15
    lc = np.pi * e * e * O.OSCILLATOR_STRENGTHS * O.TRANSITION_WAVELENGTHS / (me * O.C_CGS)
    np.testing.assert_allclose(lc, O.LEADING_CONSTANTS, rtol=2e-15)
    gam = O.TRANSITION_RATES * O.TRANSITION_WAVELENGTHS / (4 * np.pi)
    np.testing.assert_allclose(gam, O.LORENTZ_GAMMAS, rtol=2e-15)
    pixel_sigma = 1 / (2000 * 2 * np.sqrt(2 * np.log(2)) * (10 ** 1e-4 - 1))
    ip = np.exp(-0.5 * np.arange(-3, 4) ** 2 / pixel_sigma ** 2)
    np.testing.assert_allclose(ip / ip.sum(), O.INSTRUMENT_PROFILE, rtol=1e-14)


def test_voigt_mex_shape_and_limits():
    lam = 10 ** np.arange(np.log10(3600), np.log10(4300), 1e-4)
    out = O.voigt_mex(lam, 2.2, 1e20, 3)
    assert out.shape == (lam.size - 6,)
    assert np.all((out >= 0) & (out <= 1))
    assert np.all(O.voigt_mex(lam, 2.2, 0.0, 3) == np.sum(O.INSTRUMENT_PROFILE * 0 + O.INSTRUMENT_PROFILE))


def test_log_mvnpdf_low_rank_matches_dense():
    rng = np.random.default_rng(0)
    for n, k in ((50, 3), (300, 20)):
        M = 0.1 * rng.standard_normal((n, k))
        mu = rng.standard_normal(n)
        d = rng.uniform(0.02, 0.3, n)
        y = mu + M @ rng.standard_normal(k) + np.sqrt(d) * rng.standard_normal(n)
        ref = multivariate_normal(mu, M @ M.T + np.diag(d)).logpdf(y)
        assert abs(O.log_mvnpdf_low_rank(y, mu, M, d) - ref) < 1e-10 * max(1, abs(ref))


def test_golden_mvn_fixture(golden_dir):
    g = np.load(golden_dir / "mvn.npz")
    for i in range(4):
        got = O.log_mvnpdf_low_rank(g[f"y_{i}"], g[f"mu_{i}"], g[f"M_{i}"], g[f"d_{i}"])
        assert abs(got - float(g[f"out_{i}"])) <= 1e-12 * abs(float(g[f"out_{i}"]))
        dense = multivariate_normal(g[f"mu_{i}"], g[f"M_{i}"] @ g[f"M_{i}"].T + np.diag(g[f"d_{i}"]))
        assert abs(dense.logpdf(g[f"y_{i}"]) - got) < 1e-9 * abs(got)


def test_golden_voigt_fixture(golden_dir):
    g = np.load(golden_dir / "voigt.npz")
    for i in range(g["z"].size):
        got = O.voigt_mex(g[f"lam_{i}"], g["z"][i], g["N"][i], int(g["num_lines"][i]))
        np.testing.assert_array_equal(got, g[f"out_{i}"])


def test_golden_process_fixture_and_cddf_invariant(golden_dir):
    g = np.load(golden_dir / "process.npz")
    model = {k: g[k] for k in ("rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0", "log_beta")}
    q = 3
    a, b = g["offsets"][q], g["offsets"][q + 1]
    res = O.process_spectrum(g["wavelengths"][a:b], g["flux"][a:b], g["noise_variance"][a:b],
                             g["pixel_mask"][a:b].astype(bool), g["z_qsos"][q], model,
                             g["offset_samples"][:16], g["nhi_samples"][:16], num_lines=3)
    np.testing.assert_allclose(res["sample_log_likelihoods_dla"],
                               g["reference_sample_log_likelihoods_dla"][q, :16], rtol=1e-13)
    assert abs(res["log_likelihood_no_dla"] - g["reference_log_likelihood_no_dla"][q]) < 1e-9
    # calc_cddf.py:246: sum_s exp(ll_s - (ll_dla + log S)) == 1 (by construction, to rounding)
    for mode in ("reference", "unmasked"):
        sll = g[f"{mode}_sample_log_likelihoods_dla"]
        lld = g[f"{mode}_log_likelihood_dla"]
        S = sll.shape[1]
        tot = np.exp(sll - (lld[:, None] + np.log(S))).sum(axis=1)
        np.testing.assert_allclose(tot, 1.0, atol=1e-12)


def test_absorption_quirk_changes_masked_spectra(golden_dir):
    g = np.load(golden_dir / "process.npz")
    n, m = g["reference_n"], g["reference_m"]
    masked = n < m
    assert masked.any() and (~masked).any()
    ref, unm = g["reference_sample_log_likelihoods_dla"], g["unmasked_sample_log_likelihoods_dla"]
    # identical when no in-range pixel is masked (process_qsos.m:180 quirk is then a no-op)
    np.testing.assert_array_equal(ref[~masked], unm[~masked])
    assert np.all(np.abs(ref[masked] - unm[masked]).max(axis=1) > 1e-6)
