"""The C++ OpenMP restatement (oracle/cpu_ref.cpp; the CPU baseline of bench.py) against the
numpy oracle and scipy: its own Faddeeva function against scipy.special.wofz / voigt_profile
over the Lyman-line argument domain, the MEX voigt and log_mvnpdf_low_rank
against the golden fixtures, whole sample log-likelihoods against gpdla_oracle, and the
sanitizer self-tests (ASan / UBSan builds of the host code)."""
import shutil
import subprocess

import numpy as np
import pytest
from scipy.special import voigt_profile, wofz

from gp_dla_detection_amd import synthetic as syn
from oracle import cpu_ref as CR
from oracle import gpdla_oracle as O


@pytest.fixture(scope="module", autouse=True)
def built():
    if shutil.which("make") is None or shutil.which("g++") is None:
        pytest.skip("no host C++ toolchain")
    CR.build()


def test_faddeeva_against_scipy():
    # x over core, transition (|x| = 6) and wings up to the 1.6e4 of the spectral range; y the
    # Lyman-line dampings gamma / (sigma sqrt 2) and a few larger values
    xs = np.concatenate([np.linspace(0, 10, 1001), np.geomspace(10, 2e4, 400), [7.999999, 8.0, 8.000001]])
    for y in (4.717e-4, 1.205e-4, 4.895e-5, 1e-6, 0.01, 0.05):
        ref = wofz(xs + 1j * y)
        got = np.array([CR.faddeeva_w(x, y) for x in xs])
        assert np.max(np.abs(got.real - ref.real) / np.abs(ref.real)) < 2e-13, y
        assert np.max(np.abs(got.imag - ref.imag) / np.maximum(np.abs(ref.imag), 1e-300)) < 2e-13, y
        got_neg = np.array([CR.faddeeva_w(-x, y) for x in xs[::37]])
        np.testing.assert_allclose(got_neg, np.conj(got[::37]), rtol=0, atol=0)


def test_voigt_and_mvn_match_golden(golden_dir):
    g = np.load(golden_dir / "voigt.npz")
    for i in range(g["z"].size):
        ref = g[f"out_{i}"]
        got = CR.voigt(g[f"lam_{i}"], g["z"][i], g["N"][i], int(g["num_lines"][i]))
        assert np.max(np.abs(got - ref)) < 1e-12
        big = ref > 1e-200
        assert np.max(np.abs(got[big] - ref[big]) / ref[big]) < 1e-9
    g = np.load(golden_dir / "mvn.npz")
    for i in range(4):
        got = CR.log_mvnpdf_low_rank(g[f"y_{i}"], g[f"mu_{i}"], g[f"M_{i}"], g[f"d_{i}"])
        ref = float(g[f"out_{i}"])
        assert abs(got - ref) <= 1e-10 * max(1, abs(ref))


@pytest.mark.parametrize("k", [20, 50])
def test_sample_lls_match_oracle(k):
    model = syn.make_model(k=k)
    samples = syn.make_samples(48)
    for s in syn.make_dr12q_like_spectra(model, 2, seed=k, mask_fraction=0.05):
        prep = O.prepare_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"], s["z_qso"], model)
        zs = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * samples["offset_samples"]
        ref = np.array([O.sample_log_likelihood(prep, z, N, 3) for z, N in zip(zs, samples["nhi_samples"])])
        got = CR.sample_lls(prep, samples["offset_samples"], samples["nhi_samples"], 3, nthreads=2)
        assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)) < 1e-10


def test_voigt_profile_definition():
    # libcerf voigt(x, sigma, gamma) == scipy.special.voigt_profile
    lam = 10 ** (np.log10(4000.0) + 1e-4 * np.arange(-3, 400))
    got = CR.voigt(lam, 2.29, 10 ** 21.3, 3)
    ref = O.voigt_mex(lam, 2.29, 10 ** 21.3, 3)
    np.testing.assert_allclose(got, ref, rtol=1e-11, atol=1e-300)
    assert voigt_profile(1.0, 1.0, 0.5) == pytest.approx(wofz((1 + 0.5j) / np.sqrt(2)).real / np.sqrt(2 * np.pi))


@pytest.mark.parametrize("target", ["selftest-asan", "selftest-ubsan"])
def test_sanitizer_builds(target):
    r = subprocess.run(["make", "-s", "-C", str(CR.HERE), target], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu_ref selftest ok" in r.stdout
