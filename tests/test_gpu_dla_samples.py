"""GPU parity of the DLA-sample generator (generate_dla_samples.m:8-57 on the device, csrc/dla_samples.hip;
SURVEY.md 8f-2) against its two checkers:

* oracle/dla_samples_oracle.py -- MATLAB's order step by step (digit-by-digit RR2 Halton, ksdensity
  loop, QR polyfit, quadrature integral, bracket + Brent fzero), one sample at a time: the Halton
  coordinates of every sample bit for bit, log10 N_HI on a strided subset (its quadrature roots are
  slow) to 1e-12 absolute;
* oracle/dla_samples_closed_form.py -- the same closed-form algorithm vectorised in numpy: every
  sample's log10 N_HI to 1e-12 absolute, the fit and its normaliser.

At S = 10^4 (BASELINE configs[1]-[3]) and 10^5 (configs[4]).  The Halton points also keep MATLAB's own
documented haltonset/scramble output.  Parity is pinned by the published algorithms (no catalogue or
sample file ships with the reference)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import dla_samples as DS  # noqa: E402
from gp_dla_detection_amd import matv73 as M  # noqa: E402
from gp_dla_detection_amd import process as PR  # noqa: E402
from oracle import dla_samples_closed_form as CF  # noqa: E402
from oracle import dla_samples_oracle as DO  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _catalogue(seed=5, n=1000):
    rng = np.random.default_rng(seed)
    return np.r_[rng.normal(20.55, 0.3, int(0.8 * n)), rng.uniform(20.3, 21.8, n - int(0.8 * n))]


def test_halton_rr2_matches_matlab_documented_output():
    """MATLAB's haltonset/scramble documentation example (p = haltonset(3, 'Skip', 1e3, 'Leap', 1e2);
    p = scramble(p, 'RR2'); net(p, 4)): points 1000, 1101, 1202, 1303 in bases 2, 3, 5, as printed."""
    documented = np.array([[0.0928, 0.6950, 0.0029],
                           [0.6958, 0.2958, 0.8269],
                           [0.3013, 0.6497, 0.4141],
                           [0.9087, 0.7883, 0.2166]])
    pts = DS.halton_rr2(4, bases=(2, 3, 5), start=1000, stride=101)
    assert np.array_equal(np.round(pts, 4), documented)


@pytest.mark.parametrize("S", [10_000, 100_000])
def test_halton_bit_exact(S):
    got = DS.halton_rr2(S)
    want = np.stack([[DO.halton_rr2_point(i, 2) for i in range(S)], [DO.halton_rr2_point(i, 3) for i in range(S)]], 1)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert np.array_equal(got, CF.halton_rr2(S))
    # other bases, a start and a stride (the Skip / Leap of haltonset)
    got5 = DS.halton_rr2(3000, bases=(5, 7, 11, 13), start=777, stride=3)
    want5 = np.array([[DO.halton_rr2_point(777 + 3 * j, b) for b in (5, 7, 11, 13)] for j in range(3000)])
    assert np.array_equal(got5, want5)


@pytest.mark.parametrize("S", [10_000, 100_000])
def test_generate_dla_samples_matches_both_checkers(S):
    log_nhis = _catalogue()
    cells = list(np.array_split(log_nhis, 60)) + [np.zeros(0)]
    got = DS.generate_dla_samples(cells, S)
    cf = CF.generate_dla_samples(cells, S)
    assert np.array_equal(got["offset_samples"], cf["offset_samples"])
    np.testing.assert_allclose(got["log_nhi_samples"], cf["log_nhi_samples"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(got["nhi_samples"], 10.0 ** got["log_nhi_samples"], rtol=4e-16)
    # the fit against the closed form's (np.polyfit's least squares; the device solves by QR as MATLAB)
    prior = CF.ColumnDensityPrior(log_nhis)
    np.testing.assert_allclose(got["fit"]["coeffs"], prior.coeffs, rtol=1e-9)
    assert got["fit"]["Z"] == pytest.approx(prior.Z, rel=1e-12)
    assert got["fit"]["bandwidth"] == CF.ksdensity_bandwidth(log_nhis)
    # MATLAB's order on a strided subset of the samples (quadrature + Brent per sample)
    sub = np.arange(0, S, S // 150)
    mo = DO.generate_dla_samples(cells, S, sample_indices=sub)
    assert np.array_equal(got["offset_samples"].view(np.uint64), mo["offset_samples"].view(np.uint64))
    np.testing.assert_allclose(got["log_nhi_samples"][sub], mo["log_nhi_samples"][sub], rtol=0, atol=1e-12)
    # inverse-transform sanity: the prior's CDF at each sample is its Halton coordinate
    u = CF.halton_rr2(S)[:, 1]
    np.testing.assert_allclose(prior.cdf(got["log_nhi_samples"]), u, rtol=0, atol=1e-13)   # np.polyfit vs QR coefficients
    assert got["log_nhi_samples"][0] == 20.0 and np.all(got["log_nhi_samples"] < 25.0)


def test_non_concave_fit_takes_the_quadrature():
    """A catalogue whose log-density fit is convex (mass at both ends of the fit range) integrates by
    Gauss-Legendre on the device; against the closed-form checker's adaptive quadrature."""
    rng = np.random.default_rng(9)
    log_nhis = np.r_[rng.uniform(19.8, 22.2, 2000), rng.normal(20.1, 0.15, 200), rng.normal(21.9, 0.15, 200)]
    prior = CF.ColumnDensityPrior(log_nhis)
    assert prior.coeffs[0] > 0                      # c2 = 0.206: U-shaped, Z = 7.86 over [20, 25]
    got = DS.generate_dla_samples(log_nhis, 3000)
    want = CF.generate_dla_samples(log_nhis, 3000)
    np.testing.assert_allclose(got["log_nhi_samples"], want["log_nhi_samples"], rtol=0, atol=1e-10)
    assert got["fit"]["Z"] == pytest.approx(prior.Z, rel=1e-11)
    u = CF.halton_rr2(3000)[:, 1]
    np.testing.assert_allclose(prior.cdf(got["log_nhi_samples"]), u, rtol=0, atol=1e-12)


def test_errors_are_loud():
    with pytest.raises(ValueError):
        DS.generate_dla_samples([20.5], 10)
    with pytest.raises(L.GpdlaError, match="non-finite"):
        DS.generate_dla_samples(np.r_[20.5, np.nan, 20.7], 10)
    with pytest.raises(L.GpdlaError, match="base"):
        DS.halton_rr2(4, bases=(1, 3))
    out = DS.generate_dla_samples(_catalogue(), 0)
    assert out["log_nhi_samples"].size == 0 and out["fit"]["Z"] > 0


def test_run_generate_dla_samples_files(tmp_path):
    """The script on files: catalog.mat (log_nhis keyed by catalogue name) in, dla_samples.mat out, read
    back by the loader process_qsos uses (process_qsos.m:38-40)."""
    log_nhis = _catalogue(seed=6)
    d = tmp_path / "dr12q" / "processed"
    d.mkdir(parents=True)
    cells = list(np.array_split(log_nhis, 100))
    M.savemat73(str(d / "catalog.mat"), dict(log_nhis=dict(dr9q_concordance=cells)))
    out = DS.run_generate_dla_samples(str(tmp_path), "dr12q", "dr9q_concordance", num_dla_samples=500)
    r = M.loadmat73(str(d / "dla_samples.mat"))
    assert r["offset_samples"].shape == (1, 500)                   # MATLAB row (h5py (500, 1))
    np.testing.assert_array_equal(r["log_nhi_samples"].ravel(), out["log_nhi_samples"])
    assert float(r["alpha"][0, 0]) == 0.9
    s = PR.load_dla_samples(str(d / "dla_samples.mat"))
    np.testing.assert_array_equal(s["nhi_samples"], out["nhi_samples"])
    np.testing.assert_allclose(out["log_nhi_samples"], CF.generate_dla_samples(cells, 500)["log_nhi_samples"],
                               rtol=0, atol=1e-12)


def test_generate_reports_its_kernel_times():
    DS.generate_dla_samples(np.r_[np.linspace(20.3, 21.5, 50), np.linspace(20.4, 22.0, 30)], 1000)
    ms = L.last_call_kernel_ms()
    assert len(ms) == 3 and all(0 < t < 1000 for t in ms)          # KDE, Halton, inverse CDF
