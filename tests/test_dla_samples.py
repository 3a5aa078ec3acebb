"""The checkers of generate_dla_samples (generate_dla_samples.m:1-63), pinned on the CPU before they judge
the device kernels (tests/test_gpu_dla_samples.py): oracle/dla_samples_closed_form.py (the algorithm
csrc/dla_samples.hip implements, vectorised in numpy) against MATLAB's documented Halton output, the
published definitions (RR2 digits, ksdensity's default bandwidth and Gaussian kernel, the mixture CDF
and its inverse) and oracle/dla_samples_oracle.py (MATLAB's order, step by step).  No sample file or
catalogue ships with the reference.  The product itself has no CPU path."""
import numpy as np
import pytest
from scipy import integrate, stats

from oracle import dla_samples_closed_form as D


def test_rr2_permutations():
    assert D.rr2_permutation(2).tolist() == [0, 1]
    assert D.rr2_permutation(3).tolist() == [0, 2, 1]          # 2-bit reversal 0,2,1,3 minus 3
    assert D.rr2_permutation(5).tolist() == [0, 4, 2, 1, 3]     # 3-bit reversal 0,4,2,6,1,5,3,7 below 5


def test_halton_rr2_first_points():
    h = D.halton_rr2(7)
    assert h[0].tolist() == [0.0, 0.0]                           # MATLAB haltonset starts at the origin
    np.testing.assert_allclose(h[:, 0], [0, .5, .25, .75, .125, .625, .375], rtol=0, atol=1e-16)
    # base 3 digits 1 -> 2, 2 -> 1: i=1 '1' -> 2/3; i=2 '2' -> 1/3; i=3 '10' -> 2/9; i=4 '11' -> 8/9;
    # i=5 '12' -> 1/3 + 2/9; i=6 '20' -> 1/9
    np.testing.assert_allclose(h[:, 1], [0, 2 / 3, 1 / 3, 2 / 9, 8 / 9, 5 / 9, 1 / 9], rtol=0, atol=1e-16)
    assert np.array_equal(D.halton_rr2(5, start=2), h[2:7])


def test_halton_rr2_matches_matlab_documented_output():
    """Pinned against MATLAB's own published output of the generator generate_dla_samples.m:8-9 calls:
    the MathWorks documentation example for haltonset/scramble,

        p = haltonset(3, 'Skip', 1e3, 'Leap', 1e2); p = scramble(p, 'RR2'); X0 = net(p, 4)

    prints (4 decimals) the rows below.  Skip 1e3 drops points 0..999 (point 0 is the origin) and Leap
    1e2 keeps every 101st point, i.e. points 1000, 1101, 1202, 1303 of the sequence in bases 2, 3, 5."""
    documented = np.array([[0.0928, 0.6950, 0.0029],
                           [0.6958, 0.2958, 0.8269],
                           [0.3013, 0.6497, 0.4141],
                           [0.9087, 0.7883, 0.2166]])
    pts = np.vstack([D.halton_rr2(1, bases=(2, 3, 5), start=1000 + 101 * j) for j in range(4)])
    assert np.array_equal(np.round(pts, 4), documented)


def test_ksdensity_matches_gaussian_kde_at_the_matlab_bandwidth():
    rng = np.random.default_rng(4)
    x = rng.normal(20.6, 0.35, 500)
    h = D.ksdensity_bandwidth(x)
    mad = np.median(np.abs(x - np.median(x)))
    assert h == pytest.approx(mad / 0.6745 * (4 / (3 * x.size)) ** 0.2, rel=1e-15)
    pts = np.linspace(20, 22, 1000)
    kde = stats.gaussian_kde(x, bw_method=h / np.std(x, ddof=1))
    np.testing.assert_allclose(D.ksdensity(x, pts), kde(pts), rtol=1e-12)


@pytest.fixture(scope="module")
def prior():
    rng = np.random.default_rng(5)
    log_nhis = np.r_[rng.normal(20.55, 0.3, 800), rng.uniform(20.3, 21.8, 200)]
    return D.ColumnDensityPrior(log_nhis), log_nhis


def test_prior_normalised_and_fit_integral(prior):
    p, _ = prior
    # the fitted density integrates to Z over [20, 25] (generate_dla_samples.m:37-38), by quadrature
    q, _ = integrate.quad(lambda t: float(p._fit_pdf(t)), 20, 25, epsabs=0, epsrel=1e-13, limit=200)
    assert p.Z == pytest.approx(q, rel=1e-12)
    assert p.cdf(20.0) == 0.0
    assert p.cdf(25.0) == pytest.approx(1.0, abs=1e-14)
    tt = np.linspace(20, 24, 41)
    for a, b in zip(tt[:-1], tt[1:]):
        q, _ = integrate.quad(lambda t: float(p.pdf(t)), a, b, epsabs=0, epsrel=1e-13, points=[23.0] if a < 23 < b else None)
        assert p.cdf(b) - p.cdf(a) == pytest.approx(q, rel=1e-10, abs=1e-15)


def test_inverse_cdf_roundtrip(prior):
    p, _ = prior
    u = D.halton_rr2(2000)[:, 1]
    t = p.inverse_cdf(u)
    assert t[0] == 20.0                                            # u = 0 at the origin point
    np.testing.assert_allclose(p.cdf(t), u, rtol=0, atol=1e-14)   # the CDF's own rounding
    assert np.all(np.diff(t[np.argsort(u)]) >= 0)


def test_generate_dla_samples_marginals(prior):
    _, log_nhis = prior
    out = D.generate_dla_samples(list(np.array_split(log_nhis, 50)) + [np.zeros(0)], num_dla_samples=4000)
    assert out["offset_samples"].shape == (4000,) and out["log_nhi_samples"].shape == (4000,)
    np.testing.assert_array_equal(out["nhi_samples"], 10.0 ** out["log_nhi_samples"])
    assert out["log_nhi_samples"].min() >= 20.0 and out["log_nhi_samples"].max() < 25.0
    # quasi-random samples reproduce the mixture CDF (Kolmogorov distance well below MC noise)
    p = D.ColumnDensityPrior(log_nhis)
    grid = np.linspace(20, 23.5, 200)
    emp = np.searchsorted(np.sort(out["log_nhi_samples"]), grid, side="right") / 4000
    assert np.max(np.abs(emp - p.cdf(grid))) < 2e-3
    assert np.max(np.abs(np.sort(out["offset_samples"]) - (np.arange(4000) + 0.5) / 4000)) < 1e-3


def test_matches_the_oracle_restatement(prior):
    """Closed form vs oracle/dla_samples_oracle.py, the step-by-step MATLAB-order restatement of
    generate_dla_samples.m (digit-by-digit RR2 Halton, ksdensity loop, QR polyfit, quadrature
    integral for Z and the CDF, bracket + Brent fzero): offsets bit for bit, log N_HI to 1e-11
    (the oracle's quadrature and root tolerances; the closed form integrates exactly)."""
    from oracle import dla_samples_oracle as DO
    _, log_nhis = prior
    cells = list(np.array_split(log_nhis, 40)) + [np.zeros(0)]
    got = D.generate_dla_samples(cells, num_dla_samples=300)
    want = DO.generate_dla_samples(cells, 300)
    np.testing.assert_array_equal(got["offset_samples"], want["offset_samples"])
    np.testing.assert_allclose(got["log_nhi_samples"], want["log_nhi_samples"], rtol=0, atol=1e-11)
    np.testing.assert_allclose(got["nhi_samples"], want["nhi_samples"], rtol=1e-10)


def test_product_has_no_cpu_path():
    """The product generator runs on the device only: without one it fails loudly (no numpy fallback)."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import dla_samples as DS
    if L.load().gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(L.GpdlaError, match="no HIP device"):
        DS.generate_dla_samples(np.r_[20.3, 20.6, 21.0], 10)
    with pytest.raises(L.GpdlaError, match="no HIP device"):
        DS.halton_rr2(4)
