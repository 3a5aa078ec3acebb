"""GP null-model training objective (spectrum_loss.m / objective.m / learn_qso_model.m;
SURVEY.md 8f-3).  CPU: the oracle restatement pinned by a dense Gaussian log-density and by
finite differences of its own f (the reference's gradient formulas are checked, not assumed),
plus the host preprocessing.  GPU (-m gpu): libgpdla's objective kernels against the oracle."""
import numpy as np
import pytest
from scipy.stats import multivariate_normal

from gp_dla_detection_amd import synthetic as syn
from gp_dla_detection_amd import training as T
from oracle import gpdla_oracle as O


def _problem(n=60, k=4, seed=0):
    rng = np.random.default_rng(seed)
    M = 0.3 * rng.standard_normal((n, k))
    omega2 = rng.uniform(0.01, 0.05, n)
    y = rng.standard_normal(n) * 0.3
    lya = rng.uniform(2.5, 4.5, n)
    nv = rng.uniform(0.01, 0.1, n)
    return y, lya, nv, M, omega2, 0.1, 0.0023, 3.65


def test_oracle_spectrum_loss_is_the_gaussian_nll():
    y, lya, nv, M, om2, c0, t0, b = _problem()
    nlp = O.spectrum_loss(y, lya, nv, M, om2, c0, t0, b)[0]
    sf = 1 - np.exp(-t0 * lya ** b) + c0
    d = nv + om2 * sf ** 2
    ref = -multivariate_normal(np.zeros(y.size), M @ M.T + np.diag(d)).logpdf(y)
    assert nlp == pytest.approx(ref, rel=1e-12)


def test_oracle_gradient_matches_finite_differences():
    """Central differences of f in x = [M(:); log omega; log c0; log tau0; log beta]."""
    y, lya, nv, M, om2, c0, t0, b = _problem(n=40, k=3, seed=1)
    n, k = M.shape
    x = np.concatenate([M.ravel(order="F"), 0.5 * np.log(om2), [np.log(c0), np.log(t0), np.log(b)]])

    def f(x):
        Mx = x[:n * k].reshape(n, k, order="F")
        return O.spectrum_loss(y, lya, nv, Mx, np.exp(2 * x[n * k:n * (k + 1)]), np.exp(x[-3]),
                               np.exp(x[-2]), np.exp(x[-1]))[0]

    _, dM, dlo, dc, dt, db = O.spectrum_loss(y, lya, nv, M, om2, c0, t0, b)
    g = np.concatenate([dM.ravel(order="F"), dlo, [dc, dt, db]])
    h = 1e-6
    fd = np.array([(f(x + h * e) - f(x - h * e)) / (2 * h) for e in np.eye(x.size)])
    np.testing.assert_allclose(g, fd, rtol=1e-6, atol=1e-7)


def test_oracle_objective_sums_spectra_and_adds_priors_to_g_only():
    rng = np.random.default_rng(2)
    Q, Pn, k = 4, 30, 3
    y = rng.standard_normal((Q, Pn)) * 0.3
    y[rng.uniform(size=y.shape) < 0.2] = np.nan
    lya = rng.uniform(2.5, 4.5, (Q, Pn))
    nv = rng.uniform(0.01, 0.1, (Q, Pn))
    x = np.concatenate([0.3 * rng.standard_normal(Pn * k), np.log(0.15) + 0.1 * rng.standard_normal(Pn),
                        [np.log(0.1), np.log(0.003), np.log(3.5)]])
    f, g = O.objective(x, y, lya, nv)
    M = x[:Pn * k].reshape(Pn, k, order="F")
    tot = 0.0
    for i in range(Q):
        ind = ~np.isnan(y[i])
        tot += O.spectrum_loss(y[i, ind], lya[i, ind], nv[i, ind], M[ind], np.exp(2 * x[Pn * k:Pn * (k + 1)])[ind],
                               0.1, 0.003, 3.5)[0]
    assert f == pytest.approx(tot, rel=1e-14)
    # prior gradient terms (objective.m:60-71) at tau0 = 0.003, beta = 3.5
    _, g0 = O.objective(x, np.full_like(y, np.nan), lya, nv)
    assert g0[-2] == pytest.approx(0.003 * (0.003 - 0.0023) / 0.0007 ** 2, rel=1e-12)
    assert g0[-1] == pytest.approx(3.5 * (3.5 - 3.65) / 0.21 ** 2, rel=1e-12)


def test_interp1_matlab_semantics():
    x = np.array([3.0, 1.0, 2.0])
    v = np.array([30.0, 10.0, 20.0])
    xq = np.array([0.5, 1.0, 1.5, 2.0, 3.0, 3.5])
    got = T._interp1(x, v, xq)
    assert np.isnan(got[0]) and np.isnan(got[-1])
    np.testing.assert_allclose(got[1:5], [10, 15, 20, 30])


def test_pairwise_pca_without_missing_is_pca():
    rng = np.random.default_rng(3)
    X = rng.standard_normal((200, 12)) @ rng.standard_normal((12, 12))
    coef, lat = T.pairwise_pca(X, 4)
    w, V = np.linalg.eigh(np.cov(X, rowvar=False))
    np.testing.assert_allclose(lat, w[::-1][:4], rtol=1e-10)
    np.testing.assert_allclose(np.abs(coef), np.abs(V[:, ::-1][:, :4]), atol=1e-8)


def test_pairwise_pca_missing_values_hand_checked():
    """Hand-computed pca(X, 'rows', 'pairwise'): columns centred by nanmean (3, 16/3), then the
    non-centred pairwise covariance over common rows: C = [[8/2, 8/1], [8/1, (168/9)/2]]."""
    X = np.array([[1.0, 2.0], [3.0, np.nan], [5.0, 6.0], [np.nan, 8.0]])
    coef, lat = T.pairwise_pca(X, 2)
    np.testing.assert_allclose(lat, [(20 + 8 * np.sqrt(10)) / 3, (20 - 8 * np.sqrt(10)) / 3], rtol=1e-13)
    w, V = np.linalg.eigh(np.array([[4.0, 8.0], [8.0, 28.0 / 3.0]]))
    np.testing.assert_allclose(np.abs(coef), np.abs(V[:, ::-1]), atol=1e-13)
    assert np.all(coef[np.argmax(np.abs(coef), axis=0), [0, 1]] > 0)


def test_prepare_training_data_shapes():
    model = syn.make_model(k=4)
    spectra = syn.make_dr12q_like_spectra(model, 6, seed=4)
    z = [s["z_qso"] for s in spectra]
    rest, mu, y, lya, nv = T.prepare_training_data(spectra, z)
    assert rest.size == 1217 and y.shape == (6, 1217) and lya.shape == y.shape
    assert np.array_equal(np.isnan(y), np.isnan(nv) | np.isnan(y))
    assert np.all(nv[~np.isnan(nv)] <= 1.0)
    x0, M0, lo0 = T.initial_parameters(y, 4)
    assert x0.size == 5 * 1217 + 3 and M0.shape == (1217, 4)


# ------------------------------------------------------------------------------- GPU
def _training_set(Q=12, k=6, seed=5):
    model = syn.make_model(k=k)
    spectra = syn.make_dr12q_like_spectra(model, Q, seed=seed)
    z = [s["z_qso"] for s in spectra]
    rest, mu, y, lya, nv = T.prepare_training_data(spectra, z)
    x0, _, _ = T.initial_parameters(y, k)
    x0 = np.nan_to_num(x0, nan=np.log(0.1))
    return y, lya, nv, x0, k


@pytest.mark.gpu
def test_gpu_spectrum_loss_matches_oracle():
    y, lya, nv, M, om2, c0, t0, b = _problem(n=700, k=20, seed=6)
    got = T.spectrum_loss(y, lya, nv, M, om2, c0, t0, b)
    ref = O.spectrum_loss(y, lya, nv, M, om2, c0, t0, b)
    assert got[0] == pytest.approx(ref[0], rel=1e-11)
    np.testing.assert_allclose(got[1], ref[1], rtol=1e-9, atol=1e-12 * np.abs(ref[1]).max())
    np.testing.assert_allclose(got[2], ref[2], rtol=1e-9, atol=1e-12 * np.abs(ref[2]).max())
    for a, r in zip(got[3:], ref[3:]):
        assert a == pytest.approx(r, rel=1e-9, abs=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [6, 20, 50])
def test_gpu_objective_matches_oracle(k):
    y, lya, nv, x0, k = _training_set(Q=10, k=k)
    f, g = T.objective(x0, y, lya, nv)
    fr, gr = O.objective(x0, y, lya, nv)
    assert f == pytest.approx(fr, rel=1e-11)
    scale = np.abs(gr).max()
    np.testing.assert_allclose(g, gr, rtol=1e-8, atol=1e-11 * scale)


@pytest.mark.gpu
def test_gpu_objective_batches_and_repeat_evaluations_deterministic():
    y, lya, nv, x0, k = _training_set(Q=9, k=8, seed=7)
    with T.Objective(y, lya, nv, k) as obj:
        f1, g1 = obj(x0)
        f2, g2 = obj(x0)
        x1 = x0 + 1e-3
        f3, _ = obj(x1)
    assert f1 == f2 and np.array_equal(g1, g2)
    assert f3 != f1


@pytest.mark.gpu
def test_gpu_learn_qso_model_decreases_objective():
    model = syn.make_model(k=4)
    spectra = syn.make_dr12q_like_spectra(model, 24, seed=8)
    out = T.learn_qso_model(spectra, [s["z_qso"] for s in spectra], k=4, max_iter=5, max_fun_evals=20)
    _, _, y, lya, nv = T.prepare_training_data(spectra, [s["z_qso"] for s in spectra])
    x0, _, lo = T.initial_parameters(y, 4)
    bad = ~np.isfinite(lo)
    x0[4 * 1217:5 * 1217][bad] = np.median(lo[~bad])
    x0 = np.nan_to_num(x0)
    f0, _ = O.objective(x0, y, lya, nv)
    assert out["M"].shape == (1217, 4) and np.isfinite(out["log_likelihood"])
    assert out["log_likelihood"] < f0


@pytest.mark.gpu
def test_gpu_objective_large_grid_high_rank():
    """> 64 KiB of dynamic LDS per block (3,000-pixel rows, k = 40) against the oracle."""
    rng = np.random.default_rng(9)
    Q, Pn, k = 3, 3000, 40
    y = 0.3 * rng.standard_normal((Q, Pn))
    y[rng.uniform(size=y.shape) < 0.2] = np.nan
    lya = rng.uniform(2.5, 4.5, (Q, Pn))
    nv = rng.uniform(0.01, 0.1, (Q, Pn))
    x = np.concatenate([0.05 * rng.standard_normal(Pn * k), np.log(0.15) + 0.1 * rng.standard_normal(Pn),
                        [np.log(0.1), np.log(0.0023), np.log(3.65)]])
    f, g = T.objective(x, y, lya, nv)
    fr, gr = O.objective(x, y, lya, nv)
    assert f == pytest.approx(fr, rel=1e-11)
    np.testing.assert_allclose(g, gr, rtol=1e-8, atol=1e-11 * np.abs(gr).max())


@pytest.mark.gpu
def test_gpu_objective_multi_launch_matches_one_launch(monkeypatch):
    """Spectra in launches of 7 (a ragged last one; GPDLA_OBJECTIVE_BATCH) against one launch and the
    oracle: the per-launch Gram / dM GEMM tiles are 32 spectra, so every launch has padding rows."""
    y, lya, nv, x0, k = _training_set(Q=40, k=20, seed=11)
    f1, g1 = T.objective(x0, y, lya, nv)
    monkeypatch.setenv("GPDLA_OBJECTIVE_BATCH", "7")
    f7, g7 = T.objective(x0, y, lya, nv)
    fr, gr = O.objective(x0, y, lya, nv)
    assert f7 == pytest.approx(f1, rel=1e-13) and f7 == pytest.approx(fr, rel=1e-11)
    scale = np.abs(gr).max()
    np.testing.assert_allclose(g7, g1, rtol=1e-11, atol=1e-13 * scale)
    np.testing.assert_allclose(g7, gr, rtol=1e-8, atol=1e-11 * scale)
