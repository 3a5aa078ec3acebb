"""GPU: the reference's whole workflow on files (README.md:54-315), each script through this
framework -- preload_qsos (FITS in) -> learn_qso_model (GPU objective) -> generate_dla_samples ->
process_qsos (GPU engine) -> processed_qsos_<set>.mat (v7.3) -- at a small synthetic scale."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from fits_writer import write_speclite  # noqa: E402
from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import dla_samples as DS  # noqa: E402
from gp_dla_detection_amd import ingest as I  # noqa: E402
from gp_dla_detection_amd import matv73 as M  # noqa: E402
from gp_dla_detection_amd import parameters as P  # noqa: E402
from gp_dla_detection_amd import process as PR  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd import training as T  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _speclite(rng, model, z, normalizer=7.3):
    """A raw DR12Q-like coadd: 3600 A .. beyond the 1310-1325 A rest normalisation window."""
    loglam = np.arange(np.log10(3600.0), np.log10(1340.0 * (1 + z)), 1e-4)
    lam = 10 ** loglam
    rest = lam / (1 + z)
    cont = np.where((rest >= P.MIN_LAMBDA) & (rest <= P.MAX_LAMBDA),
                    np.interp(rest, model["rest_wavelengths"], model["mu"]), 1.0)
    sigma = rng.uniform(0.05, 0.15, lam.size)
    flux = normalizer * (cont + sigma * rng.standard_normal(lam.size))
    ivar = 1.0 / (normalizer * sigma) ** 2
    ivar[rng.uniform(size=lam.size) < 0.02] = 0.0
    and_mask = np.where(rng.uniform(size=lam.size) < 0.01, 1 << 23, 0)
    return flux, loglam, ivar, and_mask


def test_reference_workflow_on_files(tmp_path):
    rng = np.random.default_rng(21)
    model = syn.make_model(k=6)
    Q = 24
    z_qsos = rng.uniform(2.3, 3.6, Q)
    base = tmp_path / "data"
    proc = base / "dr12q" / "processed"
    proc.mkdir(parents=True)
    plates, mjds, fibers = 4000 + np.arange(Q), 55000 + np.arange(Q), 1 + np.arange(Q)
    for q in range(Q):
        d = base / "dr12q" / "spectra" / str(plates[q])
        d.mkdir(parents=True, exist_ok=True)
        write_speclite(str(d / f"spec-{plates[q]}-{mjds[q]}-{fibers[q]:04d}.fits"), *_speclite(rng, model, z_qsos[q]))
    filter_flags = np.zeros(Q, dtype=np.uint8)
    filter_flags[3] = 1                                      # e.g. z < z_qso_cut upstream
    log_nhis = [np.array([rng.normal(20.6, 0.3)]) if rng.uniform() < 0.5 else np.zeros(0) for _ in range(Q)]
    catalog = dict(z_qsos=z_qsos, plates=plates.astype(float), mjds=mjds.astype(float),
                   fiber_ids=fibers.astype(float), filter_flags=filter_flags,
                   in_dr9=np.ones(Q, dtype=bool),
                   los_inds=dict(dr9q_concordance=np.ones(Q, dtype=bool)),
                   dla_inds=dict(dr9q_concordance=np.array([c.size > 0 for c in log_nhis])),
                   z_dlas=dict(dr9q_concordance=[np.array([z - 0.4]) if c.size else np.zeros(0)
                                                 for z, c in zip(z_qsos, log_nhis)]),
                   log_nhis=dict(dr9q_concordance=log_nhis))
    M.savemat73(str(proc / "catalog.mat"), catalog)

    pre = I.run_preload_qsos(str(base), "dr12q")                                       # preload_qsos
    assert pre["filter_flags"][3] == 1 and np.count_nonzero(pre["filter_flags"]) == 1
    assert all(pre["all_normalizers"][q] == pytest.approx(7.3, rel=0.05) for q in range(Q) if q != 3)

    learned = T.run_learn_qso_model(str(base), "dr12q", "dr9q_minus_concordance",     # learn_qso_model
                                    "(catalog.filter_flags == 0)", k=6, max_iter=4, max_fun_evals=12)
    assert np.isfinite(learned["log_likelihood"])
    lm = PR.load_model(str(proc / "learned_qso_model_dr9q_minus_concordance.mat"))
    assert lm["M"].shape == (1217, 6) and np.array_equal(lm["M"], learned["M"])

    # the (tiny) synthetic catalogue has few DLAs: pad the column densities for the KDE fit
    cat = M.loadmat73(str(proc / "catalog.mat"))
    cells = list(cat["log_nhis"]["dr9q_concordance"].ravel()) + [rng.normal(20.6, 0.3, 200)]
    cat["log_nhis"] = dict(dr9q_concordance=cells)
    M.savemat73(str(proc / "catalog.mat"), cat)
    samples = DS.run_generate_dla_samples(str(base), "dr12q", "dr9q_concordance", num_dla_samples=256)
    assert samples["log_nhi_samples"].shape == (256,)

    prior_ind = " prior_catalog.in_dr9 & (prior_catalog.filter_flags == 0) & prior_catalog.los_inds(dla_catalog_name)"
    out = PR.run_process_qsos(str(base), "dr12q", "dr9q_minus_concordance", "dr9q_concordance",  # process_qsos
                              prior_ind, "dr12q", "dr12q", "(catalog.filter_flags == 0)")
    saved = M.loadmat73(str(proc / "processed_qsos_dr12q.mat"))
    Qt = Q - 1
    sll = saved["sample_log_likelihoods_dla"]
    assert sll.shape == (Qt, 256)
    ok = np.isfinite(saved["log_likelihoods_dla"][:, 0])
    assert ok.sum() >= Qt - 2                                 # all usable spectra evaluated
    inv = np.exp(sll[ok] - (saved["log_likelihoods_dla"][ok] + np.log(256))).sum(axis=1)
    np.testing.assert_allclose(inv, 1.0, rtol=1e-10)        # calc_cddf.py:246 normalisation
    p = saved["p_dlas"][ok, 0]
    assert np.all((p >= 0) & (p <= 1))
    assert saved["test_ind"].ravel().tolist() == (pre["filter_flags"] == 0).tolist()
