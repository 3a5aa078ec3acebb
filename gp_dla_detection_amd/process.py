"""``process_qsos`` mirror (process_qsos.m:1-249) over the native engine.

The MATLAB script reads seven workspace variables and four ``.mat`` files, loops over spectra
and saves ``processed_qsos_<test_set>.mat``.  Here the same steps are one function call:

    params = set_parameters()
    out = process_qsos(model, samples, spectra, prior, params=params, test_ind=...)
    save_processed_qsos(path, out)

``spectra`` is the preloaded_qsos content: either a list of dicts (``wavelengths``, ``flux``,
``noise_variance``, ``pixel_mask``, ``z_qso``) or CSR arrays from ``synthetic.pack_spectra``.
The likelihood of every (spectrum, DLA sample) pair, the null model and the log-mean-exp run on
the GPU (libgpdla.so); priors and posteriors are O(Q) host bookkeeping (process_qsos.m:4-27,
122-132, 222-232).
"""
from __future__ import annotations

import numpy as np

from . import parameters as P
from .engine import Engine
from .parameters import Parameters, set_parameters
from .synthetic import pack_spectra


def filter_prior_dlas(prior_z_qsos, prior_dla_ind, prior_z_dlas):
    """process_qsos.m:20-25: drop prior DLAs whose Lya lies below the QSO's Lyman limit."""
    dla_ind = np.array(prior_dla_ind, dtype=bool).copy()
    for i in np.flatnonzero(dla_ind):
        zd = np.atleast_1d(np.asarray(prior_z_dlas[i], dtype=np.float64))
        # MATLAB `if` on a vector is true only if every element is true
        if zd.size and np.all(P.observed_wavelengths(P.LYA_WAVELENGTH, zd)
                              < P.observed_wavelengths(P.LYMAN_LIMIT, prior_z_qsos[i])):
            dla_ind[i] = False
    return dla_ind


def dla_priors(z_qsos, prior_z_qsos, prior_dla_ind, prior_z_qso_increase=P.PRIOR_Z_QSO_INCREASE):
    """process_qsos.m:122-132, vectorised with a sorted prior catalogue."""
    pz = np.asarray(prior_z_qsos, dtype=np.float64)
    order = np.argsort(pz, kind="stable")
    pz_sorted = pz[order]
    dla_cum = np.concatenate([[0], np.cumsum(np.asarray(prior_dla_ind, dtype=bool)[order])])
    cut = np.searchsorted(pz_sorted, np.asarray(z_qsos, dtype=np.float64) + prior_z_qso_increase, side="left")
    num_quasars = cut.astype(np.float64)
    num_dlas = dla_cum[cut].astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        log_priors_dla = np.log(num_dlas) - np.log(num_quasars)
        log_priors_no_dla = np.log(num_quasars - num_dlas) - np.log(num_quasars)
    return log_priors_no_dla, log_priors_dla


def model_posteriors(log_posteriors_no_dla, log_posteriors_dla):
    """process_qsos.m:222-232."""
    lp = np.stack([log_posteriors_no_dla, log_posteriors_dla], axis=1)
    mx = np.max(lp, axis=1, keepdims=True)
    post = np.exp(lp - mx)
    post = post / np.sum(post, axis=1, keepdims=True)
    p_no = post[:, 0]
    return post, p_no, 1 - p_no


def _select(spectra, test_ind):
    if isinstance(spectra, dict) and "offsets" in spectra:
        packed = spectra
        if test_ind is None:
            return packed
        idx = np.flatnonzero(np.asarray(test_ind)) if np.asarray(test_ind).dtype == bool else np.asarray(test_ind)
        lst = []
        for q in idx:
            a, b = packed["offsets"][q], packed["offsets"][q + 1]
            lst.append(dict(wavelengths=packed["wavelengths"][a:b], flux=packed["flux"][a:b],
                            noise_variance=packed["noise_variance"][a:b],
                            pixel_mask=packed["pixel_mask"][a:b], z_qso=packed["z_qsos"][q]))
        return pack_spectra(lst)
    lst = list(spectra)
    if test_ind is not None:
        ti = np.asarray(test_ind)
        idx = np.flatnonzero(ti) if ti.dtype == bool else ti
        lst = [lst[i] for i in idx]
    return pack_spectra(lst)


def process_qsos(model: dict, samples: dict, spectra, prior: dict | None = None,
                 params: Parameters | None = None, test_ind=None, engine: Engine | None = None,
                 device: int = 0, metadata: dict | None = None) -> dict:
    """Run the DLA search (process_qsos.m:88-232) and return the saved variables."""
    params = params or set_parameters(k=np.asarray(model["M"]).shape[1])
    packed = _select(spectra, test_ind)
    eng = engine or Engine(model, samples, params, device=device)
    try:
        res = eng.process(packed, want_samples=True)
    finally:
        if engine is None:
            eng.close()
    Q = packed["z_qsos"].size
    out = dict(
        min_z_dlas=res["min_z_dlas"], max_z_dlas=res["max_z_dlas"],
        log_likelihoods_no_dla=res["log_likelihoods_no_dla"],
        sample_log_likelihoods_dla=res["sample_log_likelihoods_dla"],
        log_likelihoods_dla=res["log_likelihoods_dla"], num_pixels=res["num_pixels"],
        num_lines=params.num_lines, max_z_cut=params.max_z_cut,
        prior_z_qso_increase=params.prior_z_qso_increase)
    if prior is not None:
        dla_ind = filter_prior_dlas(prior["z_qsos"], prior["dla_ind"], prior.get("z_dlas", [None] * len(prior["z_qsos"])))
        lp_no, lp_dla = dla_priors(packed["z_qsos"], prior["z_qsos"], dla_ind, params.prior_z_qso_increase)
    else:
        lp_no, lp_dla = np.full(Q, np.log(0.5)), np.full(Q, np.log(0.5))
    out["log_priors_no_dla"], out["log_priors_dla"] = lp_no, lp_dla
    out["log_posteriors_no_dla"] = lp_no + out["log_likelihoods_no_dla"]      # process_qsos.m:154-155
    out["log_posteriors_dla"] = lp_dla + out["log_likelihoods_dla"]           # process_qsos.m:211-212
    post, p_no, p_dla = model_posteriors(out["log_posteriors_no_dla"], out["log_posteriors_dla"])
    out["model_posteriors"], out["p_no_dlas"], out["p_dlas"] = post, p_no, p_dla
    if test_ind is not None:
        out["test_ind"] = np.asarray(test_ind)
    if "numeric_warning" in res:
        out["numeric_warning"] = res["numeric_warning"]
    for key, val in (metadata or {}).items():
        out[key] = val
    return out


# names of process_qsos.m:235-243, in order
PROCESSED_VARIABLES = ("training_release", "training_set_name", "dla_catalog_name", "prior_ind",
                       "release", "test_set_name", "test_ind", "prior_z_qso_increase", "max_z_cut",
                       "num_lines", "min_z_dlas", "max_z_dlas", "log_priors_no_dla", "log_priors_dla",
                       "log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla",
                       "log_posteriors_no_dla", "log_posteriors_dla", "model_posteriors", "p_no_dlas",
                       "p_dlas")


def save_processed_qsos(path: str, out: dict) -> None:
    """Write the processed_qsos variables with MATLAB shapes (Q-vectors as Q x 1 columns,
    sample_log_likelihoods_dla as Q x S).  Format: MATLAB v5 .mat via scipy (each variable must
    stay under 2 GB; the reference's -v7.3/HDF5 container is a listed next step)."""
    from scipy.io import savemat
    mat = {}
    for key in PROCESSED_VARIABLES:
        if key not in out:
            continue
        v = out[key]
        if isinstance(v, np.ndarray) and v.ndim == 1:
            v = v[:, None]
        mat[key] = v
    savemat(path, mat, do_compression=False, oned_as="column")
