"""GP null-model training (learn_qso_model.m, objective.m, spectrum_loss.m).

The objective and its gradient -- the per-spectrum Woodbury likelihood of the hot path plus its
derivatives wrt M, log omega, log c_0, log tau_0 and log beta, summed over the training set --
run on the GPU (libgpdla.so, ``gpdla_objective_*``; csrc/objective.hip).  The host side mirrors
the reference's scripts:

* ``spectrum_loss(...)``          spectrum_loss.m:14-76 for one spectrum;
* ``objective(x, ...)``           objective.m:13-74 (``Objective`` keeps the training matrices
                                  resident on the device across evaluations);
* ``prepare_training_data(...)``  learn_qso_model.m:27-80: rest-frame interpolation onto the
                                  911.75:0.25:1215.75 grid, noise cut, mean flux, centring;
* ``initial_parameters(...)``     learn_qso_model.m:82-101: PCA of the centred fluxes with
                                  pairwise-complete covariance (pca(..., 'rows', 'pairwise')),
                                  initial M, log omega (nanstd) and the three scalars;
* ``learn_qso_model(...)``        the optimisation (learn_qso_model.m:103-120) and the saved
                                  variables (:122-131).

minFunc (the reference's optimiser, a third-party MATLAB package, not vendored) is replaced by
scipy's L-BFGS-B, the same method family with the same iteration/evaluation caps; its iterates
differ from minFunc's, the objective and gradient it is driven by are the parity-checked ones.
As in objective.m, the tau_0 / beta priors enter the gradient but not f (objective.m:59-71).
"""
from __future__ import annotations

import ctypes as C
import warnings

import numpy as np

from . import _lib as L
from . import parameters as P


def spectrum_loss(y, lya_1pz, noise_variance, M, omega2, c_0, tau_0, beta):
    """``[nlog_p, dM, dlog_omega, dlog_c_0, dlog_tau_0, dlog_beta] = spectrum_loss(...)``."""
    lib = L.load()
    y = np.ascontiguousarray(y, dtype=np.float64).ravel()
    n = y.size
    lya = np.ascontiguousarray(lya_1pz, dtype=np.float64).ravel()
    nv = np.ascontiguousarray(noise_variance, dtype=np.float64).ravel()
    om2 = np.ascontiguousarray(omega2, dtype=np.float64).ravel()
    M = np.asarray(M, dtype=np.float64).reshape(n, -1)
    k = M.shape[1]
    Mf = np.asfortranarray(M).ravel(order="F")
    if not (lya.size == nv.size == om2.size == n):
        raise ValueError("spectrum_loss: inputs disagree on n")
    nlp = np.empty(1)
    dM = np.empty(n * k)
    dlo = np.empty(n)
    sc = np.empty(3)
    L.check(lib.gpdla_spectrum_loss_f64(L.ptr(y), L.ptr(lya), L.ptr(nv), L.ptr(Mf), L.ptr(om2), n, k,
                                        float(c_0), float(tau_0), float(beta), L.ptr(nlp), L.ptr(dM),
                                        L.ptr(dlo), L.ptr(sc[0:1]), L.ptr(sc[1:2]), L.ptr(sc[2:3])))
    return float(nlp[0]), dM.reshape(n, k, order="F"), dlo, float(sc[0]), float(sc[1]), float(sc[2])


class Objective:
    """objective.m with the training matrices resident on ``device``: ``f, g = obj(x)``."""

    def __init__(self, centered_rest_fluxes, lya_1pzs, rest_noise_variances, k: int, device: int = 0):
        self.lib = L.load()
        y = np.ascontiguousarray(centered_rest_fluxes, dtype=np.float64)
        lya = np.ascontiguousarray(lya_1pzs, dtype=np.float64)
        nv = np.ascontiguousarray(rest_noise_variances, dtype=np.float64)
        if y.ndim != 2 or y.shape != lya.shape or y.shape != nv.shape:
            raise ValueError("training matrices must share one (num_quasars, num_pixels) shape")
        self.num_quasars, self.num_pixels = y.shape
        self.k = int(k)
        self.nx = (self.k + 1) * self.num_pixels + 3
        h = C.c_void_p()
        L.check(self.lib.gpdla_objective_create(device, self.num_quasars, self.num_pixels, self.k, L.ptr(y),
                                                L.ptr(lya), L.ptr(nv), L.MEM_HOST, C.byref(h)))
        self._h = h
        self.evaluations = 0

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64).ravel()
        if x.size != self.nx:
            raise ValueError(f"x has {x.size} entries, expected {self.nx} = (k + 1) num_pixels + 3")
        f = np.empty(1)
        g = np.empty(self.nx)
        L.check(self.lib.gpdla_objective_eval(self._h, L.ptr(x), L.ptr(f), L.ptr(g)))
        self.evaluations += 1
        return float(f[0]), g

    def close(self):
        if getattr(self, "_h", None):
            self.lib.gpdla_objective_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def objective(x, centered_rest_fluxes, lya_1pzs, rest_noise_variances, device: int = 0):
    """``[f, g] = objective(x, centered_rest_fluxes, lya_1pzs, rest_noise_variances)``."""
    x = np.asarray(x, dtype=np.float64).ravel()
    num_pixels = np.asarray(centered_rest_fluxes).shape[1]
    k = (x.size - 3) // num_pixels - 1                                      # objective.m:18
    with Objective(centered_rest_fluxes, lya_1pzs, rest_noise_variances, k, device) as obj:
        return obj(x)


def _interp1(x, v, xq):
    """MATLAB interp1(x, v, xq) ('linear', NaN outside [min x, max x], NaN samples propagate)."""
    x = np.asarray(x, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    order = np.argsort(x, kind="stable")
    x, v = x[order], v[order]
    out = np.full(np.shape(xq), np.nan)
    inside = (xq >= x[0]) & (xq <= x[-1])
    j = np.clip(np.searchsorted(x, xq[inside], side="right") - 1, 0, x.size - 2)
    x0, x1 = x[j], x[j + 1]
    t = (xq[inside] - x0) / (x1 - x0)
    vals = v[j] + t * (v[j + 1] - v[j])
    exact = xq[inside] == x1                       # right endpoint of a segment: take v[j+1]
    vals = np.where(exact, v[j + 1], vals)
    out[inside] = vals
    return out


def prepare_training_data(spectra, z_qsos, max_noise_variance: float = P.MAX_NOISE_VARIANCE,
                          rest_wavelengths=None):
    """learn_qso_model.m:27-80 -> (rest_wavelengths, mu, centered_rest_fluxes, lya_1pzs,
    rest_noise_variances).  ``spectra``: dicts with wavelengths / flux / noise_variance /
    pixel_mask (the preloaded_qsos cells selected by train_ind)."""
    if rest_wavelengths is None:
        rest_wavelengths = np.arange(P.MIN_LAMBDA, P.MAX_LAMBDA + P.DLAMBDA / 2, P.DLAMBDA)   # :33
    R = rest_wavelengths.size
    Q = len(spectra)
    lya_1pzs = np.full((Q, R), np.nan)
    rest_fluxes = np.full((Q, R), np.nan)
    rest_noise_variances = np.full((Q, R), np.nan)
    for i, (s, z) in enumerate(zip(spectra, z_qsos)):
        lam = np.asarray(s["wavelengths"], dtype=np.float64)
        flux = np.array(s["flux"], dtype=np.float64)
        nv = np.array(s["noise_variance"], dtype=np.float64)
        mask = np.asarray(s["pixel_mask"], dtype=bool)
        flux[mask] = np.nan                                                   # :50-51
        nv[mask] = np.nan
        rest = P.emitted_wavelengths(lam, z)                                  # :53
        lya_1pzs[i] = _interp1(rest, 1 + (lam - P.LYA_WAVELENGTH) / P.LYA_WAVELENGTH, rest_wavelengths)  # :55-58
        rest_fluxes[i] = _interp1(rest, flux, rest_wavelengths)               # :60-61
        rest_noise_variances[i] = _interp1(rest, nv, rest_wavelengths)        # :63-65
    ind = rest_noise_variances > max_noise_variance                           # :71
    lya_1pzs[ind] = np.nan
    rest_fluxes[ind] = np.nan
    rest_noise_variances[ind] = np.nan
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)       # all-NaN rest pixels -> NaN, as in MATLAB
        mu = np.nanmean(rest_fluxes, axis=0)                                  # :77
    centered = rest_fluxes - mu                                               # :78
    return rest_wavelengths, mu, centered, lya_1pzs, rest_noise_variances


def pairwise_pca(X, k: int):
    """pca(X, 'numcomponents', k, 'rows', 'pairwise') (learn_qso_model.m:82-85): MATLAB's pca
    centres each column by its nanmean and then takes the NON-centred pairwise covariance
    (its ncnancov): C(a, b) = sum over the rows where both columns are present of x_a x_b,
    divided by (that row count - 1).  Entries with fewer than two common rows are 0 here."""
    X = np.asarray(X, dtype=np.float64)
    m = ~np.isnan(X)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        Xc = X - np.nanmean(X, axis=0)    # no-op on the already centred training fluxes (:70-71)
    Z = np.where(m, Xc, 0.0)
    Mf = m.astype(np.float64)
    N = Mf.T @ Mf                         # common-row counts
    with np.errstate(invalid="ignore", divide="ignore"):
        cov = (Z.T @ Z) / (N - 1)
    cov = np.where(N > 1, cov, 0.0)
    cov = 0.5 * (cov + cov.T)
    lat, vec = np.linalg.eigh(cov)
    order = np.argsort(lat)[::-1][:k]
    vec = vec[:, order]
    # MATLAB pca sign convention: the largest-magnitude element of each coefficient is positive
    sgn = np.sign(vec[np.argmax(np.abs(vec), axis=0), np.arange(vec.shape[1])])
    return vec * sgn, lat[order]


def initial_parameters(centered_rest_fluxes, k: int = P.K):
    """learn_qso_model.m:82-101: initial x = [M(:); log omega; log c_0; log tau_0; log beta]."""
    coefficients, latent = pairwise_pca(centered_rest_fluxes, k)             # :82-85
    initial_M = coefficients[:, :k] * np.sqrt(np.maximum(latent[:k], 0))      # :90
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        # MATLAB nanstd normalises by N - 1, except a single observation (std 0); no data -> NaN
        cnt = np.sum(~np.isnan(centered_rest_fluxes), axis=0)
        sd = np.nanstd(centered_rest_fluxes, axis=0, ddof=1)
        sd = np.where(cnt == 1, 0.0, sd)
        with np.errstate(divide="ignore"):
            initial_log_omega = np.log(sd)                                    # :92
    x0 = np.concatenate([initial_M.ravel(order="F"), initial_log_omega,
                         [np.log(P.INITIAL_C_0), np.log(P.INITIAL_TAU_0), np.log(P.INITIAL_BETA)]])
    return x0, initial_M, initial_log_omega


def learn_qso_model(spectra, z_qsos, k: int = P.K, max_iter: int = 2000, max_fun_evals: int = 4000,
                    device: int = 0) -> dict:
    """learn_qso_model.m:27-131 on preloaded spectra; returns the saved variables."""
    from scipy.optimize import minimize
    rest_wavelengths, mu, centered, lya_1pzs, noise = prepare_training_data(spectra, z_qsos)
    x0, initial_M, initial_log_omega = initial_parameters(centered, k)
    R = rest_wavelengths.size
    # Rest pixels seen by fewer than two training spectra get log omega = -Inf / NaN from nanstd
    # (as in MATLAB); real training sets cover the grid, but the optimiser cannot start from a
    # non-finite point, so those entries start at the median finite value instead (reported).
    lo = x0[R * k:R * (k + 1)]
    bad = ~np.isfinite(lo)
    if np.any(bad):
        lo[bad] = np.median(lo[~bad]) if np.any(~bad) else np.log(0.1)
    x0 = np.nan_to_num(x0, nan=0.0)
    with Objective(centered, lya_1pzs, noise, k, device) as obj:
        res = minimize(obj, x0, jac=True, method="L-BFGS-B",
                       options=dict(maxiter=max_iter, maxfun=max_fun_evals))
        evals = obj.evaluations
    x = res.x
    return dict(rest_wavelengths=rest_wavelengths, mu=mu, initial_M=initial_M,
                initial_log_omega=initial_log_omega, initial_log_c_0=np.log(P.INITIAL_C_0),
                initial_tau_0=P.INITIAL_TAU_0, initial_beta=P.INITIAL_BETA,
                M=x[:R * k].reshape(R, k, order="F"), log_omega=x[R * k:R * (k + 1)],
                log_c_0=x[-3], log_tau_0=x[-2], log_beta=x[-1], log_likelihood=res.fun,
                max_noise_variance=P.MAX_NOISE_VARIANCE,
                minFunc_output=dict(iterations=res.nit, funcCount=evals, message=str(res.message),
                                    nonfinite_initial_log_omega=int(np.count_nonzero(bad))))


def run_learn_qso_model(base_directory: str, training_release: str, training_set_name: str, train_ind,
                        k: int = P.K, max_iter: int = 2000, max_fun_evals: int = 4000, device: int = 0) -> dict:
    """The script on files (learn_qso_model.m:1-131): catalog.mat and preloaded_qsos.mat of
    ``training_release`` in, learned_qso_model_<training_set_name>.mat (v7.3) out.  ``train_ind``
    is the reference's index expression over ``catalog`` (e.g. README.md:148-152), a callable or
    a boolean array."""
    from .matv73 import loadmat, savemat73
    from .process import evaluate_index, load_preloaded_qsos, processed_directory
    d = processed_directory(base_directory, training_release)
    catalog = loadmat(f"{d}/catalog.mat")
    tind = evaluate_index(train_ind, catalog=catalog).astype(bool).ravel()
    spectra = load_preloaded_qsos(f"{d}/preloaded_qsos.mat", tind)                 # :10-19
    z_qsos = np.asarray(catalog["z_qsos"], dtype=np.float64).ravel()[tind]          # :21
    out = learn_qso_model(spectra, z_qsos, k=k, max_iter=max_iter, max_fun_evals=max_fun_evals, device=device)
    save = {key: val for key, val in out.items() if key != "minFunc_output"}
    save["minFunc_output"] = {kk: (vv if isinstance(vv, str) else np.float64(vv))
                              for kk, vv in out["minFunc_output"].items()}
    save.update(training_release=training_release, train_ind=tind,
                minFunc_options=dict(MaxIter=np.float64(max_iter), MaxFunEvals=np.float64(max_fun_evals)))
    for key in ("rest_wavelengths", "mu", "log_omega", "initial_log_omega"):
        save[key] = np.asarray(save[key], dtype=np.float64).reshape(1, -1)          # MATLAB rows
    for key in ("log_c_0", "log_tau_0", "log_beta", "log_likelihood", "initial_log_c_0",
                "initial_tau_0", "initial_beta", "max_noise_variance"):
        save[key] = np.float64(save[key])
    savemat73(f"{d}/learned_qso_model_{training_set_name}.mat", save)              # :122-131
    return out
