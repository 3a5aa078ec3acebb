"""CPU oracle for the GP-DLA likelihood hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.  The product path
(``gp_dla_detection_amd``) never imports it.

What it restates (reference = sbird/gp_dla_detection, paths relative to the repo root):

* ``voigt_mex``            -- voigt.c:253-304 (MEX entry: multipliers, velocity, line sum,
                              exp, 7-tap instrument convolution into a zero-initialised output).
* ``log_mvnpdf_low_rank``  -- log_mvnpdf_low_rank.m:5-33, in MATLAB operation order
                              (B = M'(d_inv.*M) + I, upper chol, C = L\\(L'\\D_inv_M'), ...).
* ``process_spectrum``     -- process_qsos.m:96-212 for one spectrum (pixel selection, model
                              interpolation, null model, z_DLA grid, padded grid, the
                              ``ind = ~this_pixel_mask(ind)`` absorption-index quirk, the
                              per-sample modulated likelihood, log-mean-exp).
* ``dla_priors`` / ``model_posteriors`` -- process_qsos.m:4-27,122-132,222-232.
* ``spectrum_loss`` / ``objective`` -- spectrum_loss.m:14-76 and objective.m:13-74 (the GP
                              null-model training likelihood and gradient).

Third-party dependency on the path: **libcerf** ``voigt(x, sigma, gamma)`` (called at
voigt.c:288; install note README.md:210-218; not vendored, *no pinned version*).  libcerf 1.x
computes ``Re w((x + i*gamma)/(sigma*sqrt 2)) / (sigma*sqrt(2*pi))`` with S. G. Johnson's
Faddeeva-package ``w_of_z``.  ``scipy.special.voigt_profile`` (scipy 1.15.3) implements the
same published definition with the same Faddeeva package, so it stands in for libcerf here.

Parity pinning.  The reference ships no tests, fixtures or golden vectors for this path
(SURVEY.md section 4), and its hot path is MATLAB + a MEX file that cannot build here (no
MATLAB/Octave, no ``mex.h``, no libcerf; building it against stand-in headers is not
allowed).  This restatement is therefore pinned against independent implementations of the
same mathematics, not against reference outputs:

* libcerf ``voigt``     -> scipy.special.voigt_profile / wofz (same published algorithm);
* log_mvnpdf_low_rank   -> dense ``scipy.stats.multivariate_normal.logpdf`` of
                           N(mu, MM' + diag(d)) (the function's documented meaning, .m:1-3);
* voigt.c constant tables -> their own commented formulas (voigt.c:141-240);
* the only invariant the reference itself asserts, calc_cddf.py:246
  (sum_s exp(ll_s - ll_dla - log S) == 1).

Status: parity is pinned to the mathematics above, *not* to executed reference outputs
("parity unpinned" with respect to running the MATLAB reference itself).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cholesky, solve_triangular
from scipy.special import voigt_profile

# ----------------------------------------------------------------------------------------
# voigt.c constant tables (CGS).  Values restated from voigt.c; line numbers cited.
# ----------------------------------------------------------------------------------------
C_CGS = 2.99792458e10  # voigt.c:22 speed of light, cm/s

TRANSITION_WAVELENGTHS = np.array([  # voigt.c:31-64, cm
    1.2156701e-05, 1.0257223e-05, 9.725368e-06, 9.497431e-06, 9.378035e-06,
    9.307483e-06, 9.262257e-06, 9.231504e-06, 9.209631e-06, 9.193514e-06,
    9.181294e-06, 9.171806e-06, 9.16429e-06, 9.15824e-06, 9.15329e-06,
    9.14919e-06, 9.14576e-06, 9.14286e-06, 9.14039e-06, 9.13826e-06,
    9.13641e-06, 9.13480e-06, 9.13339e-06, 9.13215e-06, 9.13104e-06,
    9.13006e-06, 9.12918e-06, 9.12839e-06, 9.12768e-06, 9.12703e-06,
    9.12645e-06])

OSCILLATOR_STRENGTHS = np.array([  # voigt.c:66-99
    0.416400, 0.079120, 0.029000, 0.013940, 0.007799, 0.004814, 0.003183,
    0.002216, 0.001605, 0.00120, 0.000921, 0.0007226, 0.000577, 0.000469,
    0.000386, 0.000321, 0.000270, 0.000230, 0.000197, 0.000170, 0.000148,
    0.000129, 0.000114, 0.000101, 0.000089, 0.000080, 0.000071, 0.000064,
    0.000058, 0.000053, 0.000048])

TRANSITION_RATES = np.array([  # voigt.c:101-134 (Gammas), s^-1
    6.265e+08, 1.897e+08, 8.127e+07, 4.204e+07, 2.450e+07, 1.236e+07, 8.255e+06,
    5.785e+06, 4.210e+06, 3.160e+06, 2.432e+06, 1.911e+06, 1.529e+06, 1.243e+06,
    1.024e+06, 8.533e+05, 7.186e+05, 6.109e+05, 5.237e+05, 4.523e+05, 3.933e+05,
    3.443e+05, 3.030e+05, 2.679e+05, 2.382e+05, 2.127e+05, 1.907e+05, 1.716e+05,
    1.550e+05, 1.405e+05, 1.277e+05])

SIGMA = 9.08537121627923800e+05  # voigt.c:146, Gaussian width cm/s (b / sqrt 2, T = 1e4 K)

LEADING_CONSTANTS = np.array([  # voigt.c:151-184, cm^2
    1.34347262962625339e-07, 2.15386482180851912e-08, 7.48525170087141461e-09,
    3.51375347286007472e-09, 1.94112336271172934e-09, 1.18916112899713152e-09,
    7.82448627128742997e-10, 5.42930932279390593e-10, 3.92301197282493829e-10,
    2.92796010451409027e-10, 2.24422239410389782e-10, 1.75895684469038289e-10,
    1.40338556137474778e-10, 1.13995374637743197e-10, 9.37706429662300083e-11,
    7.79453203101192392e-11, 6.55369055970184901e-11, 5.58100321584169051e-11,
    4.77895916635794548e-11, 4.12301389852588843e-11, 3.58872072638707592e-11,
    3.12745536798214080e-11, 2.76337116167110415e-11, 2.44791750078032772e-11,
    2.15681362798480253e-11, 1.93850080479346101e-11, 1.72025364178111889e-11,
    1.55051698336865945e-11, 1.40504672409331934e-11, 1.28383057589411395e-11,
    1.16264059622218997e-11])

LORENTZ_GAMMAS = np.array([  # voigt.c:187-220 (gammas), cm/s
    6.06075804241938613e+02, 1.54841462408931704e+02, 6.28964942715328164e+01,
    3.17730561586147395e+01, 1.82838676775503330e+01, 9.15463131005758157e+00,
    6.08448802613156925e+00, 4.24977523573725779e+00, 3.08542121666345803e+00,
    2.31184525202557767e+00, 1.77687796208123139e+00, 1.39477990932179852e+00,
    1.11505539984541979e+00, 9.05885451682623022e-01, 7.45877170715450677e-01,
    6.21261624902197052e-01, 5.22994533400935269e-01, 4.44469874827484512e-01,
    3.80923210837841919e-01, 3.28912390446060132e-01, 2.85949711597237033e-01,
    2.50280032040928802e-01, 2.20224061101442048e-01, 1.94686521675913549e-01,
    1.73082093051965591e-01, 1.54536566013816490e-01, 1.38539175663870029e-01,
    1.24652675945279762e-01, 1.12585442799479921e-01, 1.02045988802423507e-01,
    9.27433783998286437e-02])

VOIGT_WIDTH = 3  # voigt.c:229
INSTRUMENT_PROFILE = np.array([  # voigt.c:242-251
    2.17460992138080811e-03, 4.11623059580451742e-02, 2.40309364651846963e-01,
    4.32707438937454059e-01, 2.40309364651846963e-01, 4.11623059580451742e-02,
    2.17460992138080811e-03])
MAX_LINES = 31  # voigt.c:16

LOG_2PI = 1.83787706640934534  # log_mvnpdf_low_rank.m:7


# ----------------------------------------------------------------------------------------
# set_parameters.m restatement (the subset the hot path reads)
# ----------------------------------------------------------------------------------------
LYA_WAVELENGTH = 1215.6701   # set_parameters.m:5
LYMAN_LIMIT = 911.7633       # set_parameters.m:7
SPEED_OF_LIGHT = 299792458   # set_parameters.m:8 (m/s)
MIN_LAMBDA = 911.75          # set_parameters.m:33
MAX_LAMBDA = 1215.75         # set_parameters.m:34
PIXEL_SPACING = 1e-4         # set_parameters.m:60
WIDTH = 3                    # set_parameters.m:59


def kms_to_z(kms):  # set_parameters.m:11
    return (kms * 1000) / SPEED_OF_LIGHT


PRIOR_Z_QSO_INCREASE = kms_to_z(30000)  # set_parameters.m:56
MAX_Z_CUT = kms_to_z(3000)              # set_parameters.m:65
MIN_Z_CUT = kms_to_z(3000)              # set_parameters.m:69


def max_z_dla(wavelengths, z_qso):  # set_parameters.m:66-67
    return (np.max(wavelengths) / LYA_WAVELENGTH - 1) - MAX_Z_CUT


def min_z_dla(wavelengths, z_qso):  # set_parameters.m:70-73
    return max(np.min(wavelengths) / LYA_WAVELENGTH - 1,
               (LYMAN_LIMIT * (1 + z_qso)) / LYA_WAVELENGTH - 1 + MIN_Z_CUT)


# ----------------------------------------------------------------------------------------
# voigt.c:253-304
# ----------------------------------------------------------------------------------------
def libcerf_voigt(x, sigma, gamma):
    """libcerf ``voigt(x, sigma, gamma)`` (voigt.c:288) == scipy.special.voigt_profile."""
    return voigt_profile(x, sigma, gamma)


def voigt_mex(lambdas, z, N, num_lines=MAX_LINES):
    """absorption = voigt(lambdas, z, N, num_lines) -- voigt.c:253-304.

    Returns numel(lambdas) - 2*width values (voigt.c:271)."""
    lambdas = np.asarray(lambdas, dtype=np.float64)
    num_points = lambdas.size
    multipliers = C_CGS / (TRANSITION_WAVELENGTHS[:num_lines] * (1 + z)) / 1e8  # :278-279
    total = np.zeros(num_points)
    for j in range(num_lines):                                                   # :285-289
        velocity = lambdas * multipliers[j] - C_CGS                              # :287
        total += -LEADING_CONSTANTS[j] * libcerf_voigt(velocity, SIGMA, LORENTZ_GAMMAS[j])
    raw_profile = np.exp(N * total)                                              # :291
    n_out = num_points - 2 * VOIGT_WIDTH
    profile = np.zeros(n_out)                                                    # :271 zero-filled
    for k in range(2 * VOIGT_WIDTH + 1):                                         # :297-299
        profile += raw_profile[k:k + n_out] * INSTRUMENT_PROFILE[k]
    return profile


# ----------------------------------------------------------------------------------------
# log_mvnpdf_low_rank.m:5-33 (MATLAB operation order)
# ----------------------------------------------------------------------------------------
def log_mvnpdf_low_rank(y, mu, M, d):
    n, k = M.shape                                    # :9
    y = y - mu                                        # :11
    d_inv = 1 / d                                     # :13
    D_inv_y = d_inv * y                               # :14
    D_inv_M = d_inv[:, None] * M                      # :15
    B = M.T @ D_inv_M                                 # :22
    B[np.diag_indices(k)] += 1                        # :23
    L = cholesky(B, lower=False)                      # :24 (MATLAB chol -> upper R, R'R = B)
    C = solve_triangular(L, solve_triangular(L, D_inv_M.T, trans='T', lower=False),
                         lower=False)                 # :26
    K_inv_y = D_inv_y - D_inv_M @ (C @ y)             # :28
    log_det_K = np.sum(np.log(d)) + 2 * np.sum(np.log(np.diag(L)))  # :30
    return -0.5 * (y @ K_inv_y + log_det_K + n * LOG_2PI)             # :32


# ----------------------------------------------------------------------------------------
# process_qsos.m:96-212 for one spectrum
# ----------------------------------------------------------------------------------------
def linspace_matlab(a, b, n):
    """MATLAB linspace: d1 + (0:n-1).*(d2-d1)/(n-1), last point exactly d2."""
    out = a + np.arange(n) * (b - a) / (n - 1)
    out[-1] = b
    return out


def prepare_spectrum(wavelengths, flux, noise_variance, pixel_mask, z_qso, model,
                     absorption_mode="reference"):
    """process_qsos.m:96-180: everything that does not depend on the DLA sample."""
    rest_wavelengths, mu, M, log_omega = (model[k] for k in ("rest_wavelengths", "mu", "M", "log_omega"))
    c_0, tau_0, beta = (np.exp(model[k]) for k in ("log_c_0", "log_tau_0", "log_beta"))  # :84-86
    this_wavelengths = np.asarray(wavelengths, dtype=np.float64)
    this_flux = np.asarray(flux, dtype=np.float64)
    this_noise_variance = np.asarray(noise_variance, dtype=np.float64)
    this_pixel_mask = np.asarray(pixel_mask, dtype=bool)

    this_rest_wavelengths = this_wavelengths / (1 + z_qso)                       # :102
    ind = (this_rest_wavelengths >= MIN_LAMBDA) & (this_rest_wavelengths <= MAX_LAMBDA)  # :104-105
    this_unmasked_wavelengths = this_wavelengths[ind]                           # :109
    inrange_mask = this_pixel_mask[ind]
    ind = ind & (~this_pixel_mask)                                              # :111
    w = this_wavelengths[ind]                                                   # :113
    rest = this_rest_wavelengths[ind]                                           # :114
    y = this_flux[ind]                                                          # :115
    noise = this_noise_variance[ind]                                            # :116
    lya_zs = (w - LYA_WAVELENGTH) / LYA_WAVELENGTH                              # :118-120

    this_mu = np.interp(rest, rest_wavelengths, mu)                             # :139
    this_M = np.stack([np.interp(rest, rest_wavelengths, M[:, j]) for j in range(M.shape[1])],
                      axis=1)                                                   # :140
    this_log_omega = np.interp(rest, rest_wavelengths, log_omega)               # :142
    this_omega2 = np.exp(2 * this_log_omega)                                    # :143
    scaling = 1 - np.exp(-tau_0 * (1 + lya_zs) ** beta) + c_0                   # :145
    this_omega2 = this_omega2 * scaling ** 2                                    # :147

    zmin = min_z_dla(w, z_qso)                                                  # :160
    zmax = max_z_dla(w, z_qso)                                                  # :161

    lo = np.log10(np.min(this_unmasked_wavelengths))                            # :169-177
    hi = np.log10(np.max(this_unmasked_wavelengths))
    padded = np.concatenate([
        10.0 ** linspace_matlab(lo - WIDTH * PIXEL_SPACING, lo - PIXEL_SPACING, WIDTH),
        this_unmasked_wavelengths,
        10.0 ** linspace_matlab(hi + PIXEL_SPACING, hi + WIDTH * PIXEL_SPACING, WIDTH)])

    n = y.size
    if absorption_mode == "reference":
        # :180,189 -- ind = ~this_pixel_mask(ind) is true(n,1), so absorption(ind) keeps the
        # first n of the m in-range profile values.
        absorption_index = np.arange(n)
    elif absorption_mode == "unmasked":
        absorption_index = np.flatnonzero(~inrange_mask)
    else:
        raise ValueError(absorption_mode)
    return dict(y=y, noise=noise, mu=this_mu, M=this_M, omega2=this_omega2, zmin=zmin,
                zmax=zmax, padded=padded, absorption_index=absorption_index, n=n,
                m=this_unmasked_wavelengths.size)


def sample_log_likelihood(prep, z_dla, nhi, num_lines):
    """process_qsos.m:186-197 for one DLA sample."""
    absorption = voigt_mex(prep["padded"], z_dla, nhi, num_lines)               # :186-187
    absorption = absorption[prep["absorption_index"]]                           # :189
    dla_mu = prep["mu"] * absorption                                            # :191
    dla_M = prep["M"] * absorption[:, None]                                     # :192
    dla_omega2 = prep["omega2"] * absorption ** 2                               # :193
    return log_mvnpdf_low_rank(prep["y"], dla_mu, dla_M, dla_omega2 + prep["noise"])  # :196-197


def null_log_likelihood(prep):
    """process_qsos.m:150-152."""
    return log_mvnpdf_low_rank(prep["y"], prep["mu"], prep["M"], prep["omega2"] + prep["noise"])


def log_mean_exp(sample_ll):
    """process_qsos.m:202-209."""
    mx = np.max(sample_ll)
    return mx + np.log(np.mean(np.exp(sample_ll - mx)))


def process_spectrum(wavelengths, flux, noise_variance, pixel_mask, z_qso, model,
                     offset_samples, nhi_samples, num_lines=3, absorption_mode="reference"):
    prep = prepare_spectrum(wavelengths, flux, noise_variance, pixel_mask, z_qso, model,
                            absorption_mode)
    ll_null = null_log_likelihood(prep)
    z_dlas = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * np.asarray(offset_samples)  # :163-165
    sample_ll = np.array([sample_log_likelihood(prep, z, N, num_lines)
                          for z, N in zip(z_dlas, nhi_samples)])
    return dict(log_likelihood_no_dla=ll_null, sample_log_likelihoods_dla=sample_ll,
                log_likelihood_dla=log_mean_exp(sample_ll), min_z_dla=prep["zmin"],
                max_z_dla=prep["zmax"], n=prep["n"], m=prep["m"])


# ----------------------------------------------------------------------------------------
# priors / posteriors: process_qsos.m:4-27,122-132,222-232
# ----------------------------------------------------------------------------------------
def dla_priors(z_qsos, prior_z_qsos, prior_dla_ind, prior_z_dlas):
    prior_dla_ind = np.array(prior_dla_ind, dtype=bool)
    for i in np.flatnonzero(prior_dla_ind):                                     # :20-25
        if LYA_WAVELENGTH * (1 + prior_z_dlas[i]) < LYMAN_LIMIT * (1 + prior_z_qsos[i]):
            prior_dla_ind[i] = False
    lp_dla, lp_no = [], []
    with np.errstate(divide="ignore"):
        for z in z_qsos:
            less = prior_z_qsos < (z + PRIOR_Z_QSO_INCREASE)                    # :123
            nd, nq = np.count_nonzero(prior_dla_ind[less]), np.count_nonzero(less)  # :125-126
            lp_dla.append(np.log(nd) - np.log(nq))                              # :129-130
            lp_no.append(np.log(nq - nd) - np.log(nq))                          # :131-132
    return np.array(lp_no), np.array(lp_dla)


def model_posteriors(log_posteriors_no_dla, log_posteriors_dla):
    lp = np.stack([log_posteriors_no_dla, log_posteriors_dla], axis=1)          # :223-224
    mx = np.max(lp, axis=1, keepdims=True)
    post = np.exp(lp - mx)                                                      # :226-227
    post = post / np.sum(post, axis=1, keepdims=True)                           # :229
    p_no = post[:, 0]                                                           # :231
    return post, p_no, 1 - p_no                                                 # :232


# ----------------------------------------------------------------------------------------
# GP null-model training objective: spectrum_loss.m:14-76 and
# objective.m:13-74, MATLAB operation order
# ----------------------------------------------------------------------------------------
def spectrum_loss(y, lya_1pz, noise_variance, M, omega2, c_0, tau_0, beta):
    n, k = M.shape                                                               # :20
    lya_optical_depth = tau_0 * lya_1pz ** beta                                  # :23
    lya_absorption = np.exp(-lya_optical_depth)                                  # :24
    scaling_factor = 1 - lya_absorption + c_0                                    # :27
    absorption_noise = omega2 * scaling_factor ** 2                              # :28
    d = noise_variance + absorption_noise                                        # :30
    d_inv = 1 / d                                                                # :32
    D_inv_y = d_inv * y                                                          # :33
    D_inv_M = d_inv[:, None] * M                                                 # :34
    B = M.T @ D_inv_M                                                            # :41
    B[np.diag_indices(k)] += 1                                                   # :42
    L = cholesky(B, lower=False)                                                 # :43
    C = solve_triangular(L, solve_triangular(L, D_inv_M.T, trans='T', lower=False),
                         lower=False)                                            # :45
    K_inv_y = D_inv_y - D_inv_M @ (C @ y)                                        # :47
    log_det_K = np.sum(np.log(d)) + 2 * np.sum(np.log(np.diag(L)))               # :49
    nlog_p = 0.5 * (y @ K_inv_y + log_det_K + n * LOG_2PI)                       # :53
    K_inv_M = D_inv_M - D_inv_M @ (C @ M)                                        # :56
    dM = -(np.outer(K_inv_y, K_inv_y @ M) - K_inv_M)                             # :57
    diag_K_inv = d_inv - np.sum(C * D_inv_M.T, axis=0)                           # :60
    dlog_omega = -(absorption_noise * (K_inv_y ** 2 - diag_K_inv))               # :63
    da = c_0 * omega2 * scaling_factor                                           # :66
    dlog_c_0 = -(K_inv_y * da) @ K_inv_y + diag_K_inv @ da                       # :67
    da = omega2 * scaling_factor * lya_optical_depth * lya_absorption            # :70
    dlog_tau_0 = -(K_inv_y * da) @ K_inv_y + diag_K_inv @ da                     # :71
    da = da * np.log(lya_1pz) * beta                                             # :74
    dlog_beta = -(K_inv_y * da) @ K_inv_y + diag_K_inv @ da                      # :75
    return nlog_p, dM, dlog_omega, dlog_c_0, dlog_tau_0, dlog_beta


def objective(x, centered_rest_fluxes, lya_1pzs, rest_noise_variances):
    num_quasars, num_pixels = centered_rest_fluxes.shape                         # :16
    k = (x.size - 3) // num_pixels - 1                                           # :18
    M = x[:num_pixels * k].reshape(num_pixels, k, order="F")                     # :20-21
    log_omega = x[num_pixels * k:num_pixels * (k + 1)]                           # :23-24
    log_c_0, log_tau_0, log_beta = x[-3], x[-2], x[-1]                           # :26-28
    omega2 = np.exp(2 * log_omega)                                               # :30
    c_0, tau_0, beta = np.exp(log_c_0), np.exp(log_tau_0), np.exp(log_beta)      # :31-33
    f = 0.0
    dM = np.zeros_like(M)
    dlog_omega = np.zeros_like(log_omega)
    dlog_c_0 = dlog_tau_0 = dlog_beta = 0.0
    for i in range(num_quasars):                                                 # :42
        ind = ~np.isnan(centered_rest_fluxes[i])                                 # :43
        tf, tdM, tdo, tc, tt, tb = spectrum_loss(
            centered_rest_fluxes[i, ind], lya_1pzs[i, ind], rest_noise_variances[i, ind],
            M[ind], omega2[ind], c_0, tau_0, beta)                               # :45-50
        f += tf
        dM[ind] += tdM
        dlog_omega[ind] += tdo
        dlog_c_0 += tc
        dlog_tau_0 += tt
        dlog_beta += tb
    dlog_tau_0 += tau_0 * (tau_0 - 0.0023) / 0.0007 ** 2                         # :60-64
    dlog_beta += beta * (beta - 3.65) / 0.21 ** 2                                # :67-71
    g = np.concatenate([dM.ravel(order="F"), dlog_omega, [dlog_c_0, dlog_tau_0, dlog_beta]])
    return f, g                                                                  # :73
