"""GPU parity of the int8 Ozaki-contraction fused path (GPDLA_PATH_FUSED_I8, kernels_i8.hip)
against the oracle's golden fixtures and against the fp64 fused kernel.

Tolerance: the north-star bound |got - ref| <= 1e-6 * max(|ref|, 1), plus a tighter 1e-8 bar for
this path (its only approximations are the 2^-31/2^-32 weight and panel quantisation and the dropped
digit levels >= 4; the numpy emulation tests/support/emulate_i8.py measures ~4e-10 on 72 bench-data samples)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from conftest import tol_ok  # noqa: E402
from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402

I8_TOL = 1e-8
KEYS = ("log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla")


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _rel_err(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    both_nan = np.isnan(got) & np.isnan(ref)
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)
    return float(np.max(np.where(both_nan, 0.0, err)))


def _run(model, samples, packed, path, **kw):
    with Engine(model, samples, set_parameters(k=model["M"].shape[1], **kw), path=path) as eng:
        return eng.process(packed)


@pytest.mark.parametrize("mode", ["reference", "unmasked"])
def test_i8_matches_golden(golden_dir, mode):
    g = np.load(golden_dir / "process.npz")
    model = {k: g[k] for k in ("rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0", "log_beta")}
    samples = dict(offset_samples=g["offset_samples"], nhi_samples=g["nhi_samples"])
    packed = {k: g[k] for k in ("offsets", "wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    out = _run(model, samples, packed, "fused_i8", absorption_mode=mode)
    for key, gkey in (("log_likelihoods_no_dla", "log_likelihood_no_dla"),
                      ("sample_log_likelihoods_dla", "sample_log_likelihoods_dla"),
                      ("log_likelihoods_dla", "log_likelihood_dla")):
        ref = g[f"{mode}_{gkey}"]
        assert np.all(tol_ok(out[key], ref)), (key, _rel_err(out[key], ref))
        assert _rel_err(out[key], ref) < I8_TOL, (key, _rel_err(out[key], ref))
    np.testing.assert_array_equal(out["num_pixels"], g[f"{mode}_n"])


def test_i8_equals_fp64_at_bench_shape():
    """configs[1] shape (n = 800, k = 20, S = 10^4) on a few spectra: the int8 path against the
    fp64 fused kernel, the calc_cddf.py:246 invariant, and run-to-run determinism."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(10000)
    packed = syn.pack_spectra(syn.make_spectra(model, 6))
    ref = _run(model, samples, packed, "fused")
    with Engine(model, samples, set_parameters(k=20), path="fused_i8") as eng:
        out = eng.process(packed)
        out2 = eng.process(packed)
    for key in KEYS:
        np.testing.assert_array_equal(out[key], out2[key])
        assert _rel_err(out[key], ref[key]) < I8_TOL, (key, _rel_err(out[key], ref[key]))
    sll, lld = out["sample_log_likelihoods_dla"], out["log_likelihoods_dla"]
    tot = np.exp(sll - (lld[:, None] + np.log(sll.shape[1]))).sum(axis=1)
    np.testing.assert_allclose(tot, 1.0, atol=1e-12)
    print("i8 vs fp64 max rel err:", {k: _rel_err(out[k], ref[k]) for k in KEYS})


def test_i8_dr12q_shapes_and_masks():
    """Ragged n (269..1250) with 5% masked pixels, both absorption modes, S not a multiple of 64."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(333)
    packed = syn.pack_spectra(syn.make_dr12q_like_spectra(model, 24, seed=5, mask_fraction=0.05))
    for mode in ("reference", "unmasked"):
        ref = _run(model, samples, packed, "fused", absorption_mode=mode)
        out = _run(model, samples, packed, "fused_i8", absorption_mode=mode)
        for key in KEYS:
            assert _rel_err(out[key], ref[key]) < I8_TOL, (mode, key, _rel_err(out[key], ref[key]))


def test_i8_edge_cases():
    """Tiny spectra (n = 1..33: a single chunk, mostly padding), an unusable spectrum (NaN outputs)."""
    model = syn.make_model(k=20, seed=3)
    samples = syn.make_samples(67)
    base = syn.make_spectrum(model, 0, z_qso=2.8, n_target=None, mask_fraction=0.1)
    spectra = []
    for npx in (1, 2, 3, 5, 9, 33, 64, 65):
        sl = slice(100, 100 + npx)
        s = {k: (v[sl] if isinstance(v, np.ndarray) else v) for k, v in base.items()}
        s["pixel_mask"] = np.zeros(npx, dtype=bool)
        spectra.append(s)
    empty = dict(base)
    empty["z_qso"] = 9.5
    spectra.append(empty)
    packed = syn.pack_spectra(spectra)
    ref = _run(model, samples, packed, "fused")
    out = _run(model, samples, packed, "fused_i8")
    for key in KEYS:
        assert _rel_err(out[key][:-1], ref[key][:-1]) < I8_TOL, (key, _rel_err(out[key][:-1], ref[key][:-1]))
        assert np.all(np.isnan(out[key][-1]))


def test_i8_unsupported_configurations_rejected():
    model = syn.make_model(k=21)  # above the int8 fused kernel's rank 20 (lower ranks run zero-padded)
    samples = syn.make_samples(8)
    with pytest.raises(L.GpdlaError):
        Engine(model, samples, set_parameters(k=21), path="fused_i8")
    model = syn.make_model(k=20)
    with pytest.raises(L.GpdlaError):
        Engine(model, samples, set_parameters(k=20, num_lines=4), path="fused_i8")


def test_i8_fused_lower_rank_runs_zero_padded():
    """k = 16 on the int8 fused kernel (compiled for 20): M padded by zero columns, whose panel entries
    quantise to zero digits -- agrees with the fp64 fused path like rank 20 does."""
    model = syn.make_model(k=16, seed=16)
    samples = syn.make_samples(130)
    spectra = syn.make_dr12q_like_spectra(model, 3, seed=16, mask_fraction=0.05)
    packed = syn.pack_spectra(spectra)
    ref = _run(model, samples, packed, "fused")
    out = _run(model, samples, packed, "fused_i8")
    for key in KEYS:
        assert _rel_err(out[key], ref[key]) < I8_TOL, (key, _rel_err(out[key], ref[key]))


def test_i8_long_spectrum_batch_falls_back_to_fp64():
    """A batch holding a spectrum longer than kI8MaxSlots (30,000 pixels: the int32 level sums stay
    exact only below that) runs on the fp64 kernel: bit-identical to path='fused'."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(64)
    base = syn.make_spectrum(model, 1)
    lo, hi = np.log10(base["wavelengths"][0]), np.log10(base["wavelengths"][-1])
    lam = 10.0 ** np.linspace(lo, hi, 30500)
    rng = np.random.default_rng(7)
    long_spec = dict(wavelengths=lam, flux=np.interp(lam, base["wavelengths"], base["flux"]),
                     noise_variance=rng.uniform(0.01, 0.09, lam.size), pixel_mask=np.zeros(lam.size, bool),
                     z_qso=base["z_qso"])
    packed = syn.pack_spectra([base, long_spec])
    ref = _run(model, samples, packed, "fused")
    out = _run(model, samples, packed, "fused_i8")
    for key in KEYS:
        np.testing.assert_array_equal(out[key], ref[key])
    assert out["num_pixels"][1] > 30000


def test_panel_gemm_i8_long_spectrum_batch_falls_back_to_fp64():
    """The same kI8MaxSlots guard on the int8 panel-GEMM path (gemm_i8.hip): the batch holding a
    30,500-pixel spectrum runs the fp64 weights + fp64 GEMM + LDL^T, bit-identical to path='panel_gemm'."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(64)
    base = syn.make_spectrum(model, 1)
    lo, hi = np.log10(base["wavelengths"][0]), np.log10(base["wavelengths"][-1])
    lam = 10.0 ** np.linspace(lo, hi, 30500)
    rng = np.random.default_rng(7)
    long_spec = dict(wavelengths=lam, flux=np.interp(lam, base["wavelengths"], base["flux"]),
                     noise_variance=rng.uniform(0.01, 0.09, lam.size), pixel_mask=np.zeros(lam.size, bool),
                     z_qso=base["z_qso"])
    packed = syn.pack_spectra([base, long_spec])
    ref = _run(model, samples, packed, "panel_gemm")
    out = _run(model, samples, packed, "panel_gemm_i8")
    for key in KEYS:
        np.testing.assert_array_equal(out[key], ref[key])
    assert out["num_pixels"][1] > 30000


# ------------------------------------------------------------ int8 panel-GEMM path (any rank)
# the 24-bit path (3 digit planes, levels <= 2): the 1e-6 north-star contract, 5e-7 regression bar
I8_24_TOL = 5e-7
PANEL_I8 = [("panel_gemm_i8", I8_TOL), ("panel_gemm_i8_24", I8_24_TOL)]


@pytest.mark.parametrize("path,tol", PANEL_I8)
@pytest.mark.parametrize("k", [1, 7, 20, 40, 50, 64])
def test_panel_gemm_i8_equals_fp64(k, path, tol):
    """The int8 panel-GEMM paths (gemm_i8.hip) against the fp64 panel-GEMM path: ragged DR12Q-shaped
    spectra with masks, 16,500 samples for k = 50.  The 24-bit path's launch layouts: k = 1 and 7, one Gram
    tile (gemm_i8_kernel<3>); k = 20, B-stationary Gram beside a u launch (no spare blocks); k = 40,
    6 / 7 Gram columns per XCD with the u tile fused on the spare blocks; k = 50 the same at 10 / 10;
    k = 64 (the largest rank), 16 / 17 columns and a u launch; spectra over 832 slots take
    gemm_i8_kernel<3> at every k."""
    model = syn.make_model(k=k, seed=k)
    S = 16500 if k == 50 else 700
    samples = syn.make_samples(S)
    packed = syn.pack_spectra(syn.make_dr12q_like_spectra(model, 3 if k == 50 else 6, seed=k, mask_fraction=0.05))
    ref = _run(model, samples, packed, "panel_gemm")
    out = _run(model, samples, packed, path)
    for key in KEYS:
        assert np.all(tol_ok(out[key], ref[key])), (k, path, key)
        assert _rel_err(out[key], ref[key]) < tol, (k, path, key, _rel_err(out[key], ref[key]))
    print(f"k={k} {path} vs fp64:", {kk: _rel_err(out[kk], ref[kk]) for kk in KEYS})


@pytest.mark.parametrize("path,tol", PANEL_I8)
def test_panel_gemm_i8_edge_cases(path, tol):
    """Tiny spectra (n = 1..65: one K step, mostly padding) and an unusable spectrum (NaN outputs) on
    each int8 panel path, against the fp64 panel path at that path's own bar (process_qsos.m:96-120,
    184-198)."""
    model = syn.make_model(k=50, seed=3)
    samples = syn.make_samples(67)
    base = syn.make_spectrum(model, 0, z_qso=2.8, n_target=None, mask_fraction=0.1)
    spectra = []
    for npx in (1, 3, 9, 33, 65):
        sl = slice(100, 100 + npx)
        s = {kk: (v[sl] if isinstance(v, np.ndarray) else v) for kk, v in base.items()}
        s["pixel_mask"] = np.zeros(npx, dtype=bool)
        spectra.append(s)
    empty = dict(base)
    empty["z_qso"] = 9.5
    spectra.append(empty)
    packed = syn.pack_spectra(spectra)
    ref = _run(model, samples, packed, "panel_gemm")
    out = _run(model, samples, packed, path)
    for key in KEYS:
        err = _rel_err(out[key][:-1], ref[key][:-1])
        assert np.all(tol_ok(out[key][:-1], ref[key][:-1])), (path, key, err)
        assert err < tol, (path, key, err)
        assert np.all(np.isnan(out[key][-1])), (path, key)
    np.testing.assert_array_equal(out["num_pixels"], ref["num_pixels"])
    print(f"{path} edge cases vs fp64:", {kk: _rel_err(out[kk][:-1], ref[kk][:-1]) for kk in KEYS})


def test_panel_gemm_i8_24_short_spectra_take_32_bit_digits():
    """The 24-bit path's error is absolute (~2^-24 of the Gram's scale), so relative to max(|ll|, 1) it
    is largest where |ll| is small -- short spectra (n = 3: 5.05e-7, profiles/round5/r10b).  Spectra of
    <= 128 pixels (kI8NarrowKs = 2 K steps, internal.h) take the 32-bit digits on that path: bitwise the
    panel_gemm_i8 results, in a batch mixed with longer spectra that keep the 24-bit scheme."""
    model = syn.make_model(k=50, seed=4)
    samples = syn.make_samples(300)
    base = syn.make_spectrum(model, 2, z_qso=2.8, n_target=None, mask_fraction=0.0)
    spectra = []
    for npx in (2, 64, 128, 129, 400):
        sl = slice(50, 50 + npx)
        s = {kk: (v[sl] if isinstance(v, np.ndarray) else v) for kk, v in base.items()}
        s["pixel_mask"] = np.zeros(npx, dtype=bool)
        spectra.append(s)
    packed = syn.pack_spectra(spectra)
    o32 = _run(model, samples, packed, "panel_gemm_i8")
    o24 = _run(model, samples, packed, "panel_gemm_i8_24")
    ref = _run(model, samples, packed, "panel_gemm")
    short = np.array([n <= 128 for n in (2, 64, 128, 129, 400)])
    for key in KEYS:
        np.testing.assert_array_equal(o24[key][short], o32[key][short])
        assert not np.array_equal(o24[key][~short], o32[key][~short]), key   # 24-bit digits there
        assert _rel_err(o24[key], ref[key]) < I8_24_TOL, (key, _rel_err(o24[key], ref[key]))


@pytest.mark.parametrize("S", [300, 1400, 3000])
def test_bst_pipeline_every_stream_length(S):
    """gemm_i8_bst_kernel's A pipeline (gemm_i8.hip bst_run) has three shapes by a wave's K-step count
    total = (sample tiles) x (64-slot K steps): one step at a time below NS + DEPTH = 5, otherwise the
    unguarded main loop and a tail of R = 2, 3 or 4 steps.  Spectra of 3..13 K steps (129..832 pixels,
    the B-stationary range) at 300 / 1,400 / 3,000 samples (1, 1-3, 1-6 sample tiles per wave) reach
    every shape, for the Gram role and the u role; each must agree with the fp64 panel path at the
    24-bit bar.  (A missing B read on the short path gave NaN at 129 pixels, caught by
    test_panel_gemm_i8_24_short_spectra_take_32_bit_digits.)"""
    model = syn.make_model(k=50, seed=11)
    samples = syn.make_samples(S)
    base = syn.make_spectrum(model, 5, z_qso=3.4, n_target=None, mask_fraction=0.0)
    i0 = int(np.searchsorted(base["wavelengths"] / (1 + base["z_qso"]), 912.0))   # first in-range pixel
    assert base["wavelengths"].size - i0 >= 832
    spectra = []
    for npx in (129, 193, 257, 321, 385, 449, 513, 577, 641, 705, 769, 832):
        sl = slice(i0, i0 + npx)
        spectra.append({kk: (v[sl] if isinstance(v, np.ndarray) else v) for kk, v in base.items()})
    packed = syn.pack_spectra(spectra)
    ref = _run(model, samples, packed, "panel_gemm")
    out = _run(model, samples, packed, "panel_gemm_i8_24")
    for key in KEYS:
        assert np.all(np.isfinite(out[key])), key
        assert _rel_err(out[key], ref[key]) < I8_24_TOL, (S, key, _rel_err(out[key], ref[key]))


def _raw_profile(lam, z, N, f32):
    import ctypes as C
    lam = np.ascontiguousarray(lam, dtype=np.float64)
    out = np.empty_like(lam)
    L.check(L.load().gpdla_diag_raw_profile3(L.ptr(lam), lam.size, z, N, 1 if f32 else 0, L.ptr(out)))
    return out


def test_weights_fp32_raw_profile_against_fp64():
    """The 24-bit path's packed-fp32 raw profile (gemm_i8.hip raw_profile3_pair_f32: x_j in fp64, T_j
    from one fp32 reciprocal, the outer wing polynomial on fp32 coefficients, exp2f) against the fp64
    profile of the 32-bit path and the oracle (scipy's Faddeeva), through the kernels' own device
    functions (gpdla_diag_raw_profile3), over z, N and velocity sweeps that cross every line's core,
    inner-wing and outer-wing zones -- densely at the |x| = kOuterX = 32 switch (411 km/s), where the
    fp32 lanes hand over to the fp64 fix-up (emulate_f32_profile rounds only the results)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from oracle import gpdla_oracle as O
    kms = 1e5
    x32 = 32 * O.SIGMA * np.sqrt(2)          # |x| = 32 in cm/s
    vels = np.concatenate([np.arange(-3000, 3000, 0.5) * kms,
                           x32 + np.linspace(-2, 2, 4001) * kms, -x32 + np.linspace(-2, 2, 4001) * kms])
    worst = {"abs": 0.0, "rel": 0.0, "oracle64": 0.0}
    for z in (2.2, 3.0, 4.5):
        for N in (1e19, 10 ** 20.3, 1e21, 1e22):
            for j in range(3):
                lam = (O.C_CGS + vels) * O.TRANSITION_WAVELENGTHS[j] * (1 + z) * 1e8 / O.C_CGS
                a32 = _raw_profile(lam, z, N, True)
                a64 = _raw_profile(lam, z, N, False)
                mult = O.C_CGS / (O.TRANSITION_WAVELENGTHS[:3] * (1 + z)) / 1e8
                tot = sum(O.LEADING_CONSTANTS[i] * O.libcerf_voigt(lam * mult[i] - O.C_CGS, O.SIGMA, O.LORENTZ_GAMMAS[i])
                          for i in range(3))
                ref = np.exp(-N * tot)
                assert np.all(np.isfinite(a32)) and np.all((a32 >= 0) & (a32 <= 1))
                e64 = np.abs(a64 - ref)
                if e64.max() > worst["oracle64"]:
                    i = int(np.argmax(e64))
                    worst["oracle64"] = float(e64[i])
                    worst["oracle64_at"] = dict(z=z, N=N, line=j, vel_kms=float(vels[i] / kms), a=float(ref[i]))
                worst["abs"] = max(worst["abs"], float(np.max(np.abs(a32 - a64))))
                big = a64 > 1e-4
                worst["rel"] = max(worst["rel"], float(np.max(np.abs(a32 - a64)[big] / a64[big])))
    print("raw profile fp32 vs fp64:", worst)
    assert worst["oracle64"] < 1e-10, worst          # fp64 profile vs scipy's Faddeeva (measured 1.6e-11)
    assert worst["abs"] < 1e-6, worst                 # fp32: an absorption in [0, 1] to ~2^-20
    assert worst["rel"] < 1e-5, worst                 # and relative where it is not negligible


@pytest.mark.parametrize("path", ["panel_gemm", "panel_gemm_i8", "panel_gemm_i8_24"])
@pytest.mark.parametrize("batch", [0, 3])
def test_panel_gemm_two_streams_bitwise(path, batch):
    """gpdla_engine_set_panel_streams: a batch's spectra alternating over two compute streams (own
    workspace per stream, forked from and joined into the engine's stream) give bitwise the one-stream
    results -- ragged spectra in one batch, or batches of 3 (the last one a single spectrum); 3 streams
    likewise; 1..4 are the accepted values."""
    model = syn.make_model(k=50, seed=11)
    samples = syn.make_samples(3001)
    packed = syn.pack_spectra(syn.make_dr12q_like_spectra(model, 7, seed=11, mask_fraction=0.05))
    with Engine(model, samples, set_parameters(k=50), max_batch_spectra=batch, path=path) as eng:
        eng.set_panel_streams(1)
        one = eng.process(packed)
        eng.set_panel_streams(2)
        two = eng.process(packed)
        again = eng.process(packed)
        eng.set_panel_streams(3)
        three = eng.process(packed)
        eng.set_panel_streams(2)
        for bad in (0, 5):
            with pytest.raises(L.GpdlaError):
                eng.set_panel_streams(bad)
    for key in KEYS:
        np.testing.assert_array_equal(two[key], one[key])
        np.testing.assert_array_equal(again[key], one[key])
        np.testing.assert_array_equal(three[key], one[key])
    assert np.all(np.isfinite(two["sample_log_likelihoods_dla"]))
