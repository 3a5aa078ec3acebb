"""GPU parity: the HIP path (through the C ABI) against the oracle's committed golden fixtures,
plus size-independent properties at the BASELINE configuration sizes.

Tolerance (north star, BASELINE.json): per-spectrum log evidences within 1e-6 relative, written
as |got - ref| <= 1e-6 * max(|ref|, 1).  The measured agreement is ~1e-10 or better; the tests
also assert a tighter 1e-9 bar so a precision regression is caught long before the contract."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from conftest import tol_ok  # noqa: E402
from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine, log_mvnpdf_low_rank, voigt, voigt_batch  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    lib = L.load()
    assert lib.gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


@pytest.fixture(scope="module")
def golden(golden_dir):
    g = np.load(golden_dir / "process.npz")
    model = {k: g[k] for k in ("rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0", "log_beta")}
    samples = dict(offset_samples=g["offset_samples"], nhi_samples=g["nhi_samples"])
    packed = {k: g[k] for k in ("offsets", "wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    return g, model, samples, packed


def _rel_err(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))


# ------------------------------------------------------------------------------ voigt MEX
def test_voigt_matches_golden(golden_dir):
    g = np.load(golden_dir / "voigt.npz")
    for i in range(g["z"].size):
        ref = g[f"out_{i}"]
        got = voigt(g[f"lam_{i}"], g["z"][i], g["N"][i], int(g["num_lines"][i]))
        assert got.shape == ref.shape
        # absorption in [0,1]; absolute agreement + relative where the value is not underflowed
        assert np.max(np.abs(got - ref)) < 1e-12
        big = ref > 1e-200
        assert np.max(np.abs(got[big] - ref[big]) / ref[big]) < 1e-9


def test_voigt_batch_equals_single(golden_dir):
    g = np.load(golden_dir / "voigt.npz")
    lam = g["lam_0"]
    zs, Ns = g["z"][:4], g["N"][:4]
    batch = voigt_batch(lam, zs, Ns, 3)
    for i in range(4):
        np.testing.assert_array_equal(batch[i], voigt(lam, zs[i], Ns[i], 3))


# ------------------------------------------------------------------------ log_mvnpdf
def test_log_mvnpdf_matches_golden(golden_dir):
    g = np.load(golden_dir / "mvn.npz")
    for i in range(4):
        got = log_mvnpdf_low_rank(g[f"y_{i}"], g[f"mu_{i}"], g[f"M_{i}"], g[f"d_{i}"])
        ref = float(g[f"out_{i}"])
        assert abs(got - ref) <= 1e-10 * max(1, abs(ref))


def test_log_mvnpdf_non_pd_raises():
    with pytest.raises(L.GpdlaNumericError):
        log_mvnpdf_low_rank(np.ones(4), np.zeros(4), np.ones((4, 2)), -np.ones(4) * 10)


# ------------------------------------------------------------------------ engine
@pytest.mark.parametrize("mode", ["reference", "unmasked"])
def test_engine_matches_golden(golden, mode):
    g, model, samples, packed = golden
    params = set_parameters(k=20, absorption_mode=mode)
    with Engine(model, samples, params) as eng:
        out = eng.process(packed)
    pre = f"{mode}_"
    for key, gkey in (("log_likelihoods_no_dla", "log_likelihood_no_dla"),
                      ("sample_log_likelihoods_dla", "sample_log_likelihoods_dla"),
                      ("log_likelihoods_dla", "log_likelihood_dla")):
        ref = g[pre + gkey]
        assert np.all(tol_ok(out[key], ref)), (key, _rel_err(out[key], ref))
        assert _rel_err(out[key], ref) < 1e-9, (key, _rel_err(out[key], ref))
    np.testing.assert_allclose(out["min_z_dlas"], g[pre + "min_z_dla"], rtol=1e-14)
    np.testing.assert_allclose(out["max_z_dlas"], g[pre + "max_z_dla"], rtol=1e-14)
    np.testing.assert_array_equal(out["num_pixels"], g[pre + "n"])


def test_engine_batching_and_sharding_bitwise(golden):
    g, model, samples, packed = golden
    params = set_parameters(k=20)
    with Engine(model, samples, params) as eng:
        full = eng.process(packed)
    with Engine(model, samples, params, max_batch_spectra=3) as eng:
        batched = eng.process(packed)
        # shard: spectra 0..3 and 4..7 processed separately
        parts = []
        for lo, hi in ((0, 4), (4, 8)):
            sub = syn.pack_spectra([_unpack(packed, q) for q in range(lo, hi)])
            parts.append(eng.process(sub))
    for key in ("log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla"):
        np.testing.assert_array_equal(batched[key], full[key])
        np.testing.assert_array_equal(np.concatenate([p[key] for p in parts]), full[key])


def _unpack(packed, q):
    a, b = packed["offsets"][q], packed["offsets"][q + 1]
    return dict(wavelengths=packed["wavelengths"][a:b], flux=packed["flux"][a:b],
                noise_variance=packed["noise_variance"][a:b], pixel_mask=packed["pixel_mask"][a:b],
                z_qso=packed["z_qsos"][q])


def test_edge_cases_small_and_empty():
    """Tiny spectra (J not a multiple of 4, n < 4), an unusable spectrum (no in-range pixel),
    S not a multiple of the 64-sample block, and one / 31 Lyman lines."""
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=8, seed=3)
    samples = syn.make_samples(67)
    base = syn.make_spectrum(model, 0, z_qso=2.8, n_target=None, mask_fraction=0.1)
    spectra = []
    for npx in (1, 2, 3, 5, 9, 33):
        s = dict(base)
        sl = slice(100, 100 + npx)
        spectra.append({k: (v[sl] if isinstance(v, np.ndarray) else v) for k, v in s.items()})
        spectra[-1]["pixel_mask"] = np.zeros(npx, dtype=bool)
    empty = dict(base)
    empty["z_qso"] = 9.5  # nothing in range
    spectra.append(empty)
    packed = syn.pack_spectra(spectra)
    for nl in (1, 31):
        params = set_parameters(k=8, num_lines=nl)
        with Engine(model, samples, params) as eng:
            out = eng.process(packed)
        for q, s in enumerate(spectra[:-1]):
            ref = O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                     s["z_qso"], model, samples["offset_samples"], samples["nhi_samples"],
                                     num_lines=nl)
            assert _rel_err(out["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"]) < 1e-9
            assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < 1e-9
            assert _rel_err(out["log_likelihoods_dla"][q], ref["log_likelihood_dla"]) < 1e-9
        assert np.isnan(out["log_likelihoods_dla"][-1]) and np.isnan(out["log_likelihoods_no_dla"][-1])
        assert np.all(np.isnan(out["sample_log_likelihoods_dla"][-1]))


@pytest.mark.parametrize("S", [1, 2])
@pytest.mark.parametrize("path,tol", [("fused", 1e-9), ("panel_gemm", 1e-9), ("fused_i8", 1e-8),
                                      ("panel_gemm_i8", 1e-8), ("panel_gemm_i8_24", 5e-7)])
def test_one_and_two_dla_samples(S, path, tol):
    """num_dla_samples of 1 and 2 (process_qsos.m:184-212 with S = 1, 2) on every likelihood path:
    the 64-sample blocks, 128-sample GEMM tiles and 16-sample LDL^T blocks almost empty, against the
    oracle; with one sample the log-mean-exp is that sample's value exactly (:202-209)."""
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=20, seed=S)
    samples = syn.make_samples(S)
    spectra = syn.make_dr12q_like_spectra(model, 3, seed=S, mask_fraction=0.05)
    with Engine(model, samples, set_parameters(k=20), path=path) as eng:
        out = eng.process(syn.pack_spectra(spectra))
    assert out["sample_log_likelihoods_dla"].shape == (3, S)
    for q, sp in enumerate(spectra):
        ref = O.process_spectrum(sp["wavelengths"], sp["flux"], sp["noise_variance"], sp["pixel_mask"],
                                 sp["z_qso"], model, samples["offset_samples"], samples["nhi_samples"])
        assert _rel_err(out["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"]) < tol, (path, q)
        assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < tol, (path, q)
        assert _rel_err(out["log_likelihoods_dla"][q], ref["log_likelihood_dla"]) < tol, (path, q)
    if S == 1:
        np.testing.assert_array_equal(out["log_likelihoods_dla"], out["sample_log_likelihoods_dla"][:, 0])


@pytest.mark.parametrize("k", [4, 10, 16, 24])
def test_other_ranks(k):
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=k, seed=k)
    samples = syn.make_samples(40)
    spectra = syn.make_dr12q_like_spectra(model, 2, seed=k, mask_fraction=0.05)
    with Engine(model, samples, set_parameters(k=k)) as eng:
        out = eng.process(syn.pack_spectra(spectra))
    for q, s in enumerate(spectra):
        ref = O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                 s["z_qso"], model, samples["offset_samples"], samples["nhi_samples"])
        assert _rel_err(out["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"]) < 1e-9
        assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < 1e-9


@pytest.mark.parametrize("G", [300, 1217, 5000])
@pytest.mark.parametrize("path", ["auto", "panel_gemm"])
def test_nonuniform_rest_grids(G, path):
    """prep_kernel's interpolation index (a two-round 64-way lane search for grids up to 4,097
    points, the binary search above) on jittered, non-uniform rest grids of 300, 1,217 and 5,000
    points, against the oracle's np.interp (process_qsos.m:66-71,139-142)."""
    from oracle import gpdla_oracle as O
    rng = np.random.default_rng(G)
    base = syn.make_model(k=20, seed=G)
    lo, hi = base["rest_wavelengths"][0], base["rest_wavelengths"][-1]
    grid = np.concatenate(([lo], np.sort(rng.uniform(lo, hi, G - 2)), [hi]))
    model = dict(base, rest_wavelengths=grid,
                 mu=np.interp(grid, base["rest_wavelengths"], base["mu"]),
                 M=np.asfortranarray(np.stack([np.interp(grid, base["rest_wavelengths"], base["M"][:, j])
                                               for j in range(20)], axis=1)),
                 log_omega=np.interp(grid, base["rest_wavelengths"], base["log_omega"]))
    samples = syn.make_samples(40)
    spectra = syn.make_dr12q_like_spectra(model, 2, seed=G, mask_fraction=0.05)
    with Engine(model, samples, set_parameters(k=20), path=path) as eng:
        out = eng.process(syn.pack_spectra(spectra))
    for q, s in enumerate(spectra):
        ref = O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                 s["z_qso"], model, samples["offset_samples"], samples["nhi_samples"])
        assert _rel_err(out["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"]) < 1e-9
        assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < 1e-9


@pytest.mark.parametrize("k", [1, 3, 7, 9, 13, 17, 23])
def test_ranks_between_compiled_ones_run_fused_zero_padded(k):
    """A rank the fused kernel is not compiled for runs on the next compiled rank with M padded by
    zero columns (engine.hip, fused_rank): against the oracle, and against the fp64 panel-GEMM path
    that runs the rank natively."""
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=k, seed=200 + k)
    samples = syn.make_samples(40)
    spectra = syn.make_dr12q_like_spectra(model, 2, seed=k, mask_fraction=0.05)
    packed = syn.pack_spectra(spectra)
    with Engine(model, samples, set_parameters(k=k)) as eng:
        out = eng.process(packed)
    with Engine(model, samples, set_parameters(k=k), path="panel_gemm") as eng:
        gemm = eng.process(packed)
    for key in ("sample_log_likelihoods_dla", "log_likelihoods_no_dla", "log_likelihoods_dla"):
        assert _rel_err(out[key], gemm[key]) < 1e-11, key
    for q, s in enumerate(spectra):
        ref = O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                 s["z_qso"], model, samples["offset_samples"], samples["nhi_samples"])
        assert _rel_err(out["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"]) < 1e-9
        assert _rel_err(out["log_likelihoods_no_dla"][q], ref["log_likelihood_no_dla"]) < 1e-9


def test_zero_padded_rank_is_bitwise_the_native_rank():
    """The padding is exact: rank 8 on likelihood_kernel<8> and the same model with two zero columns
    appended (rank 10, likelihood_kernel<10>) give bit-identical outputs."""
    model = syn.make_model(k=8, seed=88)
    padded = dict(model)
    padded["M"] = np.asfortranarray(np.concatenate([model["M"], np.zeros((model["M"].shape[0], 2))], axis=1))
    samples = syn.make_samples(70)
    spectra = syn.make_dr12q_like_spectra(model, 3, seed=8, mask_fraction=0.05)
    packed = syn.pack_spectra(spectra)
    with Engine(model, samples, set_parameters(k=8), path="fused") as eng:
        a = eng.process(packed)
    with Engine(padded, samples, set_parameters(k=10), path="fused") as eng:
        b = eng.process(packed)
    for key in ("sample_log_likelihoods_dla", "log_likelihoods_no_dla", "log_likelihoods_dla"):
        assert np.array_equal(a[key], b[key]), key


# ------------------------------------------------------------------ full-size properties
def test_full_size_config_properties():
    """BASELINE configs[1] shape (n = 800, k = 20, S = 10^4): oracle spot checks on a sample subset,
    the calc_cddf.py:246 normalisation invariant, determinism and host/device-path equality."""
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=20)
    samples = syn.make_samples(10000)
    spectra = syn.make_spectra(model, 3)
    packed = syn.pack_spectra(spectra)
    with Engine(model, samples, set_parameters(k=20)) as eng:
        out1 = eng.process(packed)
        out2 = eng.process(packed)
    for key in ("log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla"):
        np.testing.assert_array_equal(out1[key], out2[key])
    assert np.all(out1["num_pixels"] == 800)
    sll, lld = out1["sample_log_likelihoods_dla"], out1["log_likelihoods_dla"]
    tot = np.exp(sll - (lld[:, None] + np.log(sll.shape[1]))).sum(axis=1)
    np.testing.assert_allclose(tot, 1.0, atol=1e-12)
    rng = np.random.default_rng(0)
    idx = np.sort(rng.choice(10000, 24, replace=False))
    idx[:2] = [0, 9999]
    s = spectra[0]
    prep = O.prepare_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"], s["z_qso"], model)
    zs = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * samples["offset_samples"][idx]
    ref = np.array([O.sample_log_likelihood(prep, z, N, 3) for z, N in zip(zs, samples["nhi_samples"][idx])])
    assert _rel_err(sll[0, idx], ref) < 1e-9
    assert _rel_err(out1["log_likelihoods_no_dla"][0], O.null_log_likelihood(prep)) < 1e-9


def test_device_path_equals_host_path():
    model = syn.make_model(k=20)
    samples = syn.make_samples(1000)
    packed = syn.pack_spectra(syn.make_spectra(model, 4))
    D = L.DeviceArray.from_numpy
    t = {k: D(packed[k]) for k in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    Q = packed["z_qsos"].size
    o_null, o_dla = L.DeviceArray(0, Q, np.float64), L.DeviceArray(0, Q, np.float64)
    o_s = L.DeviceArray(0, (Q, 1000), np.float64)
    with Engine(model, samples, set_parameters(k=20)) as eng:
        host = eng.process(packed)
        eng.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                           t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, 1000)
        eng.synchronize()
        st = eng.stats()
    np.testing.assert_array_equal(o_null.numpy(), host["log_likelihoods_no_dla"])
    np.testing.assert_array_equal(o_dla.numpy(), host["log_likelihoods_dla"])
    np.testing.assert_array_equal(o_s.numpy(), host["sample_log_likelihoods_dla"])
    assert st["likelihood_launches"] == 2 and st["likelihood_ms"] > 0


@pytest.mark.parametrize("path", ["auto", "fused_i8", "panel_gemm"])
def test_host_pipeline_equals_device_path(path):
    """The host-buffer pipeline (engine.hip: two device stages, inputs in and results out on a copy
    stream beside the kernels) against the device-resident call, bitwise: 37 DR12Q-shaped spectra
    in batches of 4 (10 batches, the last partial), then a second, longer call on the same engine
    (its stages grow), results without the sample array, and one batch."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(300)
    spectra = syn.make_dr12q_like_spectra(model, 53, seed=4)
    D = L.DeviceArray.from_numpy

    def device_run(eng, packed):
        t = {k: D(packed[k]) for k in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
        Q = packed["z_qsos"].size
        o = [L.DeviceArray(0, Q, np.float64) for _ in range(2)] + [L.DeviceArray(0, (Q, 300), np.float64)]
        eng.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                           t["pixel_mask"].ptr, t["z_qsos"].ptr, o[0].ptr, o[1].ptr, o[2].ptr, 300)
        eng.synchronize()
        return [x.numpy() for x in o]

    with Engine(model, samples, set_parameters(k=20), max_batch_spectra=4, path=path) as eng:
        for sel in (slice(0, 37), slice(0, 53), slice(40, 43)):
            packed = syn.pack_spectra(spectra[sel])
            host = eng.process(packed)
            dev = device_run(eng, packed)
            np.testing.assert_array_equal(host["log_likelihoods_no_dla"], dev[0])
            np.testing.assert_array_equal(host["log_likelihoods_dla"], dev[1])
            np.testing.assert_array_equal(host["sample_log_likelihoods_dla"], dev[2])
        scalars = eng.process(packed, want_samples=False)
        np.testing.assert_array_equal(scalars["log_likelihoods_dla"], dev[1])
        assert "sample_log_likelihoods_dla" not in scalars


TORCH_INTEROP = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch                                   # first: its HIP runtime is the one libgpdla binds to
from gp_dla_detection_amd import synthetic as syn, _lib as L
from gp_dla_detection_amd.engine import Engine
from gp_dla_detection_amd.parameters import set_parameters
maps = open('/proc/self/maps').read()
dev = torch.device('cuda:0')
model = syn.make_model(k=20); samples = syn.make_samples(200)
packed = syn.pack_spectra(syn.make_spectra(model, 3))
t = {k: torch.from_numpy(np.ascontiguousarray(packed[k])).to(dev)
     for k in ('wavelengths', 'flux', 'noise_variance', 'pixel_mask', 'z_qsos')}
o_null = torch.empty(3, dtype=torch.float64, device=dev); o_dla = torch.empty_like(o_null)
o_s = torch.empty((3, 200), dtype=torch.float64, device=dev)
# the fused path, and the int8 panel path whose spectra alternate over two streams forked from and
# joined into torch's stream; torch's default (null) stream and a side stream.  The torch ops after
# the call are ordered on torch's stream only and must see every spectrum's results.
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.default_stream(dev))   # the inputs above were uploaded on the default stream
for path in ('auto', 'panel_gemm_i8_24'):
    for ts in (torch.cuda.default_stream(dev), side):
        with torch.cuda.stream(ts), Engine(model, samples, set_parameters(k=20), path=path) as eng:
            host = eng.process(packed)
            o_s.fill_(7.0)
            o_dla.fill_(7.0)
            eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            eng.process_device(packed['offsets'], t['wavelengths'].data_ptr(), t['flux'].data_ptr(),
                               t['noise_variance'].data_ptr(), t['pixel_mask'].data_ptr(), t['z_qsos'].data_ptr(),
                               o_null.data_ptr(), o_dla.data_ptr(), o_s.data_ptr(), 200)
            got_s, got_dla = o_s.cpu().numpy(), o_dla.cpu().numpy()
            eng.synchronize()
        assert np.array_equal(got_s, host['sample_log_likelihoods_dla']), (path, ts)
        assert np.array_equal(got_dla, host['log_likelihoods_dla']), (path, ts)
libs = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}
assert len(libs) == 1, libs
print('torch interop ok', libs)
"""


def test_torch_tensor_interop():
    """PyTorch tensors as engine buffers, the engine on torch's stream (fused path, and the int8 panel
    path with its two compute streams): torch imported first so the process holds ONE HIP runtime
    (torch ships its own libamdhip64 with the same SONAME)."""
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    r = subprocess.run([sys.executable, "-c", TORCH_INTEROP, root], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "torch interop ok" in r.stdout


def test_standalone_entry_points_timed(golden_dir, tmp_path):
    """The MEX drop-ins keep their device buffers between calls: time one call
    of each after warm-up (a MATLAB parfor body calls them once per sample) and check the cached
    path returns the same values as the first call.  The times are a printed record, not asserted
    (a shared box's wall clock is no test criterion)."""
    import json
    import os
    import time
    g = np.load(golden_dir / "voigt.npz")
    lam = g["lam_0"]
    first = voigt(lam, g["z"][0], g["N"][0], 3)
    m = np.load(golden_dir / "mvn.npz")
    args = (m["y_0"], m["mu_0"], m["M_0"], m["d_0"])
    mfirst = log_mvnpdf_low_rank(*args)
    t0 = time.perf_counter()
    for _ in range(200):
        got = voigt(lam, g["z"][0], g["N"][0], 3)
    tv = (time.perf_counter() - t0) / 200
    t0 = time.perf_counter()
    for _ in range(200):
        mg = log_mvnpdf_low_rank(*args)
    tm = (time.perf_counter() - t0) / 200
    np.testing.assert_array_equal(got, first)
    assert mg == mfirst
    rec = {"voigt_f64_call_us": tv * 1e6, "n_padded": int(lam.size),
           "log_mvnpdf_low_rank_f64_call_us": tm * 1e6, "n": int(m["y_0"].size), "k": int(m["M_0"].shape[1])}
    print(json.dumps(rec))
    (tmp_path / "standalone_timing.json").write_text(json.dumps(rec))   # the record is the printed line
