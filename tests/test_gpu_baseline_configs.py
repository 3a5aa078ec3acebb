"""GPU parity at the BASELINE.json configuration sizes (not reduced ones).

* configs[1]: all 1,024 synthetic spectra x 10^4 DLA samples, k = 20, on the benched fp64 path.
* configs[2]: the full DR12Q count, 162,861 DR12Q-shaped spectra x 10^4 samples on one GPU with
  device-resident outputs (13 GB of sample log-likelihoods).
* configs[4]: k = 50, 10^5 samples, 16 spectra on the benched int8 panel-GEMM path, against the
  oracle and against the fp64 panel-GEMM path.

Every spectrum is checked against the reference's own output invariant (calc_cddf.py:246:
sum_s exp(ll_s - (ll_DLA + log S)) == 1, asserted to 1e-12 as SURVEY.md section 4 asks) and the
oracle (process_qsos.m:150-152,184-209 / log_mvnpdf_low_rank.m:22-32 restated in
oracle/gpdla_oracle.py) is evaluated on random (spectrum, sample) pairs and null models.
Tolerance: the north-star 1e-6 * max(|ref|, 1) contract, plus a 1e-9 regression bar on the fp64
paths (1e-8 on the int8 contraction, whose measured deviation is ~4e-9)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from conftest import tol_ok  # noqa: E402
from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _rel(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)))


def _invariant(sll, lld):
    """calc_cddf.py:246 (0.95 < sum < 1.05 there; exactly 1 by process_qsos.m:202-209)."""
    S = sll.shape[1]
    return np.exp(sll - (lld[:, None] + np.log(S))).sum(axis=1)


def _oracle_spot_checks(spectra, model, samples, sll, null, pairs, num_lines=3):
    """(q, s) pairs and the null model of every spectrum in `null`, against the oracle."""
    from oracle import gpdla_oracle as O
    preps = {}

    def prep(q):
        if q not in preps:
            s = spectra[q]
            preps[q] = O.prepare_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"],
                                          s["z_qso"], model)
        return preps[q]
    got, ref = [], []
    for q, si in pairs:
        p = prep(q)
        z = p["zmin"] + (p["zmax"] - p["zmin"]) * samples["offset_samples"][si]
        ref.append(O.sample_log_likelihood(p, z, samples["nhi_samples"][si], num_lines))
        got.append(sll(q, si))
    nref = [O.null_log_likelihood(prep(q)) for q in null]
    return np.array(got), np.array(ref), np.array(nref)


def test_config1_full_1024x10k():
    """configs[1] at full size: 1,024 spectra x 10^4 samples, n = 800, k = 20, fp64."""
    model = syn.make_model(k=20)
    samples = syn.make_samples(10000)
    spectra = [syn.make_spectrum(model, q) for q in range(1024)]
    with Engine(model, samples, set_parameters(k=20)) as eng:
        out = eng.process(syn.pack_spectra(spectra))
    sll, lld, lln = out["sample_log_likelihoods_dla"], out["log_likelihoods_dla"], out["log_likelihoods_no_dla"]
    assert "numeric_warning" not in out
    assert np.all(out["num_pixels"] == 800)
    assert np.isfinite(sll).all() and np.isfinite(lld).all() and np.isfinite(lln).all()
    np.testing.assert_allclose(_invariant(sll, lld), 1.0, rtol=0, atol=1e-12)
    rng = np.random.default_rng(11)
    pairs = list(zip(rng.integers(0, 1024, 64), rng.integers(0, 10000, 64))) + [(0, 0), (1023, 9999)]
    null = list(range(0, 1024, 8)) + [1023]
    got, ref, nref = _oracle_spot_checks(spectra, model, samples, lambda q, s: sll[q, s], null, pairs)
    assert np.all(tol_ok(got, ref)) and _rel(got, ref) < 1e-9, _rel(got, ref)
    assert np.all(tol_ok(lln[null], nref)) and _rel(lln[null], nref) < 1e-9, _rel(lln[null], nref)


def test_config4_panel_gemm_i8_k50_100k():
    """configs[4] on the int8 panel paths: k = 50, 10^5 samples, 16 spectra, on panel_gemm_i8_24
    (the benched path: 24-bit operand digits, levels <= 2) and panel_gemm_i8 (32-bit, levels <= 3).
    Oracle spot checks, the invariant, and agreement with the fp64 panel-GEMM path on every output:
    1e-8 for the 32-bit contraction, the 1e-6 north-star contract (|d| <= 1e-6 max(|ref|, 1)) with a
    5e-7 regression bar for the 24-bit one (emulated: 1.6e-7, tests/support/emulate_i8.py)."""
    model = syn.make_model(k=50)
    samples = syn.make_samples(100000)
    spectra = [syn.make_spectrum(model, q) for q in range(16)]
    packed = syn.pack_spectra(spectra)
    params = set_parameters(k=50)
    outs = {}
    for path in ("panel_gemm_i8_24", "panel_gemm_i8", "panel_gemm"):
        with Engine(model, samples, params, path=path) as eng:
            outs[path] = eng.process(packed)
    f64 = outs["panel_gemm"]
    for out in outs.values():
        assert "numeric_warning" not in out and np.isfinite(out["sample_log_likelihoods_dla"]).all()
        np.testing.assert_allclose(_invariant(out["sample_log_likelihoods_dla"], out["log_likelihoods_dla"]),
                                   1.0, rtol=0, atol=1e-12)
    for path, bar in (("panel_gemm_i8", 1e-8), ("panel_gemm_i8_24", 5e-7)):
        for key in ("sample_log_likelihoods_dla", "log_likelihoods_dla", "log_likelihoods_no_dla"):
            err = _rel(outs[path][key], f64[key])
            print(f"{path} {key} vs fp64: {err:.2e}")
            assert np.all(tol_ok(outs[path][key], f64[key])) and err < bar, (path, key, err)
    rng = np.random.default_rng(12)
    pairs = list(zip(rng.integers(0, 16, 48), rng.integers(0, 100000, 48))) + [(0, 0), (15, 99999)]
    for path, bar in (("panel_gemm_i8_24", 5e-7), ("panel_gemm_i8", 1e-8), ("panel_gemm", 1e-9)):
        out = outs[path]
        sll = out["sample_log_likelihoods_dla"]
        got, ref, nref = _oracle_spot_checks(spectra, model, samples, lambda q, s: sll[q, s], range(16), pairs)
        assert np.all(tol_ok(got, ref)) and _rel(got, ref) < bar, (path, _rel(got, ref))
        lln = out["log_likelihoods_no_dla"]
        assert np.all(tol_ok(lln, nref)) and _rel(lln, nref) < bar, (path, _rel(lln, nref))


def _dr12q_device_inputs(pool_packed, idx):
    """Device CSR inputs for spectra ``idx`` of the tiled DR12Q-shaped pool (spectrum i = pool entry
    idx[i]), built from the packed pool without materialising per-spectrum host copies."""
    pp = pool_packed
    lens = np.diff(pp["offsets"])
    offsets = np.zeros(idx.size + 1, np.int64)
    np.cumsum(lens[idx], out=offsets[1:])
    starts = pp["offsets"][idx]
    pix = (np.repeat(starts - offsets[:-1], lens[idx]) + np.arange(offsets[-1])).astype(np.int64)
    dev = {key: L.DeviceArray.from_numpy(pp[key][pix]) for key in ("wavelengths", "flux", "noise_variance",
                                                                     "pixel_mask")}
    dev["z_qsos"] = L.DeviceArray.from_numpy(pp["z_qsos"][idx])
    return offsets, dev


def _run_device(eng, offsets, dev, S):
    Q = offsets.size - 1
    o_null, o_dla = L.DeviceArray(0, Q, np.float64), L.DeviceArray(0, Q, np.float64)
    o_s = L.DeviceArray(0, (Q, S), np.float64)
    o_n = L.DeviceArray(0, Q, np.int32)
    eng.process_device(offsets, dev["wavelengths"].ptr, dev["flux"].ptr, dev["noise_variance"].ptr,
                       dev["pixel_mask"].ptr, dev["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, S,
                       npix_ptr=o_n.ptr)
    eng.synchronize()
    return o_null, o_dla, o_s, o_n


@pytest.fixture(scope="module")
def dr12q_full():
    """configs[2]'s workload on one GPU: 162,861 DR12Q-shaped spectra (n = 270..1,250; a seeded pool
    of 4,096 distinct spectra tiled to the count, as bench.py's c3/c4 workloads) x 10^4 samples,
    outputs resident in HBM (13 GB).  Shared by the configs[2] and configs[3] tests."""
    t0 = time.time()
    Q, S, P = 162861, 10000, 4096
    model = syn.make_model(k=20)
    samples = syn.make_samples(S)
    pool = syn.make_dr12q_like_spectra(model, P, seed=12, mask_fraction=0.0)
    pp = syn.pack_spectra(pool)
    idx = np.arange(Q) % P
    offsets, dev = _dr12q_device_inputs(pp, idx)
    print(f"setup {time.time() - t0:.1f} s", flush=True)
    with Engine(model, samples, set_parameters(k=20)) as eng:
        t1 = time.time()
        o_null, o_dla, o_s, o_n = _run_device(eng, offsets, dev, S)
        print(f"engine {time.time() - t1:.1f} s", flush=True)
    del dev
    yield dict(Q=Q, S=S, P=P, model=model, samples=samples, pool=pool, pp=pp, idx=idx,
               o_null=o_null, o_dla=o_dla, o_s=o_s, o_n=o_n)
    for a in (o_null, o_dla, o_s, o_n):
        a.free()


def test_config2_full_dr12q_count_one_gpu(dr12q_full):
    """configs[2]: the full DR12Q count on one GPU.  The invariant on every spectrum, oracle spot
    checks on sampled spectra, and the tiled copies of a pool spectrum agree bitwise (position
    independence)."""
    t0 = time.time()
    F = dr12q_full
    Q, S, P, idx, pool = F["Q"], F["S"], F["P"], F["idx"], F["pool"]
    model, samples, o_s = F["model"], F["samples"], F["o_s"]
    lld, lln, npix = F["o_dla"].numpy(), F["o_null"].numpy(), F["o_n"].numpy()
    assert np.isfinite(lld).all() and np.isfinite(lln).all()
    assert npix.min() >= 250 and npix.max() <= 1300
    # the invariant on every spectrum, streamed back in row blocks
    worst = 0.0
    for r0 in range(0, Q, 8192):
        blk = o_s.numpy(rows=8192, start=r0)
        assert np.isfinite(blk).all()
        worst = max(worst, float(np.max(np.abs(_invariant(blk, lld[r0:r0 + blk.shape[0]]) - 1.0))))
    assert worst < 1e-12, worst
    # copies of one pool spectrum at different batch positions are bitwise equal
    for p in (0, 1234, 4095):
        rows = np.flatnonzero(idx == p)
        a = o_s.numpy(rows=1, start=int(rows[0]))
        b = o_s.numpy(rows=1, start=int(rows[-1]))
        np.testing.assert_array_equal(a, b)
        assert lld[rows[0]] == lld[rows[-1]] and lln[rows[0]] == lln[rows[-1]]
    # oracle spot checks on sampled spectra (and their pool entries)
    rng = np.random.default_rng(13)
    qs = rng.integers(0, Q, 16)
    pairs = [(int(q), int(s)) for q in qs for s in rng.integers(0, S, 3)]
    rows = {q: o_s.numpy(rows=1, start=q)[0] for q in set(q for q, _ in pairs)}
    spectra = {q: pool[q % P] for q in rows}
    got, ref, nref = _oracle_spot_checks(spectra, model, samples, lambda q, s: rows[q][s], list(rows), pairs)
    assert np.all(tol_ok(got, ref)) and _rel(got, ref) < 1e-9, _rel(got, ref)
    assert _rel(lln[list(rows)], nref) < 1e-9
    print(f"total {time.time() - t0:.1f} s", flush=True)


def test_config3_dr12q_8way_lpt_split_bitwise(dr12q_full):
    """configs[3]: the same full DR12Q count split 8 ways by bench.py's LPT shard (dr12q_shard with
    split=True, the c4 workload; process_qsos.m:88's serial spectrum loop sharded).  Each of the 8
    shards runs through its own Engine (in sequence on the one GPU, as 8 ranks would on 8 GPUs) and
    the reassembled outputs are bitwise equal to the unsharded configs[2] run on every spectrum and
    every sample; the invariant holds on every spectrum of every shard."""
    import bench
    F = dr12q_full
    Q, S, P, pp = F["Q"], F["S"], F["P"], F["pp"]
    world = 8
    pix = np.diff(pp["offsets"])
    full_dla, full_null, full_n = F["o_dla"].numpy(), F["o_null"].numpy(), F["o_n"].numpy()
    full_s = F["o_s"].numpy()          # 13 GB on the host (the box has ~270 GB)
    seen = np.zeros(Q, bool)
    loads = []
    for rank in range(world):
        mine = bench.dr12q_shard(pix, Q, rank, world, split=True)   # pool indices of this rank
        ids = bench.dr12q_shard_ids(pix, Q, rank, world)
        assert np.array_equal(ids % P, mine)
        assert not seen[ids].any()
        seen[ids] = True
        loads.append(int(pix[mine].sum()))
        t1 = time.time()
        offsets, dev = _dr12q_device_inputs(pp, mine)
        with Engine(F["model"], F["samples"], set_parameters(k=20)) as eng:
            o_null, o_dla, o_s, o_n = _run_device(eng, offsets, dev, S)
        del dev
        got_s = o_s.numpy()
        np.testing.assert_array_equal(got_s, full_s[ids])
        np.testing.assert_array_equal(o_dla.numpy(), full_dla[ids])
        np.testing.assert_array_equal(o_null.numpy(), full_null[ids])
        np.testing.assert_array_equal(o_n.numpy(), full_n[ids])
        inv = _invariant(got_s, o_dla.numpy())
        assert float(np.max(np.abs(inv - 1.0))) < 1e-12
        for a in (o_null, o_dla, o_s, o_n):
            a.free()
        del got_s
        print(f"rank {rank}: {ids.size} spectra, {loads[-1]} pixels, {time.time() - t1:.1f} s", flush=True)
    assert seen.all()
    # LPT balance: every shard's sweep work within 0.1% of the mean
    assert max(loads) / (sum(loads) / world) < 1.001, loads
