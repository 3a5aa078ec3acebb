"""GPU parity of spectrum ingest (read_spec.m:27-38 and preload_qsos.m:18-67 on the device,
csrc/ingest.hip) against oracle/ingest_oracle.py's columns restatement (pinned on the
CPU to the same oracle reading the files with astropy, tests/test_ingest.py):

* read_spec's derived columns bit for bit on the committed speclite fixture and exhaustively over every
  float32 loglam of the SDSS range;
* preload_qsos on the eight branch cases (FITS files through the host reader) and on a DR12Q-count
  batch (162,861 catalogue entries, full 3600-10400 A BOSS coadds): filter flags, medians,
  normalisers, cell lengths and every cell value bit for bit;
* the script on files (catalog.mat in, preloaded_qsos.mat out, filter_flags appended)."""
import shutil
import time
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import ingest as I  # noqa: E402
from gp_dla_detection_amd import matv73 as M  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from oracle import ingest_oracle as O  # noqa: E402
from test_ingest import check_preload_rules, preload_cases, write_oracle_cases  # noqa: E402

GOLDEN = Path(__file__).parent / "golden"
KEYS = ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask")


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _same(got, want):
    return np.array_equal(np.asarray(got).view(np.uint8), np.asarray(want).view(np.uint8))


def _assert_equal_results(got, want, idx=None):
    idx = range(len(got["filter_flags"])) if idx is None else idx
    assert np.array_equal(got["filter_flags"], want["filter_flags"])
    assert np.array_equal(got["all_normalizers"], want["all_normalizers"])
    for q in idx:
        for k in KEYS:
            w = want[k][q]
            if w is None:
                assert got[k][q].size == 0, (k, q)
            else:
                assert got[k][q].dtype == w.dtype and _same(got[k][q], w), (k, q)


def test_read_spec_fixture_bit_exact():
    exp = np.load(GOLDEN / "speclite_fixture.npz")
    w, f, nv, pm = I.read_spec(str(GOLDEN / "speclite_fixture.fits"))
    ow, of, onv, opm = O.derive(exp["flux"], exp["loglam"], exp["ivar"], exp["and_mask"])
    assert w.dtype == np.float32 and nv.dtype == np.float32
    assert _same(w, ow) and _same(f, of) and _same(nv, onv) and np.array_equal(pm, opm)
    assert pm.any() and (~pm).any()


def test_read_spec_every_loglam_of_the_sdss_range():
    """The device's 10.^loglam in single is the correctly rounded value for every one of the 5.2M float32
    loglam in [3.0, 4.5] (1,000-31,623 A, around SDSS's 3,600-10,400 A); 1 ./ ivar and the mask rule on
    random columns alongside."""
    lo, hi = np.float32(3.0).view(np.uint32), np.float32(4.5).view(np.uint32)
    ll = np.arange(lo, hi + 1, dtype=np.uint32).view(np.float32)
    rng = np.random.default_rng(2)
    iv = rng.uniform(0, 100, ll.size).astype(np.float32)
    iv[rng.uniform(size=ll.size) < 0.03] = 0
    am = rng.integers(0, 2 ** 31 - 1, ll.size).astype(np.int32)
    n = ll.size
    import ctypes as C
    w, nv, pm = np.empty(n, np.float32), np.empty(n, np.float32), np.empty(n, np.uint8)
    L.check(L.load().gpdla_read_spec_f32(0, n, L.ptr(ll, C.c_float), L.ptr(iv, C.c_float), L.ptr(am, C.c_int32),
                                         L.ptr(w, C.c_float), L.ptr(nv, C.c_float), L.ptr(pm, C.c_uint8)))
    ow, _, onv, opm = O.derive(np.zeros(n, np.float32), ll, iv, am)
    mism = np.flatnonzero(w.view(np.uint32) != ow.view(np.uint32))
    assert mism.size == 0, (mism.size, ll[mism[:5]])
    assert _same(nv, onv) and np.array_equal(pm.astype(bool), opm)


def test_preload_rules_on_the_device():
    z, flags, cols = preload_cases()
    got = I.preload_batch(z, flags, cols)
    check_preload_rules(got, z, cols)
    _assert_equal_results(got, O.preload_from_columns(z, flags, cols))


def test_preload_matches_the_oracle_on_every_branch(tmp_path):
    (z, plates, mjds, fibers, flags), spectra = write_oracle_cases(tmp_path)
    loader = lambda p, m, f: I.read_spec_columns(I.spec_filename(str(spectra), p, m, f))   # noqa: E731
    got = I.preload_qsos(z, plates, mjds, fibers, flags, loader, batch=3)    # batches that split the catalogue
    want = O.preload_from_columns(z, flags, [None if flags[i] else loader(plates[i], mjds[i], fibers[i])
                                             for i in range(z.size)])
    assert sorted(set(got["filter_flags"].tolist())) == [0, 1, 4, 8]
    _assert_equal_results(got, want)


def _neighbour_cases():
    """Spectra whose loading-range neighbours sit far from the range (masked runs of 1, 255, 256, 257 and
    700 pixels on either side; a run ending at the normalisation window, which stays unmasked), none
    below (everything before masked, or the range starting at pixel 0), plus a spectrum with its pixels
    permuted (the loading range is a scattered mask, not a slice)."""
    rng = np.random.default_rng(77)
    z, cols = [], []
    for zq, run_after, run_before in ((3.0, 1, 1), (3.6, 255, 256), (3.6, 256, 257), (3.6, 700, 300),
                                      (3.0, 10 ** 6, 10 ** 6), (2.9, 0, 0)):
        f, ll, iv, am = syn.make_boss_coadd_columns(rng, zq)
        iv[(np.arange(iv.size) % 97) == 5] = 0                # scattered masked pixels everywhere
        am[:] = 0
        f[np.isnan(f)] = 1.0
        w, _, _, _ = O.derive(f, ll, iv, am)
        rest = w / np.float32(1 + zq)
        ind = np.flatnonzero((rest >= 910) & (rest <= 1217))
        iv[ind[-1] + 1:ind[-1] + 1 + run_after] = 0
        iv[max(ind[0] - run_before, 0):ind[0]] = 0
        iv[(rest >= 1310) & (rest <= 1325)] = 1.0             # keep the normalisation window usable
        z.append(zq)
        cols.append((f, ll, iv, am))
    f, ll, iv, am = syn.make_boss_coadd_columns(rng, 2.6)
    perm = rng.permutation(f.size)
    z.append(2.6)
    cols.append(tuple(c[perm] for c in (f, ll, iv, am)))
    return np.array(z), np.zeros(len(z), np.uint8), cols


def test_preload_neighbour_search_and_scattered_ranges():
    z, flags, cols = _neighbour_cases()
    got = I.preload_batch(z, flags, cols)
    want = O.preload_from_columns(z, flags, cols)
    assert (want["filter_flags"] == 0).all()
    _assert_equal_results(got, want)


ENDS = (1310.0, 1325.0, 911.75, 1215.75, 910.0, 1217.0)     # set_parameters.m:21-22, 29-30, 33-34


def _boundary_spectrum(z, nrange_target=None):
    """A BOSS grid plus every float32 loglam within 81 ulps of the six range ends at this z, fluxes all
    distinct (any change of the window's membership moves the median).  With nrange_target, all but
    that many pixels of [911.75, 1215.75] are masked -- the ones near its ends kept -- so one pixel
    counted on the wrong side flips the min_num_pixels filter (target 200 passes, 199 fails)."""
    grid = (np.log10(3600.0) + 1e-4 * np.arange(4607)).astype(np.float32)
    near = [(np.float32(np.log10(e * (1 + z))).view(np.uint32) + np.arange(-81, 82, dtype=np.int64)).astype(np.uint32)
            .view(np.float32) for e in ENDS]
    ll = np.unique(np.concatenate([grid] + near))
    f = np.arange(ll.size, dtype=np.float32) + 1
    iv = np.ones(ll.size, np.float32)
    am = np.zeros(ll.size, np.int32)
    if nrange_target is not None:
        w = O.derive(f, ll, iv, am)[0]
        rest = w / np.float32(1 + z)
        inside = np.flatnonzero((rest >= ENDS[2]) & (rest <= ENDS[3]))
        edge = np.flatnonzero(np.isin(ll, np.concatenate(near)))
        keep = np.concatenate([np.intersect1d(inside, edge), np.setdiff1d(inside, edge)])[:nrange_target]
        iv[np.setdiff1d(inside, keep)] = 0
    return f, ll, iv, am


def test_preload_range_ends_ulp_by_ulp():
    """The kernels' fast range estimate hands every pixel near a range end to the correctly rounded
    path: at 64 redshifts over [2, 6.5], every float32 loglam within 81 ulps (~4.5e-5 relative) of each
    of the six ends lands where the oracle puts it -- window membership through the median, the model
    range through the 200-pixel filter at its threshold, the loading range through the cells."""
    zs = np.linspace(2.0, 6.5, 64)
    z, cols = [], []
    for zq in zs:
        for t in (None, 200, 199):
            z.append(zq)
            cols.append(_boundary_spectrum(zq, t))
    z = np.array(z)
    flags = np.zeros(z.size, np.uint8)
    got = I.preload_batch(z, flags, cols)
    want = O.preload_from_columns(z, flags, cols)
    ff = want["filter_flags"]
    assert (ff[1::3] == 0).all() and (ff[2::3] == 8).all()      # the threshold cases sit on the threshold
    _assert_equal_results(got, want)
    assert np.array_equal(got["medians"], want["medians"], equal_nan=True)


def _fine_spectra(rng, z, dex, ties=False):
    """A finely sampled spectrum whose normalisation window holds more values than the scan sorts in LDS
    (2,048): the median then comes from the radix select.  Returned twice: as drawn, and with one more
    window pixel masked (odd and even set sizes), with the set sizes."""
    ll = np.arange(np.log10(3400.0), np.log10(6000.0), dex).astype(np.float32)
    f = rng.normal(1.0, 2.0, ll.size).astype(np.float32)
    if ties:
        f = np.round(f * 4) / 4                                   # many equal values, both signs
    iv = rng.uniform(1, 50, ll.size).astype(np.float32)
    iv[rng.uniform(size=ll.size) < 0.05] = 0
    am = np.where(rng.uniform(size=ll.size) < 0.03, 1 << 23, 0).astype(np.int32)
    f[rng.uniform(size=ll.size) < 0.02] = np.nan
    f[rng.integers(0, ll.size, 3)] = np.inf
    f[rng.integers(0, ll.size, 2)] = -np.inf
    w = O.derive(f, ll, iv, am)[0]
    rest = w / np.float32(1 + z)
    win = np.flatnonzero((rest >= 1310) & (rest <= 1325) & (iv > 0) & (am == 0) & ~np.isnan(f))
    iv2 = iv.copy()
    iv2[win[win.size // 2]] = 0
    return [(f, ll, iv, am), (f, ll, iv2, am)], [win.size, win.size - 1]


def test_preload_median_of_a_window_beyond_lds():
    rng = np.random.default_rng(12)
    z, cols, sizes = [], [], []
    for zq, dex, ties in ((2.5, 1e-6, False), (3.1, 7e-7, True), (2.5, 1e-4, False)):
        c, n = _fine_spectra(rng, zq, dex, ties)
        z += [zq, zq]
        cols += c
        sizes += n
    assert min(sizes[:4]) > 4096 and max(sizes[4:]) < 64       # radix select twice over; the register sort
    z = np.array(z)
    flags = np.zeros(z.size, np.uint8)
    got = I.preload_batch(z, flags, cols)
    want = O.preload_from_columns(z, flags, cols)
    assert (want["filter_flags"] == 0).all()
    assert np.array_equal(got["medians"], want["medians"])
    _assert_equal_results(got, want)


def test_preload_dr12q_count_batch():
    """162,861 catalogue entries (DR12Q's count, README.md:115): a pool of 4,096 distinct full coadds at
    z in [2.15, 5.5] tiled to the count, 2% pre-filtered; the device result of every entry must equal the
    oracle's for its pool spectrum bit for bit."""
    Qt, npool = 162861, 4096
    rng = np.random.default_rng(31)
    zp = rng.uniform(2.15, 5.5, npool)
    pool = [syn.make_boss_coadd_columns(rng, z) for z in zp]
    pre = (rng.uniform(size=npool) < 0.02).astype(np.uint8)
    want = O.preload_from_columns(zp, pre, [None if pre[i] else pool[i] for i in range(npool)])
    sel = np.arange(Qt) % npool
    z = zp[sel]
    flags = pre[sel]
    t0 = time.perf_counter()
    got = I.preload_qsos(z, sel, sel, sel, flags, lambda p, m, f: pool[int(p)], batch=16384)
    el = time.perf_counter() - t0
    assert sorted(set(got["filter_flags"].tolist())) == [0, 1, 4, 8]
    assert np.array_equal(got["filter_flags"], want["filter_flags"][sel])
    assert np.array_equal(got["all_normalizers"], want["all_normalizers"][sel])
    bad = 0
    for q in range(Qt):
        p = sel[q]
        for k in KEYS:
            w = want[k][p]
            g = got[k][q]
            if (g.size != 0 if w is None else not (g.dtype == w.dtype and _same(g, w))):
                bad += 1
    assert bad == 0
    n_pix = sum(pool[p][0].size for p in sel if not pre[p])
    print(f"preload_qsos on the device: {Qt} entries, {n_pix / 1e6:.0f} M pixels in {el:.1f} s (host loader, "
          f"packing and copies included)")


def _spectra_tree(tmp_path):
    spectra = tmp_path / "dr12q" / "spectra"
    for plate, mjd, fiber in ((4000, 55000, 12), (4001, 55001, 7)):
        d = spectra / str(plate)
        d.mkdir(parents=True)
        shutil.copy(GOLDEN / "speclite_fixture.fits", d / f"spec-{plate}-{mjd}-{fiber:04d}.fits")
    proc = tmp_path / "dr12q" / "processed"
    proc.mkdir(parents=True)
    return proc


def test_run_preload_qsos_tree(tmp_path):
    proc = _spectra_tree(tmp_path)
    M.savemat73(str(proc / "catalog.mat"), dict(z_qsos=np.array([2.03, 2.5]), plates=np.array([4000, 4001.0]),
                                                mjds=np.array([55000, 55001.0]), fiber_ids=np.array([12, 7.0]),
                                                filter_flags=np.array([0, 2], dtype=np.uint8)))
    out = I.run_preload_qsos(str(tmp_path), "dr12q")
    assert out["filter_flags"].tolist() == [8, 2]        # too few in-range pixels in the fixture; pre-filtered
    cat = M.loadmat73(str(proc / "catalog.mat"))
    assert cat["filter_flags"].ravel().tolist() == [8, 2]
    pre = M.loadmat73(str(proc / "preloaded_qsos.mat"))
    assert pre["all_flux"].shape == (2, 1) and float(pre["min_num_pixels"][0, 0]) == 200


def test_run_preload_qsos_appends_in_place(tmp_path):
    """preload_qsos.m:82-83 save(..., 'filter_flags', '-append'): a MATLAB catalog.mat with
    containers.Map objects (libhdf5-written fixture) keeps every byte except filter_flags' data."""
    proc = _spectra_tree(tmp_path)
    shutil.copy(GOLDEN / "catalog_mcos.mat", proc / "catalog.mat")
    before = (proc / "catalog.mat").read_bytes()
    assert M.rewrite_blockers(str(proc / "catalog.mat"))          # the Maps cannot round-trip
    out = I.run_preload_qsos(str(tmp_path), "dr12q")
    assert out["filter_flags"].tolist() == [8, 2] and out["filter_flags_path"].endswith("catalog.mat")
    after = (proc / "catalog.mat").read_bytes()
    diff = [i for i in range(len(before)) if before[i] != after[i]]
    assert len(before) == len(after) and len(diff) == 1           # the one flag byte that changed
    cat = M.loadmat73(str(proc / "catalog.mat"))
    assert cat["filter_flags"].ravel().tolist() == [8, 2] and cat["filter_flags"].dtype == np.uint8


def test_run_preload_qsos_never_rewrites_objects(tmp_path, monkeypatch):
    """When filter_flags cannot be overwritten in place and the file holds MATLAB objects, the
    catalog is left untouched and the flags go to a sidecar file."""
    proc = _spectra_tree(tmp_path)
    shutil.copy(GOLDEN / "catalog_mcos.mat", proc / "catalog.mat")
    before = (proc / "catalog.mat").read_bytes()
    monkeypatch.setattr(M, "update_variable", lambda *a, **k: False)
    with pytest.warns(UserWarning, match="not rewritten"):
        out = I.run_preload_qsos(str(tmp_path), "dr12q")
    assert (proc / "catalog.mat").read_bytes() == before
    side = M.loadmat73(out["filter_flags_path"])
    assert side["filter_flags"].ravel().tolist() == [8, 2]


def test_errors_are_loud():
    import ctypes as C
    off = np.array([0, 3, 2], np.int64)                      # decreasing offsets
    z = np.zeros(2)
    fl = np.zeros(3, np.uint8)
    p = I.preload_params()
    rc = L.load().gpdla_preload_qsos_f32(0, 2, L.ptr(off, C.c_int64), None, None, None, None, L.ptr(z), C.byref(p),
                                         L.ptr(fl, C.c_uint8), L.ptr(np.zeros(3, np.int64), C.c_int64), None, None,
                                         None, None, L.ptr(np.zeros(2)), None)
    assert rc == L.GPDLA_EINVAL


def test_last_call_kernel_times():
    """gpdla_last_call_kernel_ms reports one HIP-event time per launch of this thread's last call."""
    z, flags, cols = preload_cases()
    I.preload_batch(z, flags, cols)
    ms = L.last_call_kernel_ms()
    assert len(ms) == 3 and all(0 < t < 1000 for t in ms)          # keys, scan, write
    w, f, nv, pm = I.read_spec(str(GOLDEN / "speclite_fixture.fits"))
    assert len(L.last_call_kernel_ms()) == 1
