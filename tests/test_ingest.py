"""Spectrum ingest (read_spec.m, preload_qsos.m).  The numpy FITS reader is
checked against a file written by astropy (tests/golden/make_fits_fixture.py); read_spec and
preload_qsos against the rules of read_spec.m:27-38 and preload_qsos.m:25-72."""
import shutil
from pathlib import Path

import numpy as np
import pytest

from gp_dla_detection_amd import ingest as I
from gp_dla_detection_amd import matv73 as M
from gp_dla_detection_amd import parameters as P

GOLDEN = Path(__file__).parent / "golden"


def test_bintable_reader_matches_astropy_file():
    exp = np.load(GOLDEN / "speclite_fixture.npz")
    cols = I.read_bintable(str(GOLDEN / "speclite_fixture.fits"), 1)
    assert len(cols) == 8
    for got, key in zip(cols[:4], ("flux", "loglam", "ivar", "and_mask")):
        assert np.array_equal(got, exp[key]) and got.dtype == exp[key].dtype
    u16, flag, name, vec, k64 = I.read_bintable(str(GOLDEN / "speclite_fixture.fits"), 2)
    assert u16.tolist() == [0, 1000, 2000, 3000, 4000]                 # TZERO = 32768 convention
    assert flag.tolist() == [True, False, True, True, False]
    assert [s.decode().rstrip() for s in name] == ["abc", "de", "f", "ghijkl", ""]
    assert np.array_equal(vec, np.arange(15.0).reshape(5, 3))
    assert k64.tolist() == [1, -2, 3, 2 ** 40, -(2 ** 40)]


def test_read_spec_rules():
    exp = np.load(GOLDEN / "speclite_fixture.npz")
    w, f, nv, pm = I.read_spec(str(GOLDEN / "speclite_fixture.fits"))
    assert w.dtype == np.float32                                         # fitsread 'E' -> single
    assert np.array_equal(w, np.float32(10) ** exp["loglam"])           # :28
    with np.errstate(divide="ignore"):
        assert np.array_equal(nv, np.float32(1) / exp["ivar"])          # :31
    want = (exp["ivar"] == 0) | ((exp["and_mask"] & (1 << 23)) != 0)   # :36-38, BRIGHTSKY = bit 24
    assert np.array_equal(pm, want) and pm.any() and (~pm).any()


def _spectrum(z, n_lo=3400, n_hi=5600, step=1e-4, mask_window=False, seed=0):
    rng = np.random.default_rng(seed)
    loglam = np.arange(np.log10(n_lo), np.log10(n_hi), step).astype(np.float32)
    w = np.float32(10) ** loglam
    f = rng.normal(3, 0.2, w.size).astype(np.float32)
    nv = rng.uniform(0.01, 0.02, w.size).astype(np.float32)
    pm = rng.uniform(size=w.size) < 0.1
    if mask_window:
        rest = w / np.float32(1 + z)
        pm |= (rest >= 1310) & (rest <= 1325)
    return w, f, nv, pm


def test_preload_qsos_flags_normalisation_and_range():
    z = np.array([2.5, 2.5, 2.5, 3.2, 2.5])
    flags = np.array([0, 1, 0, 0, 0], dtype=np.uint8)
    specs = {0: _spectrum(2.5, seed=1), 2: _spectrum(2.5, mask_window=True, seed=2),
             3: _spectrum(3.2, n_lo=5000, seed=3), 4: _spectrum(2.5, seed=4)}
    out = I.preload_qsos(z, [0, 1, 2, 3, 4], [0] * 5, [0] * 5, flags, lambda p, m, f: specs[p])
    ff = out["filter_flags"]
    assert ff[1] == 1                                                   # already filtered: skipped
    assert ff[2] == 4                                                   # bit 3: no normalising pixel
    assert ff[3] == 8                                                   # bit 4: < min_num_pixels
    assert ff[0] == 0 and ff[4] == 0
    for q in (0, 4):
        w, f, nv, pm = specs[q]
        rest = w / np.float32(1 + z[q])
        win = (rest >= P.NORMALIZATION_MIN_LAMBDA) & (rest <= P.NORMALIZATION_MAX_LAMBDA) & ~pm
        med = np.median(f[win])
        assert out["all_normalizers"][q] == med
        ind = (rest >= P.LOADING_MIN_LAMBDA) & (rest <= P.LOADING_MAX_LAMBDA)
        first, last = np.flatnonzero(ind)[[0, -1]]
        avail = np.flatnonzero(~ind & ~pm)
        keep = ind.copy()
        if (avail > last).any():
            keep[avail[avail > last].min()] = True
        if (avail < first).any():                       # MATLAB: ind(max([])) = true is a no-op
            keep[avail[avail < first].max()] = True
        assert np.array_equal(out["all_wavelengths"][q], w[keep].astype(np.float64))
        assert np.array_equal(out["all_flux"][q], (f / med)[keep].astype(np.float64))
        assert np.array_equal(out["all_noise_variance"][q], (nv / (med * med))[keep].astype(np.float64))
        assert np.array_equal(out["all_pixel_mask"][q], pm[keep])
    assert out["all_wavelengths"][2].size == 0 and out["all_normalizers"][2] == 0


def test_run_preload_qsos_tree(tmp_path):
    spectra = tmp_path / "dr12q" / "spectra"
    for plate, mjd, fiber in ((4000, 55000, 12), (4001, 55001, 7)):
        d = spectra / str(plate)
        d.mkdir(parents=True)
        shutil.copy(GOLDEN / "speclite_fixture.fits", d / f"spec-{plate}-{mjd}-{fiber:04d}.fits")
    proc = tmp_path / "dr12q" / "processed"
    proc.mkdir(parents=True)
    M.savemat73(str(proc / "catalog.mat"), dict(z_qsos=np.array([2.03, 2.5]), plates=np.array([4000, 4001.0]),
                                                mjds=np.array([55000, 55001.0]), fiber_ids=np.array([12, 7.0]),
                                                filter_flags=np.array([0, 2], dtype=np.uint8)))
    out = I.run_preload_qsos(str(tmp_path), "dr12q")
    assert out["filter_flags"].tolist() == [8, 2]        # too few in-range pixels in the fixture; pre-filtered
    cat = M.loadmat73(str(proc / "catalog.mat"))
    assert cat["filter_flags"].ravel().tolist() == [8, 2]
    pre = M.loadmat73(str(proc / "preloaded_qsos.mat"))
    assert pre["all_flux"].shape == (2, 1) and float(pre["min_num_pixels"][0, 0]) == 200


def _spectra_tree(tmp_path):
    spectra = tmp_path / "dr12q" / "spectra"
    for plate, mjd, fiber in ((4000, 55000, 12), (4001, 55001, 7)):
        d = spectra / str(plate)
        d.mkdir(parents=True)
        shutil.copy(GOLDEN / "speclite_fixture.fits", d / f"spec-{plate}-{mjd}-{fiber:04d}.fits")
    proc = tmp_path / "dr12q" / "processed"
    proc.mkdir(parents=True)
    return proc


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


def test_own_fits_writer_roundtrip(tmp_path):
    """The test-side writer (tests/fits_writer.py) produces files the reader reads back exactly."""
    from fits_writer import write_speclite
    rng = np.random.default_rng(5)
    n = 300
    f, ll = rng.normal(3, 1, n).astype(np.float32), (3.55 + 1e-4 * np.arange(n)).astype(np.float32)
    iv, am = rng.uniform(0, 2, n).astype(np.float32), rng.integers(0, 2 ** 30, n).astype(np.int32)
    write_speclite(str(tmp_path / "s.fits"), f, ll, iv, am)
    got = I.read_bintable(str(tmp_path / "s.fits"), 1)
    for a, b in zip(got, (f, ll, iv, am)):
        assert np.array_equal(a, b)


H5PY_PY = "/opt/conda/bin/python3.9"


def _has_astropy():
    import os
    import subprocess
    if not os.path.exists(H5PY_PY):
        return False
    return subprocess.run([H5PY_PY, "-c", "import astropy.io.fits"], capture_output=True).returncode == 0


@pytest.mark.skipif(not _has_astropy(), reason="no interpreter with astropy (GPU box)")
def test_preload_matches_the_oracle_restatement(tmp_path):
    """Product read_spec + preload_qsos against oracle/ingest_oracle.py, the line-by-line
    restatement of read_spec.m and preload_qsos.m that reads the FITS files with astropy (run with
    the interpreter that has it).  Cases: plain spectra (odd and even counts in the normalisation
    window), a pre-filtered entry, a masked normalisation window (bit 3), too few pixels (bit 4),
    NaN fluxes in the window, BRIGHTSKY-masked pixels, loading-range edges with and without an
    unmasked neighbour.  Every saved variable must agree bit for bit (cells widened to double)."""
    import subprocess
    from fits_writer import write_speclite
    rng = np.random.default_rng(17)
    spectra = tmp_path / "spectra"
    cases = [  # (z, lo, hi, prefilter, mask window, nan in window, first-pixel masked)
        (2.5, 3400, 5600, 0, False, False, False), (2.7, 3560, 5900, 0, False, True, False),
        (3.1, 3600, 6200, 0, False, False, True), (2.4, 3300, 5200, 1, False, False, False),
        (2.6, 3500, 5700, 0, True, False, False), (3.3, 5100, 6000, 0, False, False, False),
        (2.2, 2860, 4300, 0, False, False, False), (2.9, 3700, 6100, 0, False, True, True)]
    z, plates, mjds, fibers, flags = [], [], [], [], []
    for q, (zq, lo, hi, pre, mwin, nanw, mfirst) in enumerate(cases):
        ll = np.arange(np.log10(lo), np.log10(hi), 1e-4).astype(np.float32)
        w = np.float32(10) ** ll
        rest = w / np.float32(1 + zq)
        f = rng.normal(3.0, 0.4, ll.size).astype(np.float32)
        iv = rng.uniform(20, 80, ll.size).astype(np.float32)
        iv[rng.uniform(size=ll.size) < 0.05] = 0
        am = np.where(rng.uniform(size=ll.size) < 0.05, 1 << 23, 0).astype(np.int32)   # BRIGHTSKY
        am |= np.where(rng.uniform(size=ll.size) < 0.1, 1 << 5, 0).astype(np.int32)    # an ignored bit
        win = (rest >= 1310) & (rest <= 1325)
        if mwin:
            iv[win] = 0
        if nanw:
            f[np.flatnonzero(win)[::7]] = np.nan
        if mfirst:   # the pixel just below the loading range is masked: the next unmasked one is taken
            below = np.flatnonzero(rest < 910)
            if below.size:
                iv[below[-1]] = 0
        p, m, fi = 5000 + q, 56000 + q, 10 + q
        d = spectra / str(p)
        d.mkdir(parents=True, exist_ok=True)
        write_speclite(str(d / f"spec-{p}-{m}-{fi:04d}.fits"), f, ll, iv, am)
        z.append(zq); plates.append(p); mjds.append(m); fibers.append(fi); flags.append(pre)
    got = I.preload_qsos(z, plates, mjds, fibers, np.array(flags, np.uint8),
                         lambda p, m, f: I.read_spec(I.spec_filename(str(spectra), p, m, f)))
    job = tmp_path / "job.npz"
    np.savez(job, z_qsos=np.array(z), plates=np.array(plates), mjds=np.array(mjds), fiber_ids=np.array(fibers),
             filter_flags=np.array(flags, np.uint8), spectra_dir=str(spectra))
    oracle = Path(__file__).resolve().parents[1] / "oracle" / "ingest_oracle.py"
    res = subprocess.run([H5PY_PY, "-B", str(oracle), str(job), str(tmp_path / "out.npz")], capture_output=True,
                         text=True)
    assert res.returncode == 0, res.stderr[-2000:]
    want = np.load(tmp_path / "out.npz")
    assert got["filter_flags"].tolist() == want["filter_flags"].tolist()
    assert sorted(set(got["filter_flags"].tolist())) == [0, 1, 4, 8]          # every branch exercised
    np.testing.assert_array_equal(got["all_normalizers"], want["all_normalizers"])
    for key in ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask"):
        for q in range(len(cases)):
            name = f"{key}__{q}"
            if name in want.files:
                np.testing.assert_array_equal(got[key][q], want[name].astype(got[key][q].dtype), err_msg=name)
            else:
                assert got[key][q].size == 0, name


def test_nanmedian_is_matlabs():
    """median.m's meanof for an even count (a + (b - a) / 2 for finite same-sign a, b), NaNs dropped,
    in single: cases where numpy's (a + b) / 2 rounds differently."""
    f = np.float32
    a, b = f(1.0000001), f(3.9999998)
    v = np.array([b, np.nan, a], dtype=np.float32)
    assert I.nanmedian(v) == a + (b - a) / f(2)
    rng = np.random.default_rng(3)
    seen = 0
    for _ in range(2000):
        x = (rng.lognormal(0, 3, 2 * rng.integers(1, 8)) * rng.choice([-1, 1])).astype(np.float32)
        s = np.sort(x)
        lo, hi = s[x.size // 2 - 1], s[x.size // 2]
        want = lo + (hi - lo) / f(2) if np.sign(lo) == np.sign(hi) else (lo + hi) / f(2)
        assert I.nanmedian(x) == want and I.nanmedian(x).dtype == np.float32
        seen += want != np.median(x)
    assert seen > 0                                   # numpy's median differs on some of these
    assert np.isnan(I.nanmedian(np.array([np.nan], np.float32)))
