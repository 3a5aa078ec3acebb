"""Spectrum ingest (read_spec.m, preload_qsos.m) on the CPU: the host FITS reader
against a file written by astropy (tests/golden/make_fits_fixture.py), the test-side FITS writer, and
the checker the device kernels are judged by (oracle/ingest_oracle.py) pinned to the .m files' rules:
read_spec.m:27-38, preload_qsos.m:18-67, MATLAB's median, and its columns path against its astropy path.
The product's numeric stage runs on the GPU only (tests/test_gpu_ingest.py)."""
import shutil
from pathlib import Path

import numpy as np
import pytest

from gp_dla_detection_amd import ingest as I
from gp_dla_detection_amd import parameters as P
from oracle import ingest_oracle as O

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


def test_oracle_read_spec_rules():
    exp = np.load(GOLDEN / "speclite_fixture.npz")
    w, f, nv, pm = O.derive(exp["flux"], exp["loglam"], exp["ivar"], exp["and_mask"])
    assert w.dtype == np.float32                                         # fitsread 'E' -> single
    assert np.array_equal(w, (10.0 ** exp["loglam"].astype(np.float64)).astype(np.float32))   # :28
    with np.errstate(divide="ignore"):
        assert np.array_equal(nv, np.float32(1) / exp["ivar"])          # :31
    want = (exp["ivar"] == 0) | ((exp["and_mask"] & (1 << 23)) != 0)   # :36-38, BRIGHTSKY = bit 24
    assert np.array_equal(pm, want) and pm.any() and (~pm).any()


def test_single_power_is_correctly_rounded_over_the_sdss_range():
    """read_spec.m:28's 10.^loglam in single: the double power rounded once equals the extended-precision
    value rounded once for EVERY float32 loglam in [3.0, 4.5] (5.2M values: 1000-31623 A), i.e. it is the
    correctly rounded single there -- the definition the device kernel implements.  numpy's float32
    power (C powf) is not: it differs on ~20% of them."""
    lo, hi = np.float32(3.0).view(np.uint32), np.float32(4.5).view(np.uint32)
    x = np.arange(lo, hi + 1, dtype=np.uint32).view(np.float32)
    d = (10.0 ** x.astype(np.float64)).astype(np.float32)
    ld = (np.longdouble(10) ** x.astype(np.longdouble)).astype(np.float32)
    if np.finfo(np.longdouble).nmant < 63:
        pytest.skip("no x87 extended long double here")
    assert np.array_equal(d, ld)


def _spectrum(z, n_lo=3400, n_hi=5600, step=1e-4, mask_window=False, seed=0):
    """fitsread columns (flux, loglam, ivar, and_mask) of a synthetic coadd."""
    rng = np.random.default_rng(seed)
    loglam = np.arange(np.log10(n_lo), np.log10(n_hi), step).astype(np.float32)
    f = rng.normal(3, 0.2, loglam.size).astype(np.float32)
    iv = rng.uniform(50, 100, loglam.size).astype(np.float32)
    iv[rng.uniform(size=loglam.size) < 0.05] = 0
    am = np.where(rng.uniform(size=loglam.size) < 0.05, 1 << 23, 0).astype(np.int32)
    if mask_window:
        rest = (10.0 ** loglam.astype(np.float64)).astype(np.float32) / np.float32(1 + z)
        iv[(rest >= 1310) & (rest <= 1325)] = 0
    return f, loglam, iv, am


CASES_Z = np.array([2.5, 2.5, 2.5, 3.2, 2.5])
CASES_FLAGS = np.array([0, 1, 0, 0, 0], dtype=np.uint8)


def preload_cases():
    """Five catalogue entries: plain, pre-filtered, masked normalisation window, too few pixels, plain."""
    specs = {0: _spectrum(2.5, seed=1), 2: _spectrum(2.5, mask_window=True, seed=2),
             3: _spectrum(3.2, n_lo=5000, seed=3), 4: _spectrum(2.5, seed=4)}
    return CASES_Z, CASES_FLAGS, [specs.get(q) for q in range(5)]


def check_preload_rules(out, z, cols):
    """preload_qsos.m's rules, restated inline, on a result dict (the oracle's or the device's)."""
    ff = out["filter_flags"]
    assert ff[1] == 1                                                   # already filtered: skipped
    assert ff[2] == 4                                                   # bit 3: no normalising pixel
    assert ff[3] == 8                                                   # bit 4: < min_num_pixels
    assert ff[0] == 0 and ff[4] == 0
    for q in (0, 4):
        w, f, nv, pm = O.derive(*cols[q])
        rest = w / np.float32(1 + z[q])
        win = (rest >= P.NORMALIZATION_MIN_LAMBDA) & (rest <= P.NORMALIZATION_MAX_LAMBDA) & ~pm
        med = O.matlab_median(f[win])
        assert out["all_normalizers"][q] == med
        ind = (rest >= P.LOADING_MIN_LAMBDA) & (rest <= P.LOADING_MAX_LAMBDA)
        first, last = np.flatnonzero(ind)[[0, -1]]
        avail = np.flatnonzero(~ind & ~pm)
        keep = ind.copy()
        if (avail > last).any():
            keep[avail[avail > last].min()] = True
        if (avail < first).any():                       # MATLAB: ind(max([])) = true is a no-op
            keep[avail[avail < first].max()] = True
        assert np.array_equal(out["all_wavelengths"][q], w[keep])
        assert np.array_equal(out["all_flux"][q], (f / med)[keep])
        assert np.array_equal(out["all_noise_variance"][q], (nv / (med * med))[keep])
        assert np.array_equal(out["all_pixel_mask"][q], pm[keep])
    assert out["all_wavelengths"][2] is None or out["all_wavelengths"][2].size == 0
    assert out["all_normalizers"][2] == 0


def test_oracle_preload_rules():
    z, flags, cols = preload_cases()
    check_preload_rules(O.preload_from_columns(z, flags, cols), z, cols)


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


def write_oracle_cases(tmp_path):
    """Eight catalogue entries written as speclite files that take every branch of preload_qsos.m:
    plain spectra (odd and even counts in the normalisation window), a pre-filtered entry, a masked
    normalisation window (bit 3), too few pixels (bit 4), NaN fluxes in the window, BRIGHTSKY-masked
    pixels, loading-range edges with and without an unmasked neighbour.  Returns the catalogue columns
    and the spectra directory."""
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
        rest = (10.0 ** ll.astype(np.float64)).astype(np.float32) / np.float32(1 + zq)
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
    return (np.array(z), np.array(plates), np.array(mjds), np.array(fibers), np.array(flags, np.uint8)), spectra


@pytest.mark.skipif(not _has_astropy(), reason="no interpreter with astropy (GPU box)")
def test_oracle_columns_path_equals_its_astropy_path(tmp_path):
    """The oracle's columns restatement (what the GPU tests run on the box, fed by the host FITS reader)
    against the same oracle reading the files with astropy under python3.9: every saved variable bit
    for bit on the eight branch cases."""
    import subprocess
    (z, plates, mjds, fibers, flags), spectra = write_oracle_cases(tmp_path)
    cols = [None if flags[i] > 0 else I.read_spec_columns(I.spec_filename(str(spectra), plates[i], mjds[i], fibers[i]))
            for i in range(z.size)]
    got = O.preload_from_columns(z, flags, cols)
    job = tmp_path / "job.npz"
    np.savez(job, z_qsos=z, plates=plates, mjds=mjds, fiber_ids=fibers, filter_flags=flags, spectra_dir=str(spectra))
    oracle = Path(__file__).resolve().parents[1] / "oracle" / "ingest_oracle.py"
    res = subprocess.run([H5PY_PY, "-B", str(oracle), str(job), str(tmp_path / "out.npz")], capture_output=True,
                         text=True)
    assert res.returncode == 0, res.stderr[-2000:]
    want = np.load(tmp_path / "out.npz")
    assert got["filter_flags"].tolist() == want["filter_flags"].tolist()
    assert sorted(set(got["filter_flags"].tolist())) == [0, 1, 4, 8]          # every branch exercised
    np.testing.assert_array_equal(got["all_normalizers"], want["all_normalizers"])
    for key in ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask"):
        for q in range(z.size):
            name = f"{key}__{q}"
            if name in want.files:
                np.testing.assert_array_equal(got[key][q], want[name], err_msg=name)
            else:
                assert got[key][q] is None, name


def test_nanmedian_is_matlabs():
    """The oracle's median.m: meanof for an even count (a + (b - a) / 2 for finite same-sign a, b), NaNs
    dropped by the caller, in single: cases where numpy's (a + b) / 2 rounds differently."""
    def nanmedian(v):
        return O.matlab_median(v[~np.isnan(v)])
    f = np.float32
    a, b = f(1.0000001), f(3.9999998)
    v = np.array([b, np.nan, a], dtype=np.float32)
    assert nanmedian(v) == a + (b - a) / f(2)
    rng = np.random.default_rng(3)
    seen = 0
    for _ in range(2000):
        x = (rng.lognormal(0, 3, 2 * rng.integers(1, 8)) * rng.choice([-1, 1])).astype(np.float32)
        s = np.sort(x)
        lo, hi = s[x.size // 2 - 1], s[x.size // 2]
        want = lo + (hi - lo) / f(2) if np.sign(lo) == np.sign(hi) else (lo + hi) / f(2)
        assert nanmedian(x) == want and nanmedian(x).dtype == np.float32
        seen += want != np.median(x)
    assert seen > 0                                   # numpy's median differs on some of these
    assert np.isnan(nanmedian(np.array([np.nan], np.float32)))


def test_product_has_no_cpu_path():
    """read_spec's rules and preload_qsos's numeric stage run on the device only: without one they fail
    loudly (no numpy fallback)."""
    from gp_dla_detection_amd import _lib as L
    if L.load().gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(L.GpdlaError, match="no HIP device"):
        I.read_spec(str(GOLDEN / "speclite_fixture.fits"))
    z, flags, cols = preload_cases()
    with pytest.raises(L.GpdlaError, match="no HIP device"):
        I.preload_batch(z, flags, cols)
