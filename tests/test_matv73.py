"""MATLAB v7.3 I/O (gp_dla_detection_amd/matv73.py) and the processed_qsos file layout
(process_qsos.m:235-249).

Pins, in order of strength:
* the reference's own consumer (CDDF_analysis/calc_cddf.py DLACatalogue) reads a file this
  package wrote and gets the same values (needs /root/reference and an h5py interpreter; this
  container has both, the GPU box neither -- skipped there);
* libhdf5 (h5py) reads our files with the shapes MATLAB files have;
* our reader reads libhdf5-written MATLAB-style files (committed fixtures from
  tests/golden/make_mat73_fixtures.py, both libhdf5 format generations);
* write -> read round trips for every MATLAB class the pipeline stores.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from gp_dla_detection_amd import matv73 as M
from gp_dla_detection_amd import process as PR
from gp_dla_detection_amd import synthetic as syn

GOLDEN = Path(__file__).parent / "golden"
H5PY_PY = "/opt/conda/bin/python3.9"
REF_CDDF = "/root/reference/CDDF_analysis"


def _has_h5py():
    if not os.path.exists(H5PY_PY):
        return False
    r = subprocess.run([H5PY_PY, "-c", "import h5py"], capture_output=True)
    return r.returncode == 0


needs_h5py = pytest.mark.skipif(not _has_h5py(), reason="no interpreter with h5py")


def test_roundtrip_matlab_classes(tmp_path):
    rng = np.random.default_rng(0)
    Q, S = 37, 53
    big = rng.standard_normal((Q, S))
    v = dict(p_dlas=rng.uniform(size=Q), test_ind=rng.uniform(size=100) < 0.5, release="dr12q",
             num_lines=np.float64(3), model_posteriors=rng.uniform(size=(Q, 2)), empty=np.zeros((0, 0)),
             i32=np.arange(7, dtype=np.int32), u8=np.arange(5, dtype=np.uint8), f32=np.float32([1.5, 2.5]),
             cells=[rng.standard_normal(n) for n in (5, 0, 9)], nested=[["ab", np.arange(3.0)], "xyz"],
             struct=dict(dr9q_concordance=np.array([True, False]), dr12q_visual=np.array([False, True])),
             sample_log_likelihoods_dla=M.LazyArray((Q, S), np.float64, lambda view: view.__setitem__(slice(None), big)))
    for i in range(40):                       # > 8 links: several symbol-table nodes
        v[f"var{i:02d}"] = float(i)
    path = tmp_path / "t.mat"
    M.savemat73(str(path), v)
    assert M.is_matv73(str(path))
    r = M.loadmat73(str(path))
    assert np.array_equal(r["sample_log_likelihoods_dla"], big)
    assert r["p_dlas"].shape == (Q, 1) and np.array_equal(r["p_dlas"][:, 0], v["p_dlas"])
    assert r["test_ind"].dtype == bool and np.array_equal(r["test_ind"][:, 0], v["test_ind"])
    assert r["release"] == "dr12q"
    assert r["num_lines"].shape == (1, 1) and r["num_lines"][0, 0] == 3
    assert np.array_equal(r["model_posteriors"], v["model_posteriors"])
    assert r["empty"].shape == (0, 0)
    assert r["i32"].dtype == np.int32 and r["u8"].dtype == np.uint8 and r["f32"].dtype == np.float32
    assert [c.size for c in r["cells"].ravel()] == [5, 0, 9]
    assert np.array_equal(r["cells"][2, 0].ravel(), v["cells"][2])
    assert r["nested"][1, 0] == "xyz" and r["nested"][0, 0][0, 0] == "ab"
    assert np.array_equal(r["struct"]["dr12q_visual"].ravel(), [False, True])
    assert all(f"var{i:02d}" in r for i in range(40))


def test_large_array_streams_in_blocks(tmp_path):
    a = np.random.default_rng(1).standard_normal((1500, 6000))     # 72 MB > the stream threshold
    path = tmp_path / "big.mat"
    M.savemat73(str(path), dict(big=a))
    assert np.array_equal(M.loadmat73(str(path))["big"], a)


@pytest.mark.parametrize("chunk_rows", [1, 7, 64])
def test_chunked_deferred_region_written_by_blocks(tmp_path, chunk_rows):
    """Sharded saves: a deferred chunked Q x S region (chunks = blocks of whole rows, a multi-level
    chunk B-tree when there are > 64 chunks), filled by several writers with write_chunks in
    arbitrary block order, each a run of whole chunks; the last chunk is partial.  Misaligned
    blocks are refused."""
    rng = np.random.default_rng(6)
    Q, S = 203, 77
    full = rng.standard_normal((Q, S))
    path = str(tmp_path / "c.mat")
    reg = M.savemat73(path, dict(x=np.arange(3.0), sample_log_likelihoods_dla=M.LazyArray(
        (Q, S), np.float64, chunk_rows=chunk_rows)))["sample_log_likelihoods_dla"]
    assert reg.chunk_rows == chunk_rows and reg.chunk_stride % 4096 == 0
    nb = -(-Q // chunk_rows)
    blocks = np.array_split(rng.permutation(nb), 3)
    for blk in blocks:
        for b in sorted(blk):
            r0, r1 = b * chunk_rows, min(Q, (b + 1) * chunk_rows)
            M.write_chunks(path, reg, full[r0:r1], row0=r0, threads=2)
    assert np.array_equal(M.loadmat73(path)["sample_log_likelihoods_dla"], full)
    if chunk_rows > 1:
        with pytest.raises(ValueError):
            M.write_chunks(path, reg, full[1:chunk_rows + 1], row0=1)
    with pytest.raises(ValueError):
        M.open_region(path, reg)


@needs_h5py
def test_h5py_reads_chunked_sample_array(tmp_path):
    """libhdf5 (h5py) reads the chunked layout: 251 chunks of 8 rows (a two-level chunk B-tree),
    the (S, Q) shape and (S, 8) chunk shape MATLAB-style, whole-array, column (one spectrum,
    calc_cddf.py:240) and partial-last-chunk reads."""
    rng = np.random.default_rng(7)
    Q, S = 2003, 50
    full = rng.standard_normal((Q, S))
    path = tmp_path / "c.mat"
    M.savemat73(str(path), dict(x=np.arange(3.0), sample_log_likelihoods_dla=M.LazyArray(
        (Q, S), np.float64, src=full, chunk_rows=8)))
    np.save(tmp_path / "full.npy", full)
    code = ("import h5py,json,sys,numpy as np; f=h5py.File(sys.argv[1],'r'); d=f['sample_log_likelihoods_dla']; "
            "a=np.load(sys.argv[2]); print(json.dumps([list(d.shape), list(d.chunks), "
            "bool(np.array_equal(d[...], a.T)), bool(np.array_equal(d[:, 1234], a[1234])), "
            "bool(np.array_equal(d[:, 2000:], a[2000:].T))]))")
    res = subprocess.run([H5PY_PY, "-B", "-c", code, str(path), str(tmp_path / "full.npy")], capture_output=True,
                         text=True, check=True)
    assert json.loads(res.stdout.strip().splitlines()[-1]) == [[S, Q], [S, 8], True, True, True]


def test_deferred_region_written_in_row_blocks(tmp_path):
    """process.run_process_qsos with world > 1: rank 0 lays out a deferred Q x S region, then every
    rank pwrites its own spectra (rows) of it with write_transposed; uneven blocks, S not a multiple
    of the band."""
    rng = np.random.default_rng(5)
    Q, S = 203, 77
    full = rng.standard_normal((Q, S))
    path = str(tmp_path / "d.mat")
    reg = M.savemat73(path, dict(x=np.arange(3.0), sample_log_likelihoods_dla=M.LazyArray((Q, S), np.float64)))
    reg = reg["sample_log_likelihoods_dla"]
    for r0, r1 in ((0, 70), (70, 71), (71, Q)):
        M.write_transposed(path, reg.offset, full[r0:r1], row0=r0, rows_total=Q, band=8, threads=3)
    assert np.array_equal(M.loadmat73(path)["sample_log_likelihoods_dla"], full)


@pytest.mark.parametrize("tag", ["earliest", "latest"])
def test_reads_libhdf5_written_matlab_files(tag):
    """Files written by libhdf5 the way MATLAB -v7.3 does (chunked + deflate + shuffle, cells in
    #refs#, complex compound, logical, char, empty), superblock v0 and v3 generations."""
    exp = np.load(GOLDEN / "mat73_expected.npz")
    r = M.loadmat73(str(GOLDEN / f"mat73_{tag}.mat"))
    keys = [k.split("__", 1)[1] for k in exp.files if k.startswith(tag + "__")]
    for k in keys:
        if k.startswith("cell_"):
            continue
        assert r[k].shape == exp[f"{tag}__{k}"].shape, k
        assert np.array_equal(r[k], exp[f"{tag}__{k}"]), k
    cells = r["all_flux"].ravel(order="F")
    assert np.array_equal([c.shape[0] for c in cells], exp[f"{tag}__cell_lengths"])
    assert np.array_equal(np.concatenate([c[:, 0] for c in cells]), exp[f"{tag}__cell_concat"])
    # the bulk cell reader: libhdf5's v1 headers (with their modification-time messages) match a
    # template, its chunked cells and v2 headers are decoded one by one; same values either way
    with M.MatFile(str(GOLDEN / f"mat73_{tag}.mat")) as mf:
        n = mf.cell_count("all_flux")
        vals, lens = mf.cell_vectors("all_flux", np.arange(n), np.float64)
        assert np.array_equal(lens, exp[f"{tag}__cell_lengths"]) and np.array_equal(vals, exp[f"{tag}__cell_concat"])
        sel = np.arange(n)[::-3]
        vals, lens = mf.cell_vectors("all_flux", sel, np.float32)
        assert vals.dtype == np.float32 and np.array_equal(vals, np.concatenate([cells[i][:, 0] for i in sel]).astype(np.float32))
        if tag == "earliest":
            addrs = mf._r.dataset(mf._links["all_flux"])[0].ravel().astype(np.int64)
            groups = list(M._bulk_cells(mf._r, addrs))
            assert [g[1] is not None for g in groups] == [True, False]
            chunked = [i for i in range(n) if dict(mf._r.messages(int(addrs[i])))[0x08][1] == 2]
            assert sorted(groups[1][0].tolist()) == chunked and len(chunked) == 11   # the deflated ones
    if tag == "earliest":
        assert r["release"] == "dr12q" and r["empty_var"].shape == (0, 5)


def _processed_out(Q=6, S=200, k=8):
    """processed_qsos variables from the CPU oracle (the checker, never the product)."""
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    spectra = syn.make_spectra(model, Q, dla_fraction=0.5)
    res = [O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"], s["z_qso"],
                              model, samples["offset_samples"], samples["nhi_samples"]) for s in spectra]
    out = dict(training_release="dr12q", training_set_name="dr9q_minus_concordance",
               dla_catalog_name="dr9q_concordance", prior_ind=np.ones(50, dtype=bool), release="dr12q",
               test_set_name="dr12q", test_ind=np.r_[np.ones(Q, dtype=bool), np.zeros(3, dtype=bool)],
               prior_z_qso_increase=PR.P.PRIOR_Z_QSO_INCREASE, max_z_cut=PR.P.MAX_Z_CUT, num_lines=3,
               min_z_dlas=np.array([r["min_z_dla"] for r in res]), max_z_dlas=np.array([r["max_z_dla"] for r in res]),
               log_likelihoods_no_dla=np.array([r["log_likelihood_no_dla"] for r in res]),
               sample_log_likelihoods_dla=np.stack([r["sample_log_likelihoods_dla"] for r in res]),
               log_likelihoods_dla=np.array([r["log_likelihood_dla"] for r in res]))
    out["log_priors_no_dla"] = np.full(Q, np.log(0.8))
    out["log_priors_dla"] = np.full(Q, np.log(0.2))
    out["log_posteriors_no_dla"] = out["log_priors_no_dla"] + out["log_likelihoods_no_dla"]
    out["log_posteriors_dla"] = out["log_priors_dla"] + out["log_likelihoods_dla"]
    out["model_posteriors"], out["p_no_dlas"], out["p_dlas"] = PR.model_posteriors(
        out["log_posteriors_no_dla"], out["log_posteriors_dla"])
    return out, samples


def test_processed_qsos_layout(tmp_path):
    out, _ = _processed_out()
    path = tmp_path / "processed_qsos_dr12q.mat"
    PR.save_processed_qsos(str(path), out)
    r = M.loadmat73(str(path))
    assert sorted(r) == sorted(k for k in PR.PROCESSED_VARIABLES if k in out)
    Q, S = out["sample_log_likelihoods_dla"].shape
    assert r["sample_log_likelihoods_dla"].shape == (Q, S)
    assert np.array_equal(r["sample_log_likelihoods_dla"], out["sample_log_likelihoods_dla"])
    assert r["p_dlas"].shape == (Q, 1) and r["model_posteriors"].shape == (Q, 2)
    assert r["test_ind"].dtype == bool and r["training_set_name"] == "dr9q_minus_concordance"
    assert r["num_lines"].dtype == np.float64


@needs_h5py
def test_h5py_sees_matlab_shapes(tmp_path):
    out, _ = _processed_out()
    path = tmp_path / "processed_qsos_dr12q.mat"
    PR.save_processed_qsos(str(path), out)
    code = ("import h5py,json,sys; f=h5py.File(sys.argv[1],'r'); "
            "print(json.dumps({k: [list(f[k].shape), f[k].attrs['MATLAB_class'].decode()] for k in f if k[0] != '#'}))")
    res = subprocess.run([H5PY_PY, "-c", code, str(path)], capture_output=True, text=True, check=True)
    shapes = json.loads(res.stdout.strip().splitlines()[-1])
    Q, S = out["sample_log_likelihoods_dla"].shape
    assert shapes["sample_log_likelihoods_dla"] == [[S, Q], "double"]      # calc_cddf.py:92,98
    assert shapes["p_dlas"] == [[1, Q], "double"]                          # calc_cddf.py:64
    assert shapes["test_ind"] == [[1, Q + 3], "logical"]                   # calc_cddf.py:69
    assert shapes["release"] == [[5, 1], "char"]


@needs_h5py
@pytest.mark.skipif(not os.path.isdir(REF_CDDF), reason="reference not present (GPU box)")
@pytest.mark.parametrize("layout", ["contiguous", "chunked"])
def test_reference_consumer_reads_our_file(tmp_path, layout):
    """calc_cddf.py's DLACatalogue loads processed_qsos + dla_samples written here and recovers
    p_dla, z ranges, test_ind and the normalised sample likelihoods (with its own
    0.95 < sum < 1.05 assert, calc_cddf.py:246).  Both layouts of the sample array: contiguous
    and chunked in blocks of whole rows (what large and sharded saves write), here 4 rows a chunk
    so the 6 spectra span two chunks, the second one partial."""
    out, samples = _processed_out()
    sll = out["sample_log_likelihoods_dla"]
    saved = dict(out)
    if layout == "chunked":
        saved["sample_log_likelihoods_dla"] = M.LazyArray(sll.shape, np.float64, src=sll, chunk_rows=4)
    proc = tmp_path / "processed_qsos_dr12q.mat"
    samp = tmp_path / "dla_samples.mat"
    snrs = tmp_path / "snrs_qsos_dr12q.mat"
    PR.save_processed_qsos(str(proc), saved)
    PR.save_dla_samples(str(samp), samples)
    Q = out["p_dlas"].size
    M.savemat73(str(snrs), dict(snrs=np.full(Q, 5.0)))
    res = subprocess.run([H5PY_PY, "-B", str(Path(__file__).parent / "cddf_consumer.py"), REF_CDDF, str(proc),
                          str(samp), str(snrs)], capture_output=True, text=True)
    assert res.returncode == 0, res.stderr[-2000:]
    got = json.loads(res.stdout.strip().splitlines()[-1])
    assert np.array_equal(got["p_dla"], out["p_dlas"])
    assert np.array_equal(got["z_min"], out["min_z_dlas"]) and np.array_equal(got["z_max"], out["max_z_dlas"])
    assert got["real_index"] == list(range(Q))
    assert np.array_equal(got["z_offsets"], samples["offset_samples"])
    assert np.array_equal(got["lnhi"], samples["log_nhi_samples"])
    S = out["sample_log_likelihoods_dla"].shape[1]
    norm = {**got["log_norm_like"], **got["log_norm_like_on_demand"]}
    assert norm, "no spectrum passed the reference's p_dla threshold"
    for spec, vals in norm.items():
        spec = int(spec)
        want = out["sample_log_likelihoods_dla"][spec] - (out["log_likelihoods_dla"][spec] + np.log(S))
        np.testing.assert_allclose(vals, want, rtol=0, atol=1e-12)


def test_index_expressions_from_readme():
    """process_qsos.m:7-9,53-55 eval the README's index strings (README.md:242-253)."""
    prior_catalog = dict(in_dr9=np.array([[1], [1], [0], [1]], dtype=bool),
                         filter_flags=np.array([[0], [1], [0], [0]], dtype=np.uint8),
                         los_inds=dict(dr9q_concordance=np.array([[True], [True], [True], [False]])))
    expr = (" prior_catalog.in_dr9 & "
            "(prior_catalog.filter_flags == 0) & "
            " prior_catalog.los_inds(dla_catalog_name)")
    got = PR.evaluate_index(expr, prior_catalog=prior_catalog, dla_catalog_name="dr9q_concordance")
    assert got.tolist() == [True, False, False, False]
    got = PR.evaluate_index("(catalog.filter_flags == 0)", catalog=prior_catalog)
    assert got.tolist() == [True, False, True, True]
    got = PR.evaluate_index("~catalog.in_dr9", catalog=prior_catalog)
    assert got.tolist() == [False, False, True, False]
    mask = np.array([True, False])
    assert PR.evaluate_index(mask) is not None and PR.evaluate_index(mask).tolist() == [True, False]
    got = PR.evaluate_index("catalog.in_dr9 | (catalog.filter_flags ~= 0) && ~false", catalog=prior_catalog)
    assert got.tolist() == [True, True, False, True]
    from gp_dla_detection_amd.index_expr import IndexExpressionError
    # nothing reaches Python's eval: builtins, dunder chains, unknown names and calls are refused
    for bad in ("__import__('os')", "().__class__.__base__.__subclasses__()",
                "catalog.__class__", "catalog._d", "open('x')", "catalog.filter_flags(1)",
                "catalog.in_dr9; 1", "lambda: 0", "catalog.in_dr9 + [1]", "catalog.nope == 0",
                "catalog.los_inds('missing')"):
        with pytest.raises(IndexExpressionError):
            PR.evaluate_index(bad, catalog=prior_catalog)


def write_reference_tree(base, Q=5, S=64, k=8, seed=3):
    """The reference's processed/ directory (set_parameters.m:85-86) with every file process_qsos
    reads, written by this package: catalog.mat (containers.Map variables as structs),
    learned_qso_model_<set>.mat, dla_samples.mat and preloaded_qsos.mat (cells)."""
    rng = np.random.default_rng(seed)
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    spectra = syn.make_dr12q_like_spectra(model, Q, seed=seed)
    d = Path(base) / "dr12q" / "processed"
    d.mkdir(parents=True, exist_ok=True)
    Np = 40
    prior_z = rng.uniform(2.0, 5.0, Np)
    catalog = dict(z_qsos=np.r_[[s["z_qso"] for s in spectra], rng.uniform(2, 4, Np - Q)],
                   filter_flags=np.r_[np.zeros(Q, np.uint8), np.ones(Np - Q, np.uint8)],
                   in_dr9=rng.uniform(size=Np) < 0.8,
                   los_inds=dict(dr9q_concordance=rng.uniform(size=Np) < 0.9),
                   dla_inds=dict(dr9q_concordance=rng.uniform(size=Np) < 0.3),
                   z_dlas=dict(dr9q_concordance=[np.array([z - 0.3]) for z in prior_z]))
    catalog["z_qsos"][Q:] = prior_z[Q:]
    M.savemat73(str(d / "catalog.mat"), catalog)
    M.savemat73(str(d / "learned_qso_model_dr9q_minus_concordance.mat"),
                dict(rest_wavelengths=model["rest_wavelengths"], mu=model["mu"], M=model["M"],
                     log_omega=model["log_omega"], log_c_0=model["log_c_0"], log_tau_0=model["log_tau_0"],
                     log_beta=model["log_beta"]))
    PR.save_dla_samples(str(d / "dla_samples.mat"), samples)
    pad = [syn.make_spectrum(model, 100 + i, dla_fraction=0.0) for i in range(Np - Q)]
    allq = spectra + pad
    M.savemat73(str(d / "preloaded_qsos.mat"),
                dict(all_wavelengths=[s["wavelengths"] for s in allq], all_flux=[s["flux"] for s in allq],
                     all_noise_variance=[s["noise_variance"] for s in allq],
                     all_pixel_mask=[np.asarray(s["pixel_mask"], dtype=bool) for s in allq]))
    return model, samples, spectra, catalog


def test_reference_tree_loaders(tmp_path):
    model, samples, spectra, catalog = write_reference_tree(tmp_path)
    d = tmp_path / "dr12q" / "processed"
    m2 = PR.load_model(str(d / "learned_qso_model_dr9q_minus_concordance.mat"))
    assert np.array_equal(m2["M"], model["M"]) and m2["log_beta"] == model["log_beta"]
    s2 = PR.load_dla_samples(str(d / "dla_samples.mat"))
    assert np.array_equal(s2["nhi_samples"], samples["nhi_samples"])
    tind = PR.evaluate_index("(catalog.filter_flags == 0)", catalog=M.loadmat73(str(d / "catalog.mat")))
    sp = PR.load_preloaded_qsos(str(d / "preloaded_qsos.mat"), tind)
    assert len(sp) == len(spectra)
    for a, b in zip(sp, spectra):
        assert np.array_equal(a["flux"], b["flux"]) and np.array_equal(a["pixel_mask"], b["pixel_mask"])


def _per_cell(mf, name, idx):
    addrs = mf._r.dataset(mf._links[name])[0].ravel().astype(np.int64)
    return [M._decode(mf._r, int(addrs[i])) for i in idx]


def test_bulk_cells_match_per_cell_decode(tmp_path):
    """matv73's bulk cell reader (header templates, run-coalesced copies) against decoding every cell
    on its own: cell arrays mixing doubles of every length (empty included), a matrix, single,
    int32, logical (1-byte data, padded apart in the file), char and nested cells; sorted, reversed,
    repeated and sparse selections."""
    rng = np.random.default_rng(11)
    mixed = [rng.standard_normal(int(n)) for n in rng.integers(1, 40, 50)]
    mixed[3] = np.zeros(0)
    mixed[7] = rng.standard_normal((3, 4))
    mixed[9] = np.float32([1.5, -2.5, 3.0])
    mixed[11] = np.arange(5, dtype=np.int32)
    mixed[13] = rng.uniform(size=6) < 0.5
    mixed[20] = "abc"
    mixed[21] = [np.arange(2.0), "x"]
    masks = [rng.uniform(size=int(n)) < 0.3 for n in rng.integers(1, 30, 40)]
    path = str(tmp_path / "cells.mat")
    M.savemat73(path, dict(mixed=mixed, masks=masks, plain=[rng.standard_normal(int(n)) for n in rng.integers(1, 9, 64)]))
    with M.MatFile(path) as mf:
        for name, n in (("mixed", 50), ("masks", 40), ("plain", 64)):
            for idx in (np.arange(n), np.arange(n)[::-1], np.array([0, 0, 5, 4, n - 1, 5]), np.arange(1, n, 3)):
                ref = _per_cell(mf, name, idx)
                got = mf.cell_elements(name, idx)
                for a, b in zip(ref, got):
                    if isinstance(a, np.ndarray) and a.dtype != object:
                        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
                    else:
                        assert type(a) is type(b)
                if name == "mixed":
                    idx = idx[~np.isin(idx, (20, 21))]   # char / cell cells are not numeric vectors
                    ref = _per_cell(mf, name, idx)
                for dt in (np.float64, np.uint8) if name == "masks" else (np.float64,):
                    vals, lens = mf.cell_vectors(name, idx, dt)
                    exp = [np.asarray(c).ravel(order="F") for c in ref]
                    assert np.array_equal(lens, [c.size for c in exp])
                    assert vals.dtype == dt and np.array_equal(vals, np.concatenate(exp).astype(dt))
        with pytest.raises(TypeError):
            mf.cell_vectors("mixed", [20], np.float64)
        addrs = mf._r.dataset(mf._links["plain"])[0].ravel().astype(np.int64)
        assert [t is not None for _, t, *_ in M._bulk_cells(mf._r, addrs)] == [True]


def test_preloaded_packed_matches_per_spectrum_load(tmp_path):
    """process.load_preloaded_qsos_packed (run_process_qsos's loader) == pack_spectra of the per-
    spectrum load, for a test_ind selection with gaps; cells of unequal length are refused."""
    _, _, spectra, catalog = write_reference_tree(tmp_path)
    pre = str(tmp_path / "dr12q" / "processed" / "preloaded_qsos.mat")
    for sel in (None, np.arange(len(spectra)) % 3 != 1, np.array([4, 0, 2])):
        lst = PR.load_preloaded_qsos(pre, sel)
        exp = syn.pack_spectra([dict(s, z_qso=0.0) for s in lst])
        got = PR.load_preloaded_qsos_packed(pre, sel)
        for k in ("offsets", "wavelengths", "flux", "noise_variance", "pixel_mask"):
            assert got[k].dtype == exp[k].dtype and np.array_equal(got[k], exp[k]), k
    # a mask stored as uint8 (not logical) with values other than 0 / 1 still comes back 0 / 1
    odd = str(tmp_path / "odd.mat")
    M.savemat73(odd, dict(all_wavelengths=[np.arange(3.0)], all_flux=[np.ones(3)], all_noise_variance=[np.ones(3)],
                          all_pixel_mask=[np.array([0, 2, 255], dtype=np.uint8)]))
    assert PR.load_preloaded_qsos_packed(odd)["pixel_mask"].tolist() == [0, 1, 1]
    assert PR.load_preloaded_qsos(odd)[0]["pixel_mask"].tolist() == [False, True, True]
    empty = PR.load_preloaded_qsos_packed(pre, np.zeros(len(spectra), dtype=bool))
    assert empty["offsets"].tolist() == [0] and empty["flux"].size == 0
    bad = str(tmp_path / "bad.mat")
    M.savemat73(bad, dict(all_wavelengths=[np.arange(3.0), np.arange(4.0)], all_flux=[np.arange(3.0), np.arange(5.0)],
                          all_noise_variance=[np.ones(3), np.ones(4)], all_pixel_mask=[np.zeros(3, bool), np.zeros(4, bool)]))
    with pytest.raises(ValueError, match="spectrum 1 has 4 wavelengths"):
        PR.load_preloaded_qsos_packed(bad)


def test_lazy_mat_decodes_on_access(tmp_path):
    path = str(tmp_path / "c.mat")
    M.savemat73(path, dict(z_qsos=np.arange(4.0), filter_flags=np.zeros(4, np.uint8),
                           z_dlas=dict(dr9q_concordance=[np.arange(2.0), np.zeros(0)])))
    with M.LazyMat(path) as lz:
        assert "z_dlas" in lz and "nope" not in lz and dict.__len__(lz) == 0
        assert np.array_equal(lz["z_qsos"].ravel(), np.arange(4.0)) and dict.__len__(lz) == 1
        lz["filter_flags"] = np.ones(4)
        assert lz.get("nope") is None and lz.get("filter_flags").sum() == 4
        assert sorted(lz) == ["filter_flags", "z_dlas", "z_qsos"]
        full = M.loadmat73(path)
        assert np.array_equal(lz["z_dlas"]["dr9q_concordance"][0, 0], full["z_dlas"]["dr9q_concordance"][0, 0])
    assert np.array_equal(lz["z_qsos"], full["z_qsos"])     # decoded values outlive the file
    with pytest.raises(KeyError):
        lz["nope"]


def test_update_variable_requires_matching_shape(tmp_path):
    """save(..., '-append') in place only for the stored MATLAB shape: a same-size value of another
    shape would be written in the wrong column-major order, so it is refused (file untouched)."""
    path = str(tmp_path / "u.mat")
    M.savemat73(path, dict(flags=np.zeros(6, np.uint8), grid=np.zeros((2, 3))))
    before = Path(path).read_bytes()
    assert not M.update_variable(path, "grid", np.ones((3, 2)))
    assert not M.update_variable(path, "flags", np.ones((2, 3), np.uint8))
    assert Path(path).read_bytes() == before
    assert M.update_variable(path, "grid", np.arange(6.0).reshape(2, 3))
    assert M.update_variable(path, "flags", np.arange(6, dtype=np.uint8))        # Q and Q x 1 alike
    r = M.loadmat73(path)
    assert np.array_equal(r["grid"], np.arange(6.0).reshape(2, 3))
    assert np.array_equal(r["flags"][:, 0], np.arange(6))


def test_run_process_qsos_reads_sidecar_filter_flags(tmp_path):
    """When preload_qsos's filter_flags could not go into catalog.mat (ingest.py sidecar), the
    driver's test_ind '(catalog.filter_flags == 0)' uses the sidecar's flags, not the stale ones."""
    from test_process_sharded import ARGS, oracle_compute
    write_reference_tree(tmp_path, Q=4, S=8, k=8)
    d = tmp_path / "dr12q" / "processed"
    flags = np.ravel(M.loadmat73(str(d / "catalog.mat"))["filter_flags"]).copy()
    flags[1] = 16                                       # preload_qsos.m:47: too few pixels
    M.savemat73(str(d / "catalog_filter_flags.mat"), {"filter_flags": flags.reshape(-1, 1)})
    out = PR.run_process_qsos(str(tmp_path), *ARGS, compute=oracle_compute, save=False)
    assert out["test_ind"].sum() == 3 and not out["test_ind"][1]
    assert out["log_likelihoods_dla"].size == 3
