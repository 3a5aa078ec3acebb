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

import os

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


def _engine_compute(model: dict, samples: dict, packed: dict, params: Parameters, device: int = 0,
                    engine: Engine | None = None) -> dict:
    """The hot path on the GPU: per-spectrum null / sample / DLA log likelihoods and z ranges."""
    eng = engine or Engine(model, samples, params, device=device)
    try:
        return eng.process(packed, want_samples=True)
    finally:
        if engine is None:
            eng.close()


def _finish(res: dict, z_qsos, prior: dict | None, params: Parameters, metadata: dict | None) -> dict:
    """process_qsos.m:122-132, 150-155, 202-232: priors, posteriors and the saved scalars."""
    Q = np.asarray(z_qsos).size
    out = dict(
        min_z_dlas=res["min_z_dlas"], max_z_dlas=res["max_z_dlas"],
        log_likelihoods_no_dla=res["log_likelihoods_no_dla"],
        log_likelihoods_dla=res["log_likelihoods_dla"], num_pixels=res["num_pixels"],
        num_lines=params.num_lines, max_z_cut=params.max_z_cut,
        prior_z_qso_increase=params.prior_z_qso_increase)
    if "sample_log_likelihoods_dla" in res:
        out["sample_log_likelihoods_dla"] = res["sample_log_likelihoods_dla"]
    if prior is not None:
        dla_ind = filter_prior_dlas(prior["z_qsos"], prior["dla_ind"], prior.get("z_dlas", [None] * len(prior["z_qsos"])))
        lp_no, lp_dla = dla_priors(z_qsos, prior["z_qsos"], dla_ind, params.prior_z_qso_increase)
    else:
        lp_no, lp_dla = np.full(Q, np.log(0.5)), np.full(Q, np.log(0.5))
    out["log_priors_no_dla"], out["log_priors_dla"] = lp_no, lp_dla
    out["log_posteriors_no_dla"] = lp_no + out["log_likelihoods_no_dla"]      # process_qsos.m:154-155
    out["log_posteriors_dla"] = lp_dla + out["log_likelihoods_dla"]           # process_qsos.m:211-212
    post, p_no, p_dla = model_posteriors(out["log_posteriors_no_dla"], out["log_posteriors_dla"])
    out["model_posteriors"], out["p_no_dlas"], out["p_dlas"] = post, p_no, p_dla
    if "numeric_warning" in res:
        out["numeric_warning"] = res["numeric_warning"]
    for key, val in (metadata or {}).items():
        out[key] = val
    return out


def process_qsos(model: dict, samples: dict, spectra, prior: dict | None = None,
                 params: Parameters | None = None, test_ind=None, engine: Engine | None = None,
                 device: int = 0, metadata: dict | None = None) -> dict:
    """Run the DLA search (process_qsos.m:88-232) and return the saved variables."""
    params = params or set_parameters(k=np.asarray(model["M"]).shape[1])
    packed = _select(spectra, test_ind)
    res = _engine_compute(model, samples, packed, params, device, engine)
    out = _finish(res, packed["z_qsos"], prior, params, metadata)
    if test_ind is not None:
        out["test_ind"] = np.asarray(test_ind)
    return out


# names of process_qsos.m:235-243, in order
PROCESSED_VARIABLES = ("training_release", "training_set_name", "dla_catalog_name", "prior_ind",
                       "release", "test_set_name", "test_ind", "prior_z_qso_increase", "max_z_cut",
                       "num_lines", "min_z_dlas", "max_z_dlas", "log_priors_no_dla", "log_priors_dla",
                       "log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla",
                       "log_posteriors_no_dla", "log_posteriors_dla", "model_posteriors", "p_no_dlas",
                       "p_dlas")


def save_processed_qsos(path: str, out: dict, format: str = "v7.3") -> dict:
    """``save(filename, variables_to_save{:}, '-v7.3')`` (process_qsos.m:235-249).

    MATLAB shapes: Q-vectors are Q x 1 columns, ``sample_log_likelihoods_dla`` is Q x S,
    ``model_posteriors`` Q x 2, strings are char rows, ``test_ind``/``prior_ind`` logical.  The
    default container is v7.3 (HDF5, matv73.py): what the reference writes and what
    calc_cddf.py reads with h5py (Q-vectors as (1, Q), the sample array as (S, Q)); it has no
    per-variable size limit and streams the sample array into the file.  ``format="v5"`` writes
    a scipy MATLAB v5 file instead (each variable must then stay under 2 GB)."""
    mat = {}
    for key in PROCESSED_VARIABLES:
        if key not in out:
            continue
        v = out[key]
        if isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
            v = np.float64(v)          # MATLAB numeric literals are double (num_lines = 3)
        mat[key] = v
    if format == "v7.3":
        from .matv73 import savemat73
        return savemat73(path, mat)
    elif format == "v5":
        from scipy.io import savemat
        mat = {k: (v[:, None] if isinstance(v, np.ndarray) and v.ndim == 1 else v) for k, v in mat.items()}
        savemat(path, mat, do_compression=False, oned_as="column")
        return {}
    raise ValueError("format must be 'v7.3' or 'v5'")


# ------------------------------------------------------------------------------ file-level driver
def processed_directory(base_directory: str, release: str) -> str:
    """set_parameters.m:85-86."""
    return f"{base_directory}/{release}/processed"


class _MatMap:
    def __init__(self, d: dict):
        self._d = d

    def __call__(self, key):
        v = self._d[key]
        if isinstance(v, np.ndarray) and v.dtype != object and v.ndim == 2 and 1 in v.shape:
            return v.ravel()
        if isinstance(v, np.ndarray) and v.dtype == object:
            return list(v.ravel(order="F"))
        return v


def evaluate_index(expr, **names) -> np.ndarray:
    """``if (ischar(ind)) ind = eval(ind); end`` (process_qsos.m:7-9,53-55).  A boolean/integer
    array passes through; a callable gets the named structs; a string is parsed as the
    reference's MATLAB index expression (``&``, ``|``, ``~``, ``==``, ``~=``, field access and
    containers.Map lookup, README.md:242-253) by the restricted evaluator in index_expr.py --
    never by Python's ``eval``."""
    if callable(expr):
        return np.asarray(expr(**names))
    if isinstance(expr, str):
        from .index_expr import evaluate_index_string
        return evaluate_index_string(expr, **names)
    return np.asarray(expr)


def _as_list(cells) -> list:
    if isinstance(cells, np.ndarray) and cells.dtype == object:
        return [np.asarray(c).ravel() for c in cells.ravel(order="F")]
    return [np.asarray(c).ravel() for c in cells]


def load_model(path: str) -> dict:
    """process_qsos.m:29-35 (learned_qso_model_<training_set_name>.mat)."""
    from .matv73 import loadmat
    d = loadmat(path, ["rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0", "log_beta"])
    out = {k: np.asarray(d[k], dtype=np.float64).ravel() for k in ("rest_wavelengths", "mu", "log_omega")}
    out["M"] = np.asfortranarray(np.asarray(d["M"], dtype=np.float64))
    for k in ("log_c_0", "log_tau_0", "log_beta"):
        out[k] = float(np.asarray(d[k]).ravel()[0])
    return out


def load_dla_samples(path: str) -> dict:
    """process_qsos.m:37-40 (dla_samples.mat)."""
    from .matv73 import loadmat
    d = loadmat(path, ["offset_samples", "log_nhi_samples", "nhi_samples"])
    return {k: np.asarray(v, dtype=np.float64).ravel() for k, v in d.items()}


def save_dla_samples(path: str, samples: dict, **extra) -> None:
    """dla_samples.mat (generate_dla_samples.m:59-63): the sample vectors are MATLAB 1 x S rows
    (h5py sees (S, 1); calc_cddf.py:121-123 reads ``[:, 0]``)."""
    from .matv73 import savemat73
    var = {k: np.asarray(samples[k], dtype=np.float64).reshape(1, -1)
           for k in ("offset_samples", "log_nhi_samples", "nhi_samples") if k in samples}
    var.update(extra)
    savemat73(path, var)


def load_preloaded_qsos(path: str, test_ind=None) -> list[dict]:
    """process_qsos.m:45-60 (preloaded_qsos.mat cells, selected by test_ind); z_QSO is attached
    by the caller from the catalogue.  v7.3 files decode only the selected cells."""
    from .matv73 import MatFile, is_matv73, loadmat
    keys = ("all_wavelengths", "all_flux", "all_noise_variance", "all_pixel_mask")
    if is_matv73(path):
        with MatFile(path) as mf:
            n = mf.cell_count("all_wavelengths")
            idx = _indices(test_ind, n)
            cols = {k: [np.asarray(c).ravel() for c in mf.cell_elements(k, idx)] for k in keys}
    else:
        d = loadmat(path, list(keys))
        full = {k: _as_list(d[k]) for k in d}
        idx = _indices(test_ind, len(full["all_wavelengths"]))
        cols = {k: [full[k][i] for i in idx] for k in keys}
    return [dict(wavelengths=w, flux=f, noise_variance=v, pixel_mask=m.astype(bool))
            for w, f, v, m in zip(cols["all_wavelengths"], cols["all_flux"], cols["all_noise_variance"],
                                  cols["all_pixel_mask"])]


def load_preloaded_qsos_packed(path: str, test_ind=None) -> dict:
    """``pack_spectra(load_preloaded_qsos(path, test_ind))`` without z_qsos (the caller attaches
    them from the catalogue): the engine's CSR arrays straight from the file, with the cells of a
    v7.3 file read in bulk (matv73.MatFile.cell_vectors) rather than decoded one by one."""
    from .matv73 import MatFile, is_matv73
    if not is_matv73(path):
        lst = load_preloaded_qsos(path, test_ind)
        if not lst:
            return dict(offsets=np.zeros(1, np.int64), wavelengths=np.zeros(0), flux=np.zeros(0),
                        noise_variance=np.zeros(0), pixel_mask=np.zeros(0, np.uint8))
        out = pack_spectra([dict(s, z_qso=0.0) for s in lst])
        del out["z_qsos"]
        return out
    keys = (("wavelengths", "all_wavelengths", np.float64), ("flux", "all_flux", np.float64),
            ("noise_variance", "all_noise_variance", np.float64), ("pixel_mask", "all_pixel_mask", np.bool_))
    out = {}
    with MatFile(path) as mf:
        idx = _indices(test_ind, mf.cell_count("all_wavelengths"))
        lengths = None
        for key, var, dt in keys:
            out[key], n = mf.cell_vectors(var, idx, dt)
            if lengths is None:
                lengths = n
            elif not np.array_equal(n, lengths):
                q = int(np.flatnonzero(n != lengths)[0])
                raise ValueError(f"preloaded_qsos: spectrum {int(idx[q])} has {int(lengths[q])} wavelengths "
                                 f"but {int(n[q])} entries in {var}")
    out["pixel_mask"] = out["pixel_mask"].view(np.uint8)   # 0 / 1, as pack_spectra of the bool masks
    out["offsets"] = np.zeros(idx.size + 1, dtype=np.int64)
    np.cumsum(lengths, out=out["offsets"][1:])
    return out


def _indices(sel, n: int) -> np.ndarray:
    if sel is None:
        return np.arange(n)
    sel = np.asarray(sel)
    return np.flatnonzero(sel) if sel.dtype == bool else sel.astype(np.int64)


def run_process_qsos(base_directory: str, training_release: str, training_set_name: str,
                     dla_catalog_name: str, prior_ind, release: str, test_set_name: str, test_ind,
                     params: Parameters | None = None, device: int = 0, save: bool = True,
                     rank: int = 0, world: int = 1, compute=None, timings: dict | None = None,
                     chunk_rows: int | None = None) -> dict:
    """The whole ``process_qsos`` script (process_qsos.m:1-249) on files laid out as the reference
    lays them out (set_parameters.m:79-86):

      <base>/<training_release>/processed/catalog.mat                  (prior catalogue)
      <base>/<training_release>/processed/learned_qso_model_<set>.mat
      <base>/<training_release>/processed/dla_samples.mat
      <base>/<release>/processed/catalog.mat, preloaded_qsos.mat
      -> <base>/<release>/processed/processed_qsos_<test_set_name>.mat  (v7.3)

    ``prior_ind`` / ``test_ind`` are the reference's index expressions (strings such as
    ``'(catalog.filter_flags == 0)'``), callables or boolean arrays.  The catalogue's
    containers.Map variables (los_inds, dla_inds, z_dlas) are read as structs keyed by catalogue
    name (MATLAB's MCOS Map objects are opaque outside MATLAB, SURVEY.md 7 viii).

    Multi-GPU (``world`` > 1; one process per GPU with a torch.distributed process group already
    initialised, gloo suffices): rank r decodes and evaluates only its contiguous shard of the
    test spectra on ``device``.  The Q x S sample array is a chunked HDF5 dataset whose chunks
    are blocks of whole rows (``matv73.auto_chunk_rows`` spectra each, ~4 MB), and the shards are
    whole chunk blocks, LPT-balanced on the expected pixel count of each block (``shard.py``), so
    ranks get equal sweep work and each writes only whole chunks of its own.  Rank 0 gathers the
    per-spectrum scalars (not the sample arrays), computes priors and posteriors, and writes the
    file with the sample array deferred; every rank then pwrites its own chunks (disjoint 4 KiB-
    aligned ranges of the one file), so the 13 GB full-DR12Q array is never gathered.
    ``compute(model, samples, packed, params, device) -> dict`` replaces the engine (tests);
    ``chunk_rows`` overrides the sharded file's rows per chunk (tests).
    ``timings`` (a dict) receives this rank's wall seconds per phase: load (the four input files,
    process_qsos.m:1-63), compute (the engine, :88-212) and write (priors / posteriors and the
    v7.3 file, :222-249).
    Rank 0 returns the saved scalars; other ranks their local results."""
    import time
    from .matv73 import LazyArray, LazyMat, auto_chunk_rows, is_matv73, loadmat, write_chunks
    from .shard import block_lpt_shards, expected_pixels, merge_shards
    compute = compute or _engine_compute
    tm = timings if timings is not None else {}
    t_start = time.perf_counter()
    tdir, rdir = processed_directory(base_directory, training_release), processed_directory(base_directory, release)
    prior_catalog = loadmat(f"{tdir}/catalog.mat")
    pind = evaluate_index(prior_ind, prior_catalog=prior_catalog, dla_catalog_name=dla_catalog_name).astype(bool).ravel()
    pz = np.asarray(prior_catalog["z_qsos"], dtype=np.float64).ravel()[pind]
    pdla = np.asarray(_MatMap(prior_catalog["dla_inds"])(dla_catalog_name)).astype(bool).ravel()[pind]
    z_dlas_all = _MatMap(prior_catalog["z_dlas"])(dla_catalog_name)
    pzd = [z_dlas_all[i] for i in np.flatnonzero(pind)]
    model = load_model(f"{tdir}/learned_qso_model_{training_set_name}.mat")
    samples = load_dla_samples(f"{tdir}/dla_samples.mat")
    params = params or set_parameters(k=np.asarray(model["M"]).shape[1])
    # the release catalogue: only what test_ind names, and z_qsos, is decoded (not its z_dlas cells)
    catalog = LazyMat(f"{rdir}/catalog.mat") if is_matv73(f"{rdir}/catalog.mat") else loadmat(f"{rdir}/catalog.mat")
    side = f"{rdir}/catalog_filter_flags.mat"
    if os.path.exists(side):
        # preload_qsos's filter_flags when catalog.mat could not take them in place (ingest.py:
        # a catalog holding MATLAB objects is never rewritten): the sidecar supersedes the stale copy
        catalog["filter_flags"] = loadmat(side)["filter_flags"]
    tind = evaluate_index(test_ind, catalog=catalog).astype(bool).ravel()
    tidx = np.flatnonzero(tind)
    z_all = np.asarray(catalog["z_qsos"], dtype=np.float64).ravel()[tidx]
    if isinstance(catalog, LazyMat):
        catalog.close()
    S = np.asarray(samples["nhi_samples"]).size
    if not chunk_rows:
        chunk_rows = auto_chunk_rows(S, 8, tidx.size)
        if world > 1:
            # at least ~4 blocks per rank, so a small Q still spreads over every rank (every rank
            # derives the same value from Q and world before the file exists)
            chunk_rows = max(1, min(chunk_rows, -(-tidx.size // (4 * world) // 8) * 8 or 8))
    shards = block_lpt_shards(expected_pixels(z_all), chunk_rows, world)
    mine = shards[rank]
    packed = load_preloaded_qsos_packed(f"{rdir}/preloaded_qsos.mat", tidx[mine])
    packed["z_qsos"] = np.ascontiguousarray(z_all[mine], dtype=np.float64)
    t_load = time.perf_counter()
    tm["load_s"] = t_load - t_start
    if compute is _engine_compute:  # the compute phase split: engine creation, then the batches
        eng = Engine(model, samples, params, device=device)
        tm["engine_create_s"] = time.perf_counter() - t_load
        try:
            res = eng.process(packed, want_samples=True, timings=tm)
        finally:
            eng.close()
    else:
        res = compute(model, samples, packed, params, device)
    t_comp = time.perf_counter()
    tm["compute_s"] = t_comp - t_load
    meta = dict(training_release=training_release, training_set_name=training_set_name,
                dla_catalog_name=dla_catalog_name, prior_ind=pind, release=release,
                test_set_name=test_set_name)
    prior = dict(z_qsos=pz, dla_ind=pdla, z_dlas=pzd)
    path = f"{rdir}/processed_qsos_{test_set_name}.mat"
    if world == 1:
        out = _finish(res, z_all, prior, params, meta)
        out["test_ind"] = tind
        if save:
            save_processed_qsos(path, out)
        tm["write_s"] = time.perf_counter() - t_comp
        return out
    import torch.distributed as dist
    small = {k: v for k, v in res.items() if k != "sample_log_likelihoods_dla"}
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(small, gathered, dst=0)
    region = [None]
    if rank == 0:
        merged = merge_shards(tidx.size, shards, gathered)
        # GPDLA_ENUMERIC on any rank (its likelihoods are NaN): keep every rank's report
        warns = [f"rank {r}: {g['numeric_warning']}" for r, g in enumerate(gathered) if g.get("numeric_warning")]
        if warns:
            merged["numeric_warning"] = "; ".join(warns)
        out = _finish(merged, z_all, prior, params, meta)
        out["test_ind"] = tind
        if save:   # deferred, chunked by the rows the shards were cut on
            out["sample_log_likelihoods_dla"] = LazyArray((tidx.size, S), np.float64, chunk_rows=chunk_rows)
            region[0] = save_processed_qsos(path, out)["sample_log_likelihoods_dla"]
            del out["sample_log_likelihoods_dla"]
    if save:
        dist.broadcast_object_list(region, src=0)
        # this rank's chunks, straight into the file (page cache; no msync, as matv73): one call per
        # run of consecutive blocks
        sll = np.asarray(res["sample_log_likelihoods_dla"])
        breaks = np.flatnonzero(np.diff(mine) != 1) + 1
        for lo, hi in zip(np.r_[0, breaks], np.r_[breaks, mine.size]):
            if hi > lo:
                write_chunks(path, region[0], sll[lo:hi], row0=int(mine[lo]))
        dist.barrier()
    tm["write_s"] = time.perf_counter() - t_comp
    return out if rank == 0 else res


