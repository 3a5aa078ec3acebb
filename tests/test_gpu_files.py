"""GPU: the file-level ``process_qsos`` script (process_qsos.m:1-249) end to end -- reference
directory tree in, processed_qsos_<set>.mat (v7.3) out -- against the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from conftest import tol_ok  # noqa: E402
from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import matv73 as M  # noqa: E402
from gp_dla_detection_amd import process as PR  # noqa: E402
from test_matv73 import write_reference_tree  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    assert L.load().gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def test_run_process_qsos_files(tmp_path):
    from oracle import gpdla_oracle as O
    model, samples, spectra, catalog = write_reference_tree(tmp_path, Q=5, S=64, k=8)
    prior_ind = " prior_catalog.in_dr9 & prior_catalog.los_inds(dla_catalog_name)"
    out = PR.run_process_qsos(str(tmp_path), "dr12q", "dr9q_minus_concordance", "dr9q_concordance", prior_ind,
                              "dr12q", "dr12q", "(catalog.filter_flags == 0)")
    path = tmp_path / "dr12q" / "processed" / "processed_qsos_dr12q.mat"
    saved = M.loadmat73(str(path))
    assert sorted(saved) == sorted(PR.PROCESSED_VARIABLES)
    Q, S = len(spectra), samples["nhi_samples"].size
    assert saved["sample_log_likelihoods_dla"].shape == (Q, S)
    np.testing.assert_array_equal(saved["sample_log_likelihoods_dla"], out["sample_log_likelihoods_dla"])
    for q, s in enumerate(spectra):
        ref = O.process_spectrum(s["wavelengths"], s["flux"], s["noise_variance"], s["pixel_mask"], s["z_qso"],
                                 model, samples["offset_samples"], samples["nhi_samples"])
        assert np.all(tol_ok(saved["sample_log_likelihoods_dla"][q], ref["sample_log_likelihoods_dla"], 1e-9))
        assert tol_ok(saved["log_likelihoods_dla"][q, 0], ref["log_likelihood_dla"], 1e-9)
        assert tol_ok(saved["log_likelihoods_no_dla"][q, 0], ref["log_likelihood_no_dla"], 1e-9)
    # priors (process_qsos.m:4-27,122-132) against the oracle's restatement
    pind = np.asarray(catalog["in_dr9"]) & np.asarray(catalog["los_inds"]["dr9q_concordance"])
    pz = catalog["z_qsos"][pind]
    pdla = catalog["dla_inds"]["dr9q_concordance"][pind]
    pzd = [catalog["z_dlas"]["dr9q_concordance"][i] for i in np.flatnonzero(pind)]
    lp_no, lp_dla = O.dla_priors(np.array([s["z_qso"] for s in spectra]), pz, pdla, pzd)
    np.testing.assert_allclose(saved["log_priors_dla"][:, 0], lp_dla, rtol=0, atol=1e-14)
    np.testing.assert_allclose(saved["log_priors_no_dla"][:, 0], lp_no, rtol=0, atol=1e-14)
    assert saved["prior_ind"].ravel().tolist() == pind.tolist()
    assert saved["test_ind"].ravel().tolist() == (catalog["filter_flags"] == 0).tolist()
    post = saved["model_posteriors"]
    assert post.shape == (Q, 2) and np.allclose(post.sum(axis=1), 1)


def _rank_worker(rank, world, port, base, q):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gp_dla_detection_amd import process as PRw
        devs = L.load().gpdla_device_count()
        PRw.run_process_qsos(base, "dr12q", "dr9q_minus_concordance", "dr9q_concordance",
                             " prior_catalog.in_dr9 & prior_catalog.los_inds(dla_catalog_name)", "dr12q", "dr12q",
                             "(catalog.filter_flags == 0)", device=rank % devs, rank=rank, world=world)
        q.put(rank)
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world,Q", [(2, 6), (4, 36)])
def test_run_process_qsos_ranks(tmp_path, world, Q):
    """One process per GPU (ranks share the device on a one-GPU box): the sharded run writes the
    same processed_qsos file as the single-process run -- 2 ranks on 6 spectra (one chunk block:
    rank 1 gets an empty shard) and 4 ranks on 36 (5 blocks of <= 8 rows over the ranks, each writing
    its own chunks)."""
    import socket

    import torch.multiprocessing as mp
    single, multi = tmp_path / "single", tmp_path / "multi"
    for d in (single, multi):
        write_reference_tree(d, Q=Q, S=48, k=8)
    args = ("dr12q", "dr9q_minus_concordance", "dr9q_concordance",
            " prior_catalog.in_dr9 & prior_catalog.los_inds(dla_catalog_name)", "dr12q", "dr12q",
            "(catalog.filter_flags == 0)")
    PR.run_process_qsos(str(single), *args)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, str(multi), q)) for r in range(world)]
    for pr in procs:
        pr.start()
    assert sorted(q.get(timeout=300) for _ in range(world)) == list(range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    a = M.loadmat73(str(single / "dr12q" / "processed" / "processed_qsos_dr12q.mat"))
    b = M.loadmat73(str(multi / "dr12q" / "processed" / "processed_qsos_dr12q.mat"))
    for k in a:
        if isinstance(a[k], str):
            assert a[k] == b[k]
        else:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
