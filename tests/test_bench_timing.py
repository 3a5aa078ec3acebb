"""bench.py's multi-rank machinery on CPU (gloo, world size 2): the timed region's barriers and
max-over-ranks reduction (timed_steps) and the configs[3] LPT spectrum split (dr12q_shard)."""
import importlib.util
import json
import os
import socket
import time
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _bench()
        syncs = []
        el = bench.timed_steps(lambda: time.sleep(0.05 * (rank + 1)), lambda: syncs.append(1), 3, dist)
        q.put((rank, el, len(syncs)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_timed_steps_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (el, ns) for r, el, ns in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 1 sleeps 3 x 0.10 s: both ranks report its time (the max), and each synced twice
    assert got[0][0] == got[1][0]
    assert 0.29 < got[0][0] < 2.0
    assert got[0][1] == got[1][1] == 2


def test_dr12q_lpt_shards_cover_and_balance():
    bench = _bench()
    rng = np.random.default_rng(0)
    pixels = rng.integers(270, 1251, 4096)
    total = 162861
    for world in (2, 3, 8):
        shards = [bench.dr12q_shard(pixels, total, r, world, split=True) for r in range(world)]
        # every spectrum exactly once (pool index i % 4096 counted per position)
        counts = np.bincount(np.concatenate(shards), minlength=4096)
        np.testing.assert_array_equal(counts, np.bincount(np.arange(total) % 4096, minlength=4096))
        loads = np.array([pixels[s].sum() for s in shards], dtype=np.float64)
        assert loads.max() / loads.mean() < 1.001
    np.testing.assert_array_equal(bench.dr12q_shard(pixels, total, 0, 8, split=False), np.arange(total) % 4096)


def _run_bench(*argv, env=None, timeout=240):
    import subprocess
    import sys
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *argv], capture_output=True, text=True,
                          timeout=timeout, env=e)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("workload,total", [("c2", 2048), ("c4", 162861)])
def test_launcher_starts_n_ranks(workload, total):
    """bench.py --gpus 2 with no launcher starts 2 ranks itself (torch.distributed.run children, gloo),
    and rank 0's single JSON line reports both ranks, their devices and disjoint spectrum shards."""
    r = _run_bench("--gpus", "2", "--plan-only", "--workload", workload)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2
    assert [x["rank"] for x in d["ranks"]] == [0, 1]
    assert {x["device"] for x in d["ranks"]} == {0, 1}
    assert d["disjoint"] and d["total_spectra"] == total
    if workload == "c2":
        assert [x["spectra"] for x in d["ranks"]] == [1024, 1024]
        # a multi-rank configs[1] line also measures configs[3] (the full DR12Q count LPT-split over the
        # ranks, strong scaling) and configs[2] end to end with every rank writing
        ap = d["alternatives_planned"]
        c3 = ap["configs3"]
        assert c3["total_spectra"] == 162861 and [x["rank"] for x in c3["ranks"]] == [0, 1]
        assert c3["pixels_max_over_mean"] < 1.0001 and c3["scaling"] == "strong"
        assert {"value", "ranks", "imbalance", "invariant_calc_cddf_246"} <= set(c3["fields"])
        assert ap["e2e"]["writers"] == 2 and "e2e.write_s" in ap["e2e"]["fields"]
    else:
        assert "alternatives_planned" not in d


def test_launcher_world_mismatch_fails():
    r = _run_bench("--gpus", "1", "--plan-only", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_host_cores_reports_the_grant():
    hc = _bench().host_cores()
    assert 1 <= hc["usable"] <= hc["affinity"] <= hc["nproc"]
    assert hc["cgroup_quota_cpus"] is None or hc["usable"] <= max(1, hc["cgroup_quota_cpus"])


def test_profiled_traffic_matches_exact_kernel_names():
    """configs[4]'s roofline traffic counts the GEMM launches only (not convert_gemm_i8_kernel)."""
    bench = _bench()
    f, names = bench.PROFILE_SUMMARY_C5["panel-GEMM-int8-24"]
    d = json.loads(f.read_text())
    want = sum(e["hbm_bytes_per_launch"] for e in d["kernels"] if e["kernel"] in names)
    got, src = bench.profiled_traffic(128, 100000, 50, "panel-GEMM-int8-24")
    assert got == want and "convert" not in src
    assert all(any(e["kernel"] == n for e in d["kernels"]) for n in names)


@pytest.mark.timeout(300)
def test_launcher_refuses_shared_devices():
    """2 ranks planned against 1 device would share a GPU: refused (non-zero) unless --rehearsal, which
    labels the layout and is never an N-GPU point."""
    r = _run_bench("--gpus", "2", "--plan-only", "--plan-devices", "1")
    assert r.returncode != 0
    assert "refusing" in r.stderr and "--rehearsal" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    r = _run_bench("--gpus", "2", "--plan-only", "--plan-devices", "1", "--rehearsal")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["rehearsal"] is True and d["distinct_devices"] == 1
    assert {x["device"] for x in d["ranks"]} == {0}
    r = _run_bench("--gpus", "2", "--plan-only", "--plan-devices", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["rehearsal"] is False and d["distinct_devices"] == 2


def test_assign_device_rule():
    bench = _bench()
    assert bench.assign_device(1, 0, 1, False) == (0, None)
    assert bench.assign_device(8, 5, 8, False) == (5, None)
    dev, err = bench.assign_device(8, 5, 1, False)
    assert dev is None and "refusing" in err
    assert bench.assign_device(8, 5, 2, True) == (1, None)
    assert bench.assign_device(1, 0, 0, True)[0] is None


@pytest.mark.timeout(300)
def test_torchrun_without_gpus_flag_takes_the_launcher_world():
    """DESIGN.md section 5's launch (torch.distributed.run --nproc-per-node N bench.py, no --gpus)
    takes N from WORLD_SIZE instead of failing in every rank."""
    import subprocess
    import sys
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                        "--plan-only"], capture_output=True, text=True, timeout=240, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["world_size"] == 2
