#!/usr/bin/env python3
"""Benchmark: (spectrum x DLA-sample) log-evidence evaluations per second on MI355X.

Default workload (BASELINE.json configs[1], --workload c2): 1024 synthetic spectra per GPU,
n = 800 unmasked pixels, k = 20, S = 10^4 DLA samples, fp64.  --workload c3 / c4 / c5 run the
other configs (full DR12Q count on one GPU / split over the ranks; k = 50 with 10^5 samples on the
panel-GEMM path).  One step = one pass of the hot path over the batch:
spectrum preparation, the fused Voigt x low-rank-Gaussian likelihood for every (spectrum,
sample) pair plus the null model, and the per-spectrum log-mean-exp.  Inputs are resident in HBM
before timing starts; outputs (incl. the 1024 x 10^4 sample log-likelihoods) stay in HBM.

Multi-GPU (torch.distributed.run, one process per GPU): spectra are sharded with no data-path
collective (weak scaling: 1024 spectra per rank); the only collectives are the timing barrier
and the max-over-ranks of the elapsed time, on the gloo backend (host-side: the hot path has no
exchange step, so nothing needs RCCL).  Device buffers come from libgpdla itself, so the process
holds a single HIP runtime (the system ROCm one the library was built against).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 (vector and matrix), datasheet
I8_PEAK_TOPS = 5000.0       # MI355X dense int8 MFMA (2x the ~2.5 PF dense BF16 rate; MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E, datasheet


def algorithmic_flops_per_eval(n: int, k: int) -> float:
    """packed Gram + projection + per-pixel scalars + Cholesky + solve."""
    return n * k * (k + 1) + 2 * n * k + 10 * n + k ** 3 / 3 + 2 * k ** 2


def i8_ops_per_eval(n: float, k: int, gram_pairs: int = 10) -> float:
    """int8 MFMA ops of the exact Gram/u contraction, 2 ops per multiply-add:
    n slots x (k(k+1)/2 Gram entries x gram_pairs + k u entries x 10) digit pairs.  gram_pairs = 10
    for the 32-bit scheme (4 digits, levels <= 3), 6 for panel_gemm_i8_24 (3 digits, levels <= 2;
    its u entries keep 4 digits)."""
    return 2 * n * (gram_pairs * k * (k + 1) / 2 + 10 * k)


FP32_MATRIX_PEAK_TFLOPS = 157.3   # MI355X f32-input MFMA = the f32 vector peak (MI355X_MICROARCH.md)


def i8_roofline(st: dict, n: float, k: int, Q: int, S: int, steps: int, path: str) -> dict:
    """Roofline of the int8 panel paths' dominant kernel, the int8 GEMM (gemm_i8.hip): its digit-expanded
    int8 ops per launch / its average launch time (HIP events around each launch on the engine's
    stream, gpdla_stats.contraction_ms), against the dense int8 MFMA peak (2x BF16 per clock,
    MI355X_MICROARCH.md).  ``frac`` is the MFMA utilisation of the digit scheme, not algorithmic work:
    every Gram entry costs 6 (24-bit path) or 10 (32-bit path) int8 digit-pair products and every u
    entry 10.  The whole batch (weights + GEMM + LDL^T) is reported beside it in algorithmic flops
    (SURVEY 8d F_eval), set against the FP32 matrix peak of the precision BASELINE quotes configs[4]
    in."""
    pairs = 6 if path.endswith("-24") else 10
    ops = i8_ops_per_eval(n, k, pairs)
    nl = max(st["contraction_launches"], 1)
    gemm_ms = st["contraction_ms"] / nl
    evals_per_gemm = Q * (S + 1) * steps / nl
    achieved = ops * evals_per_gemm / (gemm_ms * 1e-3) / 1e12
    batch_ms = st["likelihood_ms"] / max(st["likelihood_launches"], 1)
    evals_per_batch = Q * (S + 1) * steps / max(st["likelihood_launches"], 1)
    alg = algorithmic_flops_per_eval(n, k) * evals_per_batch / (batch_ms * 1e-3) / 1e12
    return {"bound": "mfma", "mfma_dtype": "i8", "unit": "TOPS", "peak": I8_PEAK_TOPS, "achieved": achieved,
            "frac": achieved / I8_PEAK_TOPS,
            "frac_meaning": f"MFMA utilisation of the digit scheme: {pairs} int8 digit-pair products per Gram entry "
                            f"and 10 per u entry (digit-expanded int8 ops, not algorithmic work) over the dense "
                            f"int8 peak",
            "avg_launch_ms": gemm_ms, "evals_per_launch": evals_per_gemm,
            "i8_ops_per_eval": ops,
            "whole_batch": {"avg_ms": batch_ms, "evals": evals_per_batch,
                            "digit_tops": ops * evals_per_batch / (batch_ms * 1e-3) / 1e12,
                            "digit_frac_of_i8_peak": ops * evals_per_batch / (batch_ms * 1e-3) / 1e12 / I8_PEAK_TOPS,
                            "algorithmic_tflops": alg,
                            "fp32_matrix_peak_tflops": FP32_MATRIX_PEAK_TFLOPS,
                            "algorithmic_over_fp32_matrix_peak": alg / FP32_MATRIX_PEAK_TFLOPS,
                            "note": "algorithmic_tflops = SURVEY 8d's F_eval (packed Gram, projection, per-pixel "
                                    "terms, Cholesky, solve) per evaluation over the batch time.  It may exceed "
                                    "the FP32 matrix peak because the Gram/u contraction runs exactly on the int8 "
                                    "matrix cores (DESIGN.md section 10), not in fp32 or fp64"},
            "note": "the int8 GEMM launch(es) of one spectrum and sample chunk only (the 24-bit path runs its Gram "
                    "and u contractions in one launch); the batch adds the weights and LDL^T kernels"}


def single_stream_stats(eng, step, streams: int = 2, steps: int = 2) -> dict:
    """Engine stats of ``steps`` steps with the batch on ONE compute stream, after the timed region (one
    untimed step first), for the panel paths' GEMM launch at its own rate.  In the timed region a
    batch's spectra alternate over two streams (gpdla_engine_set_panel_streams), so a GEMM launch
    shares the CUs with the other stream's weights / LDL^T kernels, and the HIP events around it also
    count the time it waits in its queue for them (rocprofv3's kernel trace, which times the kernel
    from its first wave, reads less: profiles/round5/r11c_c5_summary.md)."""
    eng.set_panel_streams(1)
    step()
    eng.synchronize()
    eng.reset_stats()
    for _ in range(steps):
        step()
    eng.synchronize()
    st = eng.stats()
    eng.set_panel_streams(streams)
    return st


def panel_roofline_streams(timed: dict, alone: dict, streams: int = 2) -> dict:
    """The panel paths' roofline record: the timed region's GEMM launches (HIP events around each launch
    while a batch's spectra alternate over ``streams`` streams), and nested beside it the kernel's own
    rate (one stream, after the timed region; agrees with a one-stream rocprofv3 trace).  With two
    streams a launch shares the CUs with, and queues behind, the other stream's weights / LDL^T
    kernels, so its event span is longer than its run time: the timed figure is the lower one."""
    if "avg_launch_ms" not in timed or "avg_launch_ms" not in alone:
        return timed
    return {**timed,
            "measured": f"GEMM launches in the timed region ({streams} panel streams, HIP events incl. queueing)",
            "one_stream": {k: alone[k] for k in ("avg_launch_ms", "achieved", "frac", "evals_per_launch") if k in alone}
            | {"measured": "GEMM launches with the batch on one compute stream, 2 steps after the timed region "
                           "(the kernel's own rate; profiles/round5/r11d_c5s1_summary.md)"}}


def f64_gemm_roofline(st: dict, n: float, k: int, Q: int, S: int, steps: int) -> dict:
    """Roofline of the fp64 panel path's dominant kernel, the Gram/u GEMM on the f64 matrix cores
    (gemm_f64.hip): 2 n (k(k+1)/2 + k) algorithmic flops per evaluation (the Gram and u part of
    SURVEY.md 8d's F_eval) over its average launch time (HIP events around the Gram + u launches of
    each spectrum and sample chunk, gpdla_stats.contraction_ms), against the FP64 matrix peak."""
    flops = 2 * n * (k * (k + 1) / 2 + k)
    if st["contraction_launches"] == 0:      # a library build without GEMM timing (A/B variants)
        return {"note": "no GEMM launch timing in this library build"}
    nl = st["contraction_launches"]
    gemm_ms = st["contraction_ms"] / nl
    evals_per_gemm = Q * (S + 1) * steps / nl
    achieved = flops * evals_per_gemm / (gemm_ms * 1e-3) / 1e12
    return {"bound": "mfma", "mfma_dtype": "f64", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS, "achieved": achieved,
            "frac": achieved / FP64_PEAK_TFLOPS, "avg_launch_ms": gemm_ms, "evals_per_launch": evals_per_gemm,
            "gemm_flops_per_eval": flops,
            "note": "gemm_f64 launches only (Gram + u per spectrum and sample chunk, counted as one); the batch "
                    "adds the weights and LDL^T kernels"}


def effective_bytes_per_eval(n: int, k: int, w: int = 8) -> float:
    """SURVEY.md 8d streamed-panel accounting (north-star 'effective HBM')."""
    return w * (n * (k + 5) + 8) + w


def _numpy_worker(task):
    """The numpy oracle on one host core (secondary CPU figure), until the time budget is spent."""
    model, spec, offsets, nhis, budget_s = task
    from threadpoolctl import threadpool_limits
    from oracle import gpdla_oracle as O
    done = 0
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        prep = O.prepare_spectrum(spec["wavelengths"], spec["flux"], spec["noise_variance"],
                                  spec["pixel_mask"], spec["z_qso"], model)
        zs = prep["zmin"] + (prep["zmax"] - prep["zmin"]) * offsets
        for z, N in zip(zs, nhis):
            O.sample_log_likelihood(prep, z, N, 3)
            done += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        el = time.perf_counter() - t0
    return done, el


def host_cores() -> dict:
    """The host cores this process may use: the affinity mask (sched_getaffinity), the cgroup CPU
    quota (cpu.max, cgroup v2; a leased GPU box grants a share of a larger host this way), nproc and
    the CPU model.  ``usable`` = the affinity count, capped by the quota when one is set."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, math.floor(quota)))
    return {"affinity": aff, "cgroup_quota_cpus": quota, "nproc": os.cpu_count(), "cpu_model": model,
            "usable": usable}


def cpu_baseline(model, samples, spectra, budget_s: float, k: int, widened: bool = False) -> dict:
    """The reference's CPU path, restated in C++ with OpenMP over the DLA samples like its parfor
    (oracle/cpu_ref.cpp: process_qsos.m:184-198, voigt.c:253-304 with an own Faddeeva function in
    place of libcerf, log_mvnpdf_low_rank.m:5-33 in MATLAB operation order), on every host core the
    process is granted (host_cores(): the affinity mask capped by the cgroup quota).
    configs[0] (one spectrum, the null model only) is timed in full; the bench workload on a
    bounded subset: whole spectra (all S samples each), at least 16, until ``budget_s`` is spent.
    The numpy restatement on one core is reported beside it.  Runs before the GPU is touched."""
    import multiprocessing as mp
    from oracle import cpu_ref as CR
    from oracle import gpdla_oracle as O
    hc = host_cores()
    threads = hc["usable"]
    # configs[0]: one spectrum, null-model log_mvnpdf_low_rank (process_qsos.m:150-152)
    s0 = spectra[0]
    p0 = O.prepare_spectrum(s0["wavelengths"], s0["flux"], s0["noise_variance"], s0["pixel_mask"], s0["z_qso"], model)
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        ll0 = CR.log_mvnpdf_low_rank(p0["y"], p0["mu"], p0["M"], p0["omega2"] + p0["noise"])
    c1_us = (time.perf_counter() - t0) / reps * 1e6
    # the bench workload: whole spectra until the budget is spent (>= 16)
    off, nhi = samples["offset_samples"], samples["nhi_samples"]
    done = nspec = 0
    t0 = time.perf_counter()
    for q in range(len(spectra)):
        sp = spectra[q]
        prep = O.prepare_spectrum(sp["wavelengths"], sp["flux"], sp["noise_variance"], sp["pixel_mask"],
                                  sp["z_qso"], model)
        out = CR.sample_lls(prep, off, nhi, 3, threads)
        assert np.all(np.isfinite(out))
        done += out.size
        nspec += 1
        if nspec >= 16 and time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    # secondary: the numpy restatement, one process, one BLAS thread, 3 s
    with mp.get_context("spawn").Pool(1) as pool:
        nd, nel = pool.map(_numpy_worker, [(model, spectra[0], off, nhi, 3.0)])[0]
    wide = widened_cpu_baseline() if widened else None
    return {"value": done / el, "unit": "evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} (spectrum, DLA-sample) evaluations = {nspec} whole spectra x {off.size} samples of the "
                      f"bench workload in {el:.1f} s; C++ OpenMP restatement of process_qsos.m:184-198 "
                      f"(oracle/cpu_ref.cpp, MATLAB operation order, {threads} OpenMP threads = every core granted: "
                      f"affinity {hc['affinity']}, cgroup quota {hc['cgroup_quota_cpus']}, nproc {hc['nproc']}); "
                      f"MATLAB is not available; n=800, k={k}, 3 lines",
            "host": hc,
            "configs0_null_eval_us": c1_us, "configs0_log_likelihood_no_dla": ll0,
            "numpy_1core": {"value": nd / nel, "unit": "evals/s", "cores": 1,
                            "sample": f"{nd} evaluations of spectrum 0 in {nel:.1f} s (oracle/gpdla_oracle.py)"},
            "widened": wide}


def widened_cpu_baseline() -> dict:
    """The numpy restatements of the widened rows, beside alternatives.dla_samples, .ingest and .objective:
    generate_dla_samples at 10^5 samples (oracle/dla_samples_closed_form.py), preload_qsos over 1,024 of
    the ingest leg's BOSS coadds (oracle/ingest_oracle.py), the training objective over 200 spectra."""
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=1):                 # one core, BLAS included
        return _widened_cpu_baseline()


def _widened_cpu_baseline() -> dict:
    from oracle import dla_samples_closed_form as DC
    from oracle import ingest_oracle as IO
    ln = widened_catalogue()
    t0 = time.perf_counter()
    DC.generate_dla_samples(ln, WIDENED_SAMPLES)
    el_s = time.perf_counter() - t0
    zp, pool = boss_pool(1024)
    t0 = time.perf_counter()
    IO.preload_from_columns(zp, np.zeros(zp.size, np.uint8), pool)
    el_p = time.perf_counter() - t0
    npx = sum(c[0].size for c in pool)
    from oracle import gpdla_oracle as GO
    y, lya, nv, x = objective_problem(Q=200)
    GO.objective(x, y[:8], lya[:8], nv[:8])           # warm-up (first-call set-up)
    t0 = time.perf_counter()
    GO.objective(x, y, lya, nv)
    el_o = time.perf_counter() - t0
    return {"objective": {"value": y.shape[0] / el_o, "unit": "spectra/s", "cores": 1, "kind": "port",
                          "sample": f"objective.m f + gradient over 200 spectra of the 5,000-spectrum problem's shape in "
                                    f"{el_o:.2f} s (numpy restatement, oracle/gpdla_oracle.py, one BLAS "
                                    "thread)"},
            "generate_dla_samples": {"value": WIDENED_SAMPLES / el_s, "unit": "samples/s", "cores": 1, "kind": "port",
                                     "sample": f"{WIDENED_SAMPLES} samples in {el_s:.2f} s (numpy/scipy restatement)"},
            "preload_qsos": {"value": npx / el_p, "unit": "pixels/s", "cores": 1, "kind": "port",
                             "sample": f"1,024 synthetic BOSS coadds ({npx:,} pixels) in {el_p:.2f} s "
                                       "(numpy restatement, columns already in memory)"}}


# BASELINE.json configs.  c2 is the bench line the driver records.
WORKLOADS = {
    "c2": dict(spectra=1024, samples=10000, k=20, dr12q=False, scaling="weak",
               label="configs[1]: 1024 synthetic spectra/GPU x 10^4 DLA samples, k=20, fp64"),
    "c3": dict(spectra=162861, samples=10000, k=20, dr12q=True, scaling="weak",
               label="configs[2]: full DR12Q count (162,861 DR12Q-shaped spectra) x 10^4 samples, k=20, fp64, 1 GPU"),
    "c4": dict(spectra=162861, samples=10000, k=20, dr12q=True, scaling="strong",
               label="configs[3]: full DR12Q count split over the ranks (spectrum shards), k=20, fp64"),
    "c5": dict(spectra=128, samples=100000, k=50, dr12q=False, scaling="weak", default_path="panel_gemm_i8_24",
               label="configs[4]: 128 spectra/GPU x 10^5 DLA samples, k=50 (quoted in fp32; run on the int8 "
                     "panel-GEMM path with the 24-bit Gram contraction and fp32 raw profiles, ~2.5e-7 from fp64; --path panel_gemm_i8 "
                     "for the 32-bit one, ~4e-9; --path panel_gemm for the fp64 GEMMs)"),
}


def run_e2e(args, world: int, rank: int, local_rank: int, dist) -> None:
    """--workload e2e: e2e_record's line on rank 0."""
    from gp_dla_detection_amd import _lib as L
    dev, err = assign_device(world, local_rank, L.load().gpdla_device_count(), args.rehearsal)
    if err:
        refuse(err, rank)
    rec = e2e_record(args.spectra or 162861, args.samples or 10000, args.k or 20, args.e2e_dir, args.e2e_keep,
                     world, rank, dist, dev)
    if rank == 0:
        if world > 1 and args.rehearsal and rec["e2e"]["devices_used"] < world:
            rec["rehearsal"] = {"value_if_counted": rec["value"], "note": "ranks shared GPUs: not an N-GPU point"}
            rec["value"] = None
        print(json.dumps(rec), flush=True)


def e2e_record(Q: int, S: int, k: int, e2e_dir, keep: bool, world: int, rank: int, dist, dev: int):
    """configs[2] end to end: the whole process_qsos script on files --
    catalog.mat, learned_qso_model_*.mat, dla_samples.mat and preloaded_qsos.mat in (written
    beforehand, untimed, as the reference's processed/ tree of 162,861 DR12Q-shaped spectra),
    processed_qsos_<set>.mat (v7.3, with the 13 GB Q x S sample array) out.  The timed region is
    process.run_process_qsos from its first file read to the last byte of the output file (no
    warm-up: a cold engine is part of the run); the load / compute / write split is reported per
    phase (max over ranks).  With N ranks each decodes, evaluates and writes its own spectra."""
    import shutil
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import process as PR
    from gp_dla_detection_amd import synthetic as syn
    base = e2e_dir or f"/tmp/gpdla_e2e_{Q}_{S}"
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    t0 = time.perf_counter()
    if rank == 0:
        pool = syn.make_dr12q_like_spectra(model, 4096, seed=12, mask_fraction=0.0)
        names = syn.write_processed_tree(base, model, samples, [pool[i % len(pool)] for i in range(Q)])
        del pool
    setup_s = time.perf_counter() - t0
    print(f"[e2e rank {rank}] processed/ tree ready in {setup_s:.1f} s", file=sys.stderr, flush=True)
    if dist is not None:
        box = [names if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        names = box[0]
        dist.barrier()
    tm = {}
    t0 = time.perf_counter()
    PR.run_process_qsos(base, names["training_release"], names["training_set_name"], names["dla_catalog_name"],
                        names["prior_ind"], names["release"], names["test_set_name"], names["test_ind"],
                        device=dev, rank=rank, world=world, timings=tm)
    if dist is not None:
        dist.barrier()
    total = time.perf_counter() - t0
    print(f"[e2e rank {rank}] run_process_qsos {total:.1f} s {tm}", file=sys.stderr, flush=True)
    phases = [tm.get("load_s", 0.0), tm.get("compute_s", 0.0), tm.get("write_s", 0.0), total]
    if dist is not None:
        import torch
        tt = torch.tensor(phases, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        phases = [float(v) for v in tt]
    load_s, compute_s, write_s, total = phases
    out_path = f"{base}/{names['release']}/processed/processed_qsos_{names['test_set_name']}.mat"
    if rank == 0:
        out_bytes = os.path.getsize(out_path)
        evals = Q * S
        # 8-GPU projection: decoding scales with ranks (load_s * world / 8), the engine's work splits
        # over the GPUs (compute_s covers the work of all `world` ranks on the devices they used:
        # ranks sharing one leased GPU each wait for the whole job), the write as measured
        ndev = max(1, min(world, L.load().gpdla_device_count()))
        proj8 = load_s * world / 8 + compute_s * ndev / 8
        rec = {
            "metric": "(spectrum x DLA-sample) log-evidence evals/sec", "value": evals / total, "unit": "evals/s",
            "n_gpus": world, "steps": 1, "warmup": 0, "ms_per_step": total * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded; DR12Q-shaped pool of 4096 spectra tiled to the count), written as the "
                    "reference's processed/ tree before the timed region",
            "config": {"workload": f"configs[2] end to end: process_qsos on files, {Q} spectra x {S} samples, k={k}, "
                                   f"fp64 -> processed_qsos v7.3 ({out_bytes / 1e9:.1f} GB)",
                       "spectra": Q, "num_samples": S, "parallelism": f"spectrum-shard x{world}"},
            "e2e": {"total_s": total, "load_s": load_s, "compute_s": compute_s, "write_s": write_s,
                    "compute_split_rank0": {k: tm[k] for k in ("engine_create_s", "host_alloc_s", "engine_process_s")
                                            if k in tm},
                    "setup_untimed_s": setup_s, "output_bytes": out_bytes, "output_dir": base,
                    "projection_8_gpus_ideal_s": {
                        "value": proj8 + write_s, "devices_used": ndev,
                        "note": "ideal-scaling estimate, not a measurement: load x world/8 + compute x "
                                "devices_used/8 (linear speed-up from the devices used to 8 assumed) + write "
                                "as measured"},
                    "devices_used": ndev,
                    "note": "load = catalogues, model, samples and this rank's preloaded_qsos cells "
                            "(process_qsos.m:1-63); compute = the engine incl. its creation (:88-212); "
                            "write = priors/posteriors and the v7.3 file (:222-249), page cache, no fsync"}}
        if not keep:
            shutil.rmtree(base, ignore_errors=True)
        return rec
    return None


# rocprofv3 summaries of the bench workloads (tools/profile.sh + tools/summarize_profile.py), committed
PROFILE_SUMMARY = ROOT / "profiles" / "round5" / "r10k_c2_summary.json"   # configs[1], fused fp64 (round-5 tree)
# configs[4] (128 spectra x 10^5 samples, k = 50): the summary file and the EXACT names of the roofline
# kernel's launches (the GEMM launches of one spectrum and sample chunk; per-batch conversion kernels
# such as convert_gemm_i8_kernel are not part of it).  The int8 paths' summaries are one-stream runs
# (--panel-streams 1), whose kernel durations are the roofline's one-stream launch time; the trace of
# the two-stream timed configuration is profiles/round5/r11c_c5_summary.md (PMC bytes per dispatch
# are the same: the counter passes serialise the kernels)
PROFILE_SUMMARY_C5 = {
    # the 32-bit path's Gram + u launch is gemm_i8_kernel<4>
    "panel-GEMM-int8": (ROOT / "profiles" / "round5" / "r11d_c5i8s1_summary.json",
                        ("void gpdla::gemm_i8_kernel<4>(gpdla::GemmI8Args)",)),
    # the 24-bit path: Gram and u contractions in one B-stationary launch (round 5)
    "panel-GEMM-int8-24": (ROOT / "profiles" / "round5" / "r11d_c5s1_summary.json",
                           ("gpdla::gemm_i8_bst_kernel(gpdla::GemmI8Args)",)),
    "panel-GEMM": (ROOT / "profiles" / "r5f_c5f64_summary.json", ("gpdla::gemm_f64_kernel(gpdla::GemmF64Args)",)),
}
# the roofline kernel's label per path
ROOFLINE_KERNEL = {"fused": "likelihood_kernel<{k}>", "fused-int8": "likelihood_i8_kernel<{k}>",
                   "panel-GEMM-int8": "gemm_i8_kernel (Gram + u)",
                   "panel-GEMM-int8-24": "gemm_i8_bst_kernel (Gram + u contractions in one launch)",
                   "panel-GEMM": "gemm_f64_kernel (Gram + u)"}


def profiled_traffic(Q: int, S: int, k: int, path: str = "fused"):
    """HBM bytes per launch of the roofline kernel from the committed PMC profile of the workload
    (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction per MI355X_MICROARCH.md; includes Infinity-Cache
    hits): the fused kernel for configs[1]; for configs[4] the GEMM launches of one spectrum and
    sample chunk (the Gram and u launches of the 24-bit path together), matched by exact kernel
    name.  None for other workloads or if no summary is present."""
    if (Q, S, k) == (128, 100000, 50) and path in PROFILE_SUMMARY_C5 and PROFILE_SUMMARY_C5[path][0].exists():
        f, names = PROFILE_SUMMARY_C5[path]
        d = json.loads(f.read_text())
        rows = [e for e in d["kernels"] if e["kernel"] in names and "hbm_bytes_per_launch" in e]
        if len(rows) == len(names):
            return (sum(e["hbm_bytes_per_launch"] for e in rows),
                    f"{f.relative_to(ROOT)} (rocprofv3 PMC: {' + '.join(e['kernel'] for e in rows)})")
        return None, None
    if (Q, S, k) != (1024, 10000, 20) or path != "fused" or not PROFILE_SUMMARY.exists():
        return None, None
    d = json.loads(PROFILE_SUMMARY.read_text())
    for ent in d["kernels"]:
        if ent["kernel"].startswith("void gpdla::likelihood_kernel<20") and "hbm_bytes_per_launch" in ent:
            return ent["hbm_bytes_per_launch"], f"{PROFILE_SUMMARY.relative_to(ROOT)} (rocprofv3 PMC)"
    return None, None


E2E_DISK_BYTES = 48e9   # alternatives.e2e: the 13 GB output, the ~5 GB processed/ tree, and headroom


def dram_record(traffic, ms, src, path: str) -> dict:
    """The roofline kernel's DRAM side, recomputable from the committed profile: its PMC bytes per
    launch (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md) over its measured launch time, as a
    fraction of the 8 TB/s HBM peak."""
    note = ("configs[1]'s fused kernel is FP64-pipe-bound (roofline.bound): the north star's >= 40% "
            "HBM-roofline target is not a statement about this kernel, whose DRAM use is this small fraction"
            if path in ("fused", "fused-int8") else
            "the roofline kernel's PMC bytes per launch over its HIP-event launch time")
    if traffic is None or not ms:
        return {"bytes_per_launch": None, "gbs": None, "frac": None, "peak": HBM_PEAK_GBS,
                "note": "no committed PMC profile for this workload and path"}
    gbs = traffic / (ms * 1e-3) / 1e9
    return {"bytes_per_launch": traffic, "gbs": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "source": src, "note": note}


def chain_dram(path: str) -> dict | None:
    """configs[4]'s whole kernel chain from its committed profile: every kernel's PMC HBM bytes over
    every kernel's time, per engine batch (tools/summarize_profile.py per_batch)."""
    if path not in PROFILE_SUMMARY_C5 or not PROFILE_SUMMARY_C5[path][0].exists():
        return None
    f = PROFILE_SUMMARY_C5[path][0]
    pb = json.loads(f.read_text()).get("per_batch")
    if not pb:
        return None
    gbs = pb["hbm_bytes_per_batch"] / (pb["kernel_ms_per_batch"] * 1e-3) / 1e9
    return {"bytes_per_batch": pb["hbm_bytes_per_batch"], "kernel_ms_per_batch": pb["kernel_ms_per_batch"],
            "gbs": gbs, "peak": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS, "source": str(f.relative_to(ROOT)),
            "note": "all kernels of the chain (weights, Gram and u GEMMs, LDL^T, per-batch prep/convert/reduce)"}


def timed_steps(step, synchronize, steps: int, dist=None, local: list | None = None) -> float:
    """The bench contract's timed region: barrier + device sync on both sides of exactly ``steps``
    steps, elapsed time max-reduced over the ranks (gloo, host-side).  ``local`` (if given) receives
    this rank's own elapsed time."""
    synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    synchronize()  # device-side completion of every enqueued step
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if local is not None:
        local.append(elapsed)
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


def dr12q_shard_ids(pool_pixels, total: int, rank: int, world: int, split: bool = True) -> np.ndarray:
    """Spectrum ids (0..total-1, ascending) of this rank's share of the DR12Q-shaped workload, where
    spectrum i is pool entry i % len(pool).  configs[2] (``split`` False) keeps all on one GPU;
    configs[3] splits them by LPT on pixel count (shard.py), so ranks get equal sweep work although
    n ranges over 270..1,250."""
    from gp_dla_detection_amd.shard import lpt_shards
    if not split or world == 1:
        return np.arange(total)
    idx = np.arange(total) % len(pool_pixels)
    return lpt_shards(np.asarray(pool_pixels, dtype=np.float64)[idx], world)[rank]


def dr12q_shard(pool_pixels, total: int, rank: int, world: int, split: bool):
    """Pool indices of this rank's DR12Q-shaped spectra (dr12q_shard_ids modulo the pool size)."""
    return dr12q_shard_ids(pool_pixels, total, rank, world, split) % len(pool_pixels)


class _stdout_to_stderr:
    """Route fd 1 to fd 2 for a block, so native libraries' prints cannot interleave with the
    one JSON line rank 0 writes to stdout."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def launch_ranks(n: int, argv: list) -> int:
    """``python bench.py --gpus N`` (N > 1) outside a launcher: start the N ranks -- one process per
    GPU -- as children through torch.distributed.run (rendezvous on 127.0.0.1), before this process
    has made any GPU call and without exec; forward their logs to stderr, print rank 0's JSON line,
    and return non-zero if any rank fails.  The ranks split process_qsos.m:88's spectrum loop."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), *argv]
    print("[bench] launching " + " ".join(cmd), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    result = None
    for line in proc.stdout:
        if line.lstrip().startswith("{") and '"n_gpus"' in line:
            result = line.strip()
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"[bench] a rank failed (torch.distributed.run exit status {rc})", file=sys.stderr, flush=True)
        return rc
    if result is None:
        print("[bench] rank 0 printed no JSON line", file=sys.stderr, flush=True)
        return 1
    print(result, flush=True)
    return 0


def rank_spectrum_ids(wl: dict, rank: int, world: int, pool_pixels=None) -> np.ndarray:
    """Ids of this rank's spectra.  configs[1]/[4]: synthetic spectrum seeds rank*Q .. rank*Q+Q-1 (Q per
    GPU, weak scaling, disjoint); configs[3]: the LPT share of DR12Q positions 0..162,860
    (dr12q_shard_ids, disjoint); configs[2]: all positions on every rank (one-GPU config)."""
    if wl["dr12q"]:
        return dr12q_shard_ids(pool_pixels, wl["spectra"], rank, world, split=wl["scaling"] == "strong")
    return rank * wl["spectra"] + np.arange(wl["spectra"])


def dr12q_pool(model):
    """The 4096 DR12Q-shaped spectra configs[2]/[3] tile to the full count."""
    from gp_dla_detection_amd import synthetic as syn
    return syn.make_dr12q_like_spectra(model, 4096, seed=12, mask_fraction=0.0)


def gather(obj, world: int, dist):
    """Every rank's ``obj`` on every rank (gloo; host-side bookkeeping, not the data path)."""
    if dist is None or world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


REFUSAL_EXIT = 3


def assign_device(world: int, local_rank: int, ndev: int, rehearsal: bool):
    """(device, error): one GPU per rank, ``local_rank`` -> device ``local_rank``.  With fewer devices
    than ranks the ranks would share GPUs and an N-rank line would not be an N-GPU point: that is
    refused (error set) unless ``rehearsal``, where ranks share devices round-robin."""
    if ndev < 1:
        return None, "no HIP device"
    if world > ndev and not rehearsal:
        return None, (f"{world} ranks but only {ndev} device(s): ranks would share GPUs, so the line would "
                      f"not be a {world}-GPU measurement; refusing (pass --rehearsal to run anyway: value null)")
    return local_rank % ndev, None


def refuse(msg: str, rank: int) -> None:
    print(f"bench.py (rank {rank}): {msg}", file=sys.stderr, flush=True)
    sys.exit(REFUSAL_EXIT)


def plan_only(wl: dict, world: int, rank: int, local_rank: int, dist, ndev: int | None = None,
              rehearsal: bool = False, alternatives: bool = False) -> None:
    """--plan-only: the multi-rank layout (which spectra each rank evaluates and on which device)
    through the same launcher and process group as a measured run, without any GPU call.  ``ndev``
    is the device count planned against (default one per rank); the device-sharing refusal of a
    measured run applies.  With ``alternatives`` (a multi-rank configs[1] line) it also plans the
    alternatives that line would measure: configs[3]'s LPT shards of the full DR12Q count and the
    configs[2] end-to-end run with every rank writing its own chunks."""
    dev, err = assign_device(world, local_rank, world if ndev is None else ndev, rehearsal)
    if err:
        refuse(err, rank)
    from gp_dla_detection_amd import synthetic as syn
    pool_pixels = None
    if wl["dr12q"] or alternatives:
        pool_pixels = [p["wavelengths"].size for p in dr12q_pool(syn.make_model(k=20 if alternatives else wl["k"]))]
    ids = rank_spectrum_ids(wl, rank, world, pool_pixels)
    mine = {"rank": rank, "local_rank": local_rank, "device": dev, "ids": ids}
    if alternatives:
        c4 = WORKLOADS["c4"]
        c3ids = dr12q_shard_ids(pool_pixels, c4["spectra"], rank, world, split=True)
        mine["c3"] = {"spectra": int(c3ids.size),
                      "pixels": int(np.sum(np.asarray(pool_pixels)[c3ids % len(pool_pixels)]))}
    allr = gather(mine, world, dist)
    if rank == 0:
        cat = np.concatenate([r["ids"] for r in allr])
        out = {
            "plan_only": True, "n_gpus": world, "rehearsal": bool(rehearsal and len({r["device"] for r in allr}) < world),
            "distinct_devices": len({r["device"] for r in allr}),
            "world_size": dist.get_world_size() if dist is not None else 1,
            "workload": wl["label"],
            "ranks": [{"rank": r["rank"], "local_rank": r["local_rank"], "device": r["device"],
                       "spectra": int(r["ids"].size), "first_spectrum": int(r["ids"][0]),
                       "last_spectrum": int(r["ids"][-1])} for r in allr],
            "disjoint": bool(np.unique(cat).size == cat.size), "total_spectra": int(cat.size)}
        if alternatives:
            px = np.array([r["c3"]["pixels"] for r in allr], dtype=np.float64)
            out["alternatives_planned"] = {
                "configs3": {"workload": WORKLOADS["c4"]["label"], "scaling": "strong",
                             "ranks": [{"rank": r["rank"], **r["c3"]} for r in allr],
                             "total_spectra": int(sum(r["c3"]["spectra"] for r in allr)),
                             "pixels_max_over_mean": float(px.max() / px.mean()),
                             "fields": ["value", "wall_s", "north_star_under_60s", "ranks", "imbalance",
                                        "invariant_calc_cddf_246", "checks_ok"]},
                "e2e": {"workload": "configs[2] end to end on files", "writers": world,
                        "note": "rank 0 writes the processed/ tree (untimed); every rank decodes, evaluates and "
                                "writes its LPT block shard of whole v7.3 chunks (process.run_process_qsos)",
                        "fields": ["value", "ms_per_step", "e2e.total_s", "e2e.load_s", "e2e.compute_s",
                                   "e2e.write_s", "e2e.devices_used"]}}
        print(json.dumps(out), flush=True)


# SURVEY 8f-2 / 8f-4 (the widened rows) beside the headline: synthetic inputs of the reference's shape
WIDENED_SAMPLES = 100_000                   # generate_dla_samples at configs[4]'s sample count
DR12Q_COUNT, BOSS_POOL, INGEST_BATCH = 162_861, 4_096, 16_384
INGEST_PROFILE = ROOT / "profiles" / "round6" / "r12w_ingest.json"


def widened_catalogue() -> np.ndarray:
    """A DLA catalogue's log N_HI column (generate_dla_samples.m:25-30's input): 1,000 values."""
    rng = np.random.default_rng(5)
    return np.r_[rng.normal(20.55, 0.3, 800), rng.uniform(20.3, 21.8, 200)]


def boss_pool(npool: int, seed: int = 31):
    """fitsread columns of npool synthetic full BOSS coadds (3600-10400 A) at z in [2.15, 5.5]."""
    from gp_dla_detection_amd import synthetic as syn
    rng = np.random.default_rng(seed)
    zp = rng.uniform(2.15, 5.5, npool)
    return zp, [syn.make_boss_coadd_columns(rng, z) for z in zp]


OBJ_Q, OBJ_P, OBJ_K = 5_000, 1_217, 20   # a DR9-training-set-sized problem on the 1,217-pixel rest grid


def objective_problem(Q: int = OBJ_Q, P: int = OBJ_P, k: int = OBJ_K, seed: int = 3):
    """learn_qso_model.m's objective inputs, synthetic: centred fluxes with ~30% missing pixels, (1 +
    z_Lya) and noise per pixel, and a parameter vector [M; log omega; log c_0, log tau_0, log beta]."""
    rng = np.random.default_rng(seed)
    y = 0.3 * rng.standard_normal((Q, P))
    y[rng.uniform(size=y.shape) < 0.3] = np.nan
    lya = rng.uniform(2.5, 4.5, (Q, P))
    nv = rng.uniform(0.01, 0.1, (Q, P))
    x = np.concatenate([0.05 * rng.standard_normal(P * k), np.log(0.15) + 0.1 * rng.standard_normal(P),
                        [np.log(0.1), np.log(0.0023), np.log(3.65)]])
    return y, lya, nv, x


def objective_flops(y, k: int) -> float:
    """Algorithmic flops of objective.m's f + g (spectrum_loss.m:23-74 over every spectrum) as the
    Woodbury form computes them: per valid pixel the Gram k(k+1), M'D^-1 y / M C y / (K^-1 y)'M 6k, the
    u = M_i B^-1 rows 2k^2, diag K^-1 2k, dM 3k; per spectrum k^3 for B^-1."""
    n = np.sum(~np.isnan(y), axis=1).astype(np.float64)
    return float(np.sum(n * (3 * k * k + 12 * k) + k ** 3))


def objective_alternative(dev: int, reps: int = 10) -> dict:
    """objective.m's f and gradient (spectrum_loss.m summed over the training set in a
    fixed order: the Gram and dM sums as pixel x spectrum GEMMs, the rest in spectrum chunks) on the device for a DR9-training-set-sized problem (5,000 spectra x 1,217 rest
    pixels, k = 20): one warm-up evaluation, then ``reps`` timed ones; kernel times from a one-launch
    evaluation under HIP events are not exposed, so the roofline is over the evaluation's wall time."""
    from gp_dla_detection_amd import training as T
    y, lya, nv, x = objective_problem()
    with T.Objective(y, lya, nv, OBJ_K, device=dev) as obj:
        f0, g0 = obj(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            f, g = obj(x)
        el = (time.perf_counter() - t0) / reps
    flops = objective_flops(y, OBJ_K)
    ok = bool(np.isfinite(f) and np.all(np.isfinite(g)) and f == f0 and np.array_equal(g, g0))
    return {"value": OBJ_Q / el, "unit": "spectra/s", "ms_per_step": el * 1e3, "steps": reps,
            "config": {"workload": "objective.m f + gradient, 5,000 synthetic training spectra x 1,217 rest pixels "
                                   "(~30% missing), k = 20 (SURVEY 8f-3)"},
            "roofline": {"bound": "fp64", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
                         "achieved": flops / el / 1e12, "frac": flops / el / 1e12 / FP64_PEAK_TFLOPS,
                         "flops": flops, "note": "algorithmic flops (objective_flops) over the whole evaluation "
                                                 "(pixel, Gram / g / dM GEMM and spectrum kernels, the sums, copies)"},
            "checks_ok": ok, "repeat_bitwise_equal": ok}


def dla_samples_alternative(dev: int, reps: int = 5) -> dict:
    """generate_dla_samples.m:8-57 on the device at 10^5 samples (RR2 Halton, the KDE on
    the fit grid, the per-sample inverse CDF; gpdla_generate_dla_samples_f64, host buffers in and
    out).  One warm-up call, then ``reps`` timed calls; kernel times from HIP events in the library."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import dla_samples as DS
    ln = widened_catalogue()
    DS.generate_dla_samples(ln, WIDENED_SAMPLES, device=dev)
    kms = np.zeros(3)
    t0 = time.perf_counter()
    for _ in range(reps):
        out = DS.generate_dla_samples(ln, WIDENED_SAMPLES, device=dev)
        kms += np.array(L.last_call_kernel_ms()[:3])
    el = (time.perf_counter() - t0) / reps
    kms /= reps
    off, lnhi, nhi = out["offset_samples"], out["log_nhi_samples"], out["nhi_samples"]
    ok = bool(np.all((off >= 0) & (off <= 1)) and np.all((lnhi >= 20) & (lnhi <= 23))
              and np.all(np.isfinite(nhi)) and np.allclose(nhi, 10.0 ** lnhi, rtol=1e-15, atol=0))
    return {"value": WIDENED_SAMPLES / el, "unit": "samples/s", "ms_per_step": el * 1e3, "steps": reps,
            "config": {"workload": "generate_dla_samples.m at 10^5 samples over a 1,000-value synthetic log N_HI "
                                   "catalogue (SURVEY 8f-2); host buffers in and out"},
            "kernel_ms": {"kde": kms[0], "halton_rr2": kms[1], "inverse_cdf": kms[2]},
            "note": "the call is launch- and copy-bound (three small kernels); the inverse CDF is one "
                    "bracketed-Newton solve per sample in fp64",
            "checks_ok": ok}


def ingest_alternative(dev: int) -> dict:
    """preload_qsos.m:18-67 (with read_spec.m:27-38) on the device over the DR12Q count --
    162,861 catalogue entries, full BOSS coadds (a pool of 4,096 distinct synthetic ones, tiled) -- in
    16,384-spectrum batches through gpdla_preload_qsos_f32.  The boundary takes host buffers (FITS is
    parsed on the host), so ``value`` (input pixels/s) includes the CSR packing, PCIe copies and the
    splitting into cells; ``roofline`` is the scan and write kernels' algorithmic bytes (12 B per
    input pixel, 29 B per selected one) over their HIP-event times."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import ingest as I
    t0 = time.perf_counter()
    zp, pool = boss_pool(BOSS_POOL)
    setup_s = time.perf_counter() - t0
    sel = np.arange(DR12Q_COUNT) % BOSS_POOL
    flags = np.zeros(DR12Q_COUNT, np.uint8)
    I.preload_batch(zp[:256], flags[:256], [pool[i] for i in range(256)], device=dev)   # warm-up
    kms = np.zeros(3)
    npx = nsel = 0
    ff = []
    ok = True
    t0 = time.perf_counter()
    for b0 in range(0, DR12Q_COUNT, INGEST_BATCH):
        idx = sel[b0:b0 + INGEST_BATCH]
        cols = [pool[i] for i in idx]
        r = I.preload_batch(zp[idx], flags[b0:b0 + INGEST_BATCH], cols, device=dev)
        kms += np.array(L.last_call_kernel_ms()[:3])
        npx += sum(c[0].size for c in cols)
        nsel += sum(c.size for c in r["all_wavelengths"])
        ff.append(r["filter_flags"])
        good = r["filter_flags"] == 0
        ok = ok and bool(np.all(np.isfinite(r["all_normalizers"][good])))
    el = time.perf_counter() - t0
    ff = np.concatenate(ff)
    alg = {"scan": 12.0 * npx, "write": 29.0 * nsel}
    per = {k: {"ms": kms[i], "algorithmic_bytes": alg[k], "gbs": alg[k] / (kms[i] * 1e-3) / 1e9,
               "frac": alg[k] / (kms[i] * 1e-3) / 1e9 / HBM_PEAK_GBS} for i, k in ((1, "scan"), (2, "write"))}
    both = (alg["scan"] + alg["write"]) / ((kms[1] + kms[2]) * 1e-3) / 1e9
    traffic = None
    if INGEST_PROFILE.exists():   # PMC bytes of the same workload (tools/profile_ingest.sh)
        kp = json.loads(INGEST_PROFILE.read_text())["kernels"]
        traffic = sum(kp[k]["pmc_bytes"] for k in ("preload_scan_kernel", "preload_write_kernel"))
    return {"value": npx / el, "unit": "pixels/s", "wall_s": el, "ms_per_step": el * 1e3, "steps": 1,
            "warmup": "one call on 256 spectra",
            "config": {"workload": "preload_qsos.m's numeric stage over the DR12Q count (162,861 entries, full "
                                   "3600-10400 A BOSS coadds: a pool of 4,096 distinct synthetic ones tiled), "
                                   "16,384 spectra per call (SURVEY 8f-4)",
                       "spectra": DR12Q_COUNT, "pixels_in": int(npx), "pixels_selected": int(nsel)},
            "kernel_ms": {"keys_total": kms[0], "scan_total": kms[1], "write_total": kms[2]},
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "achieved": both,
                         "frac": both / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": f"{INGEST_PROFILE.relative_to(ROOT)}: FETCH_SIZE x2 + WRITE_SIZE of both "
                                           "kernels over the same workload (incl. one 256-spectrum warm-up launch), "
                                           f"against {alg['scan'] + alg['write']:.3e} algorithmic bytes"
                                           if traffic else None,
                         "kernel": "preload_scan_kernel + preload_write_kernel (all launches)", "per_kernel": per,
                         "note": "algorithmic bytes: 12 B per input pixel (scan: loglam, ivar, and_mask), 29 B per "
                                 "selected pixel (write: 16 B in, 13 B out)"},
            "value_note": "host buffers in and out: CSR packing, PCIe copies and cell splitting included",
            "filter_flags": {str(int(v)): int(c) for v, c in zip(*np.unique(ff, return_counts=True))},
            "setup_untimed_s": setup_s, "checks_ok": ok}


def configs4_alternative(dev: int, steps: int) -> dict:
    """BASELINE configs[4] beside the headline: 128 spectra x 10^5 DLA samples, k = 50, on the
    panel_gemm_i8_24 path, ``steps`` timed steps on resident inputs after one warm-up step; its GEMM
    roofline (HIP events around the GEMM launches) with the committed PMC traffic of the same
    kernels, and its deviation from the fp64 panel path (gemm_f64) on the first 8 spectra
    (log_mvnpdf_low_rank.m:22-32, process_qsos.m:184-198)."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    wl = WORKLOADS["c5"]
    Q, S, k = wl["spectra"], wl["samples"], wl["k"]
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    spectra = [syn.make_spectrum(model, q) for q in range(Q)]
    packed = syn.pack_spectra(spectra)
    t = {key: L.DeviceArray.from_numpy(packed[key], device=dev)
         for key in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    o_null, o_dla = L.DeviceArray(dev, Q, np.float64), L.DeviceArray(dev, Q, np.float64)
    o_s, o_n = L.DeviceArray(dev, (Q, S), np.float64), L.DeviceArray(dev, Q, np.int32)
    with Engine(model, samples, set_parameters(k=k), device=dev, path="panel_gemm_i8_24") as eng:
        def step():
            eng.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                               t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, S,
                               npix_ptr=o_n.ptr)
        step()
        eng.synchronize()
        eng.reset_stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        eng.synchronize()
        el = time.perf_counter() - t0
        st = eng.stats()
        n_mean = float(np.mean(o_n.numpy()))
        alone = i8_roofline(single_stream_stats(eng, step), n_mean, k, Q, S, 2, "panel-GEMM-int8-24")
    sub = 8
    with Engine(model, samples, set_parameters(k=k), device=dev, path="panel_gemm") as e64:
        ref = e64.process(syn.pack_spectra(spectra[:sub]))
    rel = lambda got, want: float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)))
    sll = o_s.numpy(rows=sub)
    lld, lln = o_dla.numpy(), o_null.numpy()
    errs = {"sample_log_likelihoods_dla": rel(sll, ref["sample_log_likelihoods_dla"]),
            "log_likelihoods_dla": rel(lld[:sub], ref["log_likelihoods_dla"]),
            "log_likelihoods_no_dla": rel(lln[:sub], ref["log_likelihoods_no_dla"])}
    inv = np.exp(sll - (lld[:sub, None] + np.log(S))).sum(axis=1)
    path = "panel-GEMM-int8-24"
    roof = panel_roofline_streams(i8_roofline(st, n_mean, k, Q, S, steps, path), alone)
    traffic, src = profiled_traffic(Q, S, k, path)
    roof.update({"kernel": ROOFLINE_KERNEL[path], "traffic": traffic, "traffic_source": src})
    # PMC bytes are per dispatch (the counter passes serialise kernels): over the kernel's own time
    dram = dram_record(traffic, roof["avg_launch_ms"], src, path)
    dram["chain"] = chain_dram(path)
    for a in (*t.values(), o_null, o_dla, o_s, o_n):
        a.free()
    return {"value": Q * S * steps / el, "unit": "evals/s", "ms_per_step": el / steps * 1e3, "steps": steps,
            "warmup": 1,
            "config": {"workload": wl["label"], "spectra": Q, "num_samples": S, "k": k, "n_pixels": n_mean,
                       "likelihood_path": path},
            "kernel_ms": {"prep": st["prep_ms"] / max(st["prep_launches"], 1),
                          "gemm_per_chunk": st["contraction_ms"] / max(st["contraction_launches"], 1),
                          "batch": st["likelihood_ms"] / max(st["likelihood_launches"], 1),
                          "reduce": st["reduce_ms"] / max(st["reduce_launches"], 1)},
            "roofline": roof, "dram": dram,
            "max_rel_err_vs_fp64_panel": errs, "parity_subset": f"first {sub} of {Q} spectra, all {S} samples",
            "checks_ok": bool(np.all(np.isfinite(sll)) and errs["sample_log_likelihoods_dla"] < 5e-7
                              and np.max(np.abs(inv - 1)) < 1e-10)}


def invariant_all_rows(o_s, o_dla, S: int, threads: int = 8, rows_per_task: int = 4096) -> dict:
    """The calc_cddf.py:246 invariant sum_s exp(l_s - l_DLA - log S) = 1 and finiteness on EVERY row of
    a device-resident Q x S sample array (D2H in row blocks on a thread pool; ctypes and numpy release
    the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    lld = o_dla.numpy()
    Q = lld.size

    def block(r0):
        sll = o_s.numpy(rows=rows_per_task, start=r0)
        inv = np.exp(sll - (lld[r0:r0 + sll.shape[0], None] + np.log(S))).sum(axis=1)
        return float(np.max(np.abs(inv - 1))), bool(np.all(np.isfinite(sll)))

    with ThreadPoolExecutor(max_workers=threads) as ex:
        res = list(ex.map(block, range(0, Q, rows_per_task)))
    return {"rows": int(Q), "max_abs_dev": max(r[0] for r in res),
            "finite": all(r[1] for r in res) and bool(np.all(np.isfinite(lld)))}


def configs2_alternative(dev: int) -> dict:
    """BASELINE configs[2] beside the headline (the north star's "full DR12Q"): 162,861 DR12Q-shaped
    spectra x 10^4 DLA samples, k = 20, fp64 fused path, all on this GPU, inputs resident and the 13 GB
    of sample log-likelihoods left in HBM.  One untimed warm-up call on the first 1,024 spectra, then
    ONE timed call over all of them (process_qsos.m:88-212 over the whole catalogue); the invariant
    calc_cddf.py:246 is checked on every spectrum afterwards."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    wl = WORKLOADS["c3"]
    Q, S, k = wl["spectra"], wl["samples"], wl["k"]
    t0 = time.perf_counter()
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    pool = dr12q_pool(model)
    packed = syn.pack_spectra([pool[i % len(pool)] for i in range(Q)])
    del pool
    t = {key: L.DeviceArray.from_numpy(packed[key], device=dev)
         for key in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    o_null, o_dla = L.DeviceArray(dev, Q, np.float64), L.DeviceArray(dev, Q, np.float64)
    o_s, o_n = L.DeviceArray(dev, (Q, S), np.float64), L.DeviceArray(dev, Q, np.int32)
    setup_s = time.perf_counter() - t0
    offs = packed["offsets"]
    with Engine(model, samples, set_parameters(k=k), device=dev) as eng:
        def call(off):
            eng.process_device(off, t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                               t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, S,
                               npix_ptr=o_n.ptr)
        call(offs[:1025])
        eng.synchronize()
        eng.reset_stats()
        t0 = time.perf_counter()
        call(offs)
        eng.synchronize()
        el = time.perf_counter() - t0
        st = eng.stats()
    t0 = time.perf_counter()
    inv = invariant_all_rows(o_s, o_dla, S)
    check_s = time.perf_counter() - t0
    npix = o_n.numpy()
    n_mean = float(np.mean(npix))
    lk_ms = st["likelihood_ms"]
    flops = float(np.sum(algorithmic_flops_per_eval(npix.astype(np.float64), k))) * (S + 1)
    for a in (*t.values(), o_null, o_dla, o_s, o_n):
        a.free()
    return {"value": Q * S / el, "unit": "evals/s", "wall_s": el, "ms_per_step": el * 1e3, "steps": 1,
            "warmup": "one call on the first 1,024 spectra",
            "north_star_under_60s": bool(el < 60.0),
            "config": {"workload": wl["label"] + "; inputs resident in HBM, outputs (13 GB) left in HBM",
                       "spectra": Q, "num_samples": S, "k": k, "n_pixels_mean": n_mean, "likelihood_path": "fused"},
            "kernel_ms": {"prep_total": st["prep_ms"], "likelihood_total": lk_ms, "reduce_total": st["reduce_ms"],
                          "likelihood_launches": st["likelihood_launches"]},
            "roofline": {"bound": "mfma", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
                         "achieved": flops / (lk_ms * 1e-3) / 1e12, "frac": flops / (lk_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                         "kernel": "likelihood_kernel<20> (all launches of the call)",
                         "flops": flops, "note": "SURVEY 8d F_eval summed over every spectrum's own n, incl. the "
                                                 "null model; over the summed HIP-event times of the likelihood launches"},
            "invariant_calc_cddf_246": inv, "invariant_check_s": check_s, "setup_untimed_s": setup_s,
            "checks_ok": bool(inv["finite"] and inv["max_abs_dev"] < 1e-10)}


def configs3_alternative(dev: int, world: int, rank: int, dist, rehearsal: bool) -> dict | None:
    """BASELINE configs[3] beside a multi-rank headline: the full DR12Q count
    (162,861 DR12Q-shaped spectra x 10^4 samples, k = 20, fp64 fused path) split over the ranks by LPT on
    pixel count (strong scaling, no collective on the data path; process_qsos.m:88's spectrum loop),
    inputs resident and each rank's share of the 13 GB of sample log-likelihoods left in its HBM.  One
    untimed warm-up call on each rank's first 1,024 spectra, then ONE timed call per rank between
    barriers (elapsed max-reduced over the ranks, as the headline).  Per rank: spectra, pixels, kernel
    ms and wall; the calc_cddf.py:246 invariant on every row of every rank.  Returns the record on rank
    0 (None elsewhere)."""
    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    wl = WORKLOADS["c4"]
    Qt, S, k = wl["spectra"], wl["samples"], wl["k"]
    t0 = time.perf_counter()
    model = syn.make_model(k=k)
    samples = syn.make_samples(S)
    pool = dr12q_pool(model)
    ids = dr12q_shard_ids([p["wavelengths"].size for p in pool], Qt, rank, world, split=True)
    packed = syn.pack_spectra([pool[i % len(pool)] for i in ids])
    del pool
    Q = ids.size
    t = {key: L.DeviceArray.from_numpy(packed[key], device=dev)
         for key in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    o_null, o_dla = L.DeviceArray(dev, Q, np.float64), L.DeviceArray(dev, Q, np.float64)
    o_s, o_n = L.DeviceArray(dev, (Q, S), np.float64), L.DeviceArray(dev, Q, np.int32)
    setup_s = time.perf_counter() - t0
    offs = packed["offsets"]
    local = []
    with Engine(model, samples, set_parameters(k=k), device=dev) as eng:
        def call(off):
            eng.process_device(off, t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                               t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, S,
                               npix_ptr=o_n.ptr)
        call(offs[:min(Q, 1024) + 1])
        eng.synchronize()
        eng.reset_stats()
        el = timed_steps(lambda: call(offs), eng.synchronize, 1, dist, local)
        st = eng.stats()
    t1 = time.perf_counter()
    inv = invariant_all_rows(o_s, o_dla, S)
    check_s = time.perf_counter() - t1
    npix = o_n.numpy()
    for a in (*t.values(), o_null, o_dla, o_s, o_n):
        a.free()
    mine = {"rank": rank, "device": dev, "pci_bus_id": L.pci_bus_id(dev), "spectra": int(Q),
            "pixels": int(np.sum(npix)), "kernel_ms": st["prep_ms"] + st["likelihood_ms"] + st["reduce_ms"],
            "likelihood_ms": st["likelihood_ms"], "wall_s": local[0], "setup_untimed_s": setup_s,
            "invariant_max_abs_dev": inv["max_abs_dev"], "finite": inv["finite"], "invariant_check_s": check_s}
    ranks = gather(mine, world, dist)
    if rank != 0:
        return None
    km = np.array([r["kernel_ms"] for r in ranks])
    wm = np.array([r["wall_s"] for r in ranks])
    px = np.array([r["pixels"] for r in ranks], dtype=np.float64)
    shared = len({r["pci_bus_id"] for r in ranks}) < world
    value = Qt * S / el
    ok = all(r["finite"] for r in ranks) and max(r["invariant_max_abs_dev"] for r in ranks) < 1e-10
    rec = {"value": None if shared else value, "unit": "evals/s", "wall_s": el, "ms_per_step": el * 1e3, "steps": 1,
           "warmup": "one call on each rank's first 1,024 spectra", "scaling": "strong", "n_gpus": world,
           "north_star_under_60s": bool(el < 60.0),
           "config": {"workload": wl["label"] + "; inputs resident in HBM, each rank's outputs left in its HBM",
                      "spectra": Qt, "num_samples": S, "k": k, "likelihood_path": "fused",
                      "parallelism": f"spectrum-shard x{world} (LPT on pixel count)"},
           "ranks": ranks,
           "imbalance": {"kernel_ms_max_over_mean": float(km.max() / km.mean()),
                         "wall_max_over_mean": float(wm.max() / wm.mean()),
                         "pixels_max_over_mean": float(px.max() / px.mean())},
           "invariant_calc_cddf_246": {"rows": int(sum(r["spectra"] for r in ranks)),
                                       "max_abs_dev": max(r["invariant_max_abs_dev"] for r in ranks),
                                       "finite": all(r["finite"] for r in ranks)},
           "checks_ok": bool(ok)}
    if shared:
        rec["rehearsal"] = {"value_if_counted": value, "note": f"ranks shared {len({r['pci_bus_id'] for r in ranks})} "
                                                               f"GPU(s): not a {world}-GPU point"}
    return rec


def e2e_alternative(args, world: int, rank: int, dist, dev: int) -> dict | None:
    """alternatives.e2e: configs[2] end to end on files (e2e_record), at world = N each rank decoding,
    computing and writing its own chunks; skipped (on every rank) when the disk under the output
    directory lacks E2E_DISK_BYTES.  Returns the record on rank 0."""
    import shutil
    base = args.e2e_dir or "/tmp/gpdla_e2e_alt"
    Path(base).parent.mkdir(parents=True, exist_ok=True)
    free = shutil.disk_usage(Path(base).parent).free
    if dist is not None:
        box = [free]
        dist.broadcast_object_list(box, src=0)
        free = box[0]
    if free < E2E_DISK_BYTES:
        return {"skipped": f"{free / 1e9:.0f} GB free under {Path(base).parent}, "
                           f"{E2E_DISK_BYTES / 1e9:.0f} GB needed (13 GB output + the processed/ tree)"} if rank == 0 else None
    rec = e2e_record(162861, 10000, 20, base, False, world, rank, dist, dev)
    if rank == 0 and world > 1 and rec["e2e"]["devices_used"] < world:
        rec["rehearsal"] = {"value_if_counted": rec["value"], "note": "ranks shared GPUs: not an N-GPU point"}
        rec["value"] = None
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--e2e-dir", default=None, help="e2e: directory for the processed/ tree (default /tmp/...)")
    ap.add_argument("--e2e-keep", action="store_true", help="e2e: keep the files afterwards")
    ap.add_argument("--workload", choices=sorted(WORKLOADS) + ["e2e"], default="c2",
                    help="BASELINE.json configs: c2 = configs[1] (default bench line), c3 = configs[2] "
                         "(full DR12Q, 1 GPU), c4 = configs[3] (full DR12Q split over the ranks), "
                         "c5 = configs[4] (k=50, 10^5 samples); e2e = configs[2] end to end on files")
    ap.add_argument("--spectra", type=int, default=None, help="override: spectra per GPU (c2/c5)")
    ap.add_argument("--samples", type=int, default=None, help="override: DLA samples")
    ap.add_argument("--k", type=int, default=None, help="override: rank")
    ap.add_argument("--path", choices=["auto", "fused", "fused_i8", "panel_gemm", "panel_gemm_i8", "panel_gemm_i8_24"], default="auto",
                    help="likelihood path (Engine path=): auto = fused fp64 kernel for the compiled ranks, "
                         "fused_i8 = the int8 Ozaki contraction (k=20), panel_gemm = weights + dgemm + LDL^T")
    ap.add_argument("--panel-streams", type=int, choices=[1, 2, 3, 4], default=2,
                    help="panel-GEMM paths: compute streams a batch's spectra alternate over")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the alternative-path measurement (fused_i8 next to the fp64 line, 1 GPU, c2)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (0 = skip)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the rank/spectrum/device layout through the launcher, no GPU call")
    ap.add_argument("--plan-devices", type=int, default=None,
                    help="--plan-only: the device count to plan against (default: one per rank)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow N ranks on fewer than N devices (ranks share GPUs); the line then carries "
                         "value null and is labelled a rehearsal, never an N-GPU point")
    ap.add_argument("--no-configs3", action="store_true",
                    help="skip alternatives.configs3 (the full DR12Q count split over the ranks) in a multi-rank line")
    ap.add_argument("--no-configs2", action="store_true",
                    help="skip alternatives.configs2 (full DR12Q count on this GPU) in the default line")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip alternatives.e2e (configs[2] end to end on files) in the default line")
    ap.add_argument("--no-widened", action="store_true",
                    help="skip alternatives.dla_samples / .ingest (SURVEY 8f-2, 8f-4) in the default line")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no launcher: start the N ranks as children (nothing has touched the GPU yet)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is None:          # under torch.distributed.run without --gpus: the launcher's count
        args.gpus = world
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with _stdout_to_stderr():  # gloo prints its connection banner on stdout (fd 1)
            dist.init_process_group("gloo", rank=rank, world_size=world)

    if args.workload == "e2e":
        run_e2e(args, world, rank, local_rank, dist if world > 1 else None)
        if world > 1:
            with _stdout_to_stderr():
                dist.destroy_process_group()
        return

    wl = dict(WORKLOADS[args.workload])
    for key in ("spectra", "samples", "k"):
        if getattr(args, key) is not None:
            wl[key] = getattr(args, key)
    if args.plan_only:
        plan_only(wl, world, rank, local_rank, dist if world > 1 else None, args.plan_devices, args.rehearsal,
                  alternatives=(world > 1 and not args.no_alt and not wl["dr12q"] and wl["k"] == 20
                                and args.path == "auto"))
        if world > 1:
            with _stdout_to_stderr():
                dist.destroy_process_group()
        return

    from gp_dla_detection_amd import _lib as L
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters

    args.k, args.samples = wl["k"], wl["samples"]
    model = syn.make_model(k=args.k)
    samples = syn.make_samples(args.samples)
    if wl["dr12q"]:
        # full DR12Q count (162,861) of DR12Q-shaped spectra (n ~ 270-1250): a pool of 4096
        # distinct synthetic spectra tiled to the count; c3 = all on one GPU, c4 = split over ranks
        pool = dr12q_pool(model)
        ids = rank_spectrum_ids(wl, rank, world, [p["wavelengths"].size for p in pool])
        spectra = [pool[i % len(pool)] for i in ids]
    else:
        ids = rank_spectrum_ids(wl, rank, world)
        spectra = [syn.make_spectrum(model, int(i)) for i in ids]
    Q = ids.size
    packed = syn.pack_spectra(spectra)
    # CPU baseline first, while no process has touched the GPU (its workers are spawned)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        cpu = cpu_baseline(model, samples, spectra, args.cpu_budget, args.k,
                           widened=not args.no_alt and not args.no_widened and not wl["dr12q"] and args.k == 20)
    # one GPU per local rank; fewer devices than ranks is refused unless --rehearsal (ranks share devices)
    dev, err = assign_device(world, local_rank, L.load().gpdla_device_count(), args.rehearsal)
    if err:
        refuse(err, rank)
    D = lambda a: L.DeviceArray.from_numpy(a, device=dev)
    t = {key: D(packed[key]) for key in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
    S = args.samples
    o_null = L.DeviceArray(dev, Q, np.float64)
    o_dla = L.DeviceArray(dev, Q, np.float64)
    o_s = L.DeviceArray(dev, (Q, S), np.float64)
    o_n = L.DeviceArray(dev, Q, np.int32)

    # which physical GPU each rank drives (N distinct devices on an N-GPU node)
    ranks = gather({"rank": rank, "local_rank": local_rank, "device": dev, "pci_bus_id": L.pci_bus_id(dev),
                    "spectra": int(Q), "first_spectrum": int(ids[0]), "last_spectrum": int(ids[-1])},
                   world, dist if world > 1 else None)
    distinct = len({r["pci_bus_id"] for r in ranks})
    if distinct < world and not args.rehearsal:
        refuse(f"{world} ranks drive only {distinct} distinct GPU(s) (PCI ids "
               f"{sorted({r['pci_bus_id'] for r in ranks})}): not a {world}-GPU measurement", rank)

    if args.path == "auto" and "default_path" in wl:
        args.path = wl["default_path"]
    eng = Engine(model, samples, set_parameters(k=args.k), device=dev, path=args.path)
    eng.set_panel_streams(args.panel_streams)    # the panel paths' compute streams (others ignore it)
    if args.path == "fused_i8":
        path = "fused-int8"
    elif args.path == "panel_gemm_i8":
        path = "panel-GEMM-int8"
    elif args.path == "panel_gemm_i8_24":
        path = "panel-GEMM-int8-24"
    elif args.path == "panel_gemm" or args.k not in (4, 8, 10, 12, 16, 20, 24):
        path = "panel-GEMM"
    else:
        path = "fused"

    def step():
        eng.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                           t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null.ptr, o_dla.ptr, o_s.ptr, S,
                           npix_ptr=o_n.ptr)

    for _ in range(args.warmup):
        step()
    eng.synchronize()
    eng.reset_stats()
    local = []
    elapsed = timed_steps(step, eng.synchronize, args.steps, dist if world > 1 else None, local)
    st = eng.stats()
    npix = o_n.numpy()
    n_mean = float(np.mean(npix))
    alone = None
    if path.startswith("panel-GEMM") and args.panel_streams > 1:
        st1 = single_stream_stats(eng, step, args.panel_streams)
        alone = (i8_roofline(st1, n_mean, args.k, Q, S, 2, path) if path.startswith("panel-GEMM-int8")
                 else f64_gemm_roofline(st1, n_mean, args.k, Q, S, 2))

    # per-rank load balance: each rank's own kernel time and wall time over the timed steps
    per_rank = gather({"rank": rank, "spectra": int(Q), "pixels": int(np.sum(npix)),
                       "likelihood_ms_per_step": st["likelihood_ms"] / args.steps,
                       "kernel_ms_per_step": (st["prep_ms"] + st["likelihood_ms"] + st["reduce_ms"]) / args.steps,
                       "elapsed_ms_per_step": local[0] / args.steps * 1e3}, world, dist if world > 1 else None)
    for r, pr in zip(ranks, per_rank):
        r.update({k: v for k, v in pr.items() if k != "rank"})
    km = np.array([r["kernel_ms_per_step"] for r in per_rank])
    em = np.array([r["elapsed_ms_per_step"] for r in per_rank])
    imbalance = {"kernel_ms_max_over_mean": float(km.max() / km.mean()) if km.mean() > 0 else None,
                 "elapsed_max_over_mean": float(em.max() / em.mean()) if em.mean() > 0 else None,
                 "note": "per-rank HIP-event kernel time and rank-local wall time of the timed steps; the "
                         "line's ms_per_step is the max over ranks"}

    # alternative paths / configs on the same GPU (1 GPU, configs[1] default line).  None is `value`:
    # the headline stays on configs[1] on the path that computes the contraction in fp64.
    alt = None
    if world == 1 and not args.no_alt and not wl["dr12q"] and args.k == 20 and args.path == "auto":
        o_s2 = L.DeviceArray(dev, (Q, S), np.float64)
        o_null2, o_dla2 = L.DeviceArray(dev, Q, np.float64), L.DeviceArray(dev, Q, np.float64)
        with Engine(model, samples, set_parameters(k=args.k), device=dev, path="fused_i8") as e2:
            def step2():
                e2.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                                  t["pixel_mask"].ptr, t["z_qsos"].ptr, o_null2.ptr, o_dla2.ptr, o_s2.ptr, S)
            step2()
            e2.synchronize()
            e2.reset_stats()
            t2 = time.perf_counter()
            for _ in range(args.steps):
                step2()
            e2.synchronize()
            el2 = time.perf_counter() - t2
            st2 = e2.stats()
        a_ref, a_got = o_s.numpy(rows=256), o_s2.numpy(rows=256)
        rel = float(np.max(np.abs(a_got - a_ref) / np.maximum(np.abs(a_ref), 1.0)))
        rel_dla = float(np.max(np.abs(o_dla2.numpy() - o_dla.numpy()) / np.maximum(np.abs(o_dla.numpy()), 1.0)))
        l2 = st2["likelihood_ms"] / max(st2["likelihood_launches"], 1)
        alt = {"fused_i8": {
            "value": Q * S * args.steps / el2, "unit": "evals/s", "ms_per_step": el2 / args.steps * 1e3,
            "kernel_ms": {"prep+convert": st2["prep_ms"] / max(st2["prep_launches"], 1), "likelihood": l2},
            "algorithmic_tflops": algorithmic_flops_per_eval(n_mean, args.k) * Q * (S + 1) / (l2 * 1e-3) / 1e12,
            "algorithmic_tflops_note": "SURVEY 8d F_eval over the likelihood kernel time; the fp64 fused kernel's "
                                       "peak is 78.6 TF/s, this one computes the Gram/u contraction on int8 MFMA",
            "max_rel_err_vs_fp64": {"sample_log_likelihoods_dla(256 spectra)": rel, "log_likelihoods_dla": rel_dla},
            "note": "likelihood_i8_kernel<20>: Gram/u contraction exact on v_mfma_i32_16x16x64_i8 over "
                    "32-bit-quantised weights/panel (4 digits, levels <= 3), fp64 everywhere else; "
                    "within the 1e-6 contract, not bitwise-fp64 (DESIGN.md section 4)"}}
        for a in (o_s2, o_null2, o_dla2):
            a.free()
        # BASELINE configs[4] (k = 50, 10^5 samples) on the int8 panel-GEMM path, driver-timed
        alt["configs4"] = configs4_alternative(dev, args.steps)
        if not args.no_widened:  # SURVEY 8f-2 and 8f-4 on the device, CPU restatements in cpu_baseline
            alt["dla_samples"] = dla_samples_alternative(dev)
            alt["ingest"] = ingest_alternative(dev)
            alt["objective"] = objective_alternative(dev)

    # sanity: finite outputs and the calc_cddf.py:246 normalisation invariant on every spectrum
    inv = invariant_all_rows(o_s, o_dla, S)
    ok = bool(inv["finite"] and inv["max_abs_dev"] < 1e-10)
    for a in (*t.values(), o_null, o_dla, o_s, o_n):
        a.free()

    if world > 1 and not args.no_alt and not wl["dr12q"] and args.k == 20 and args.path == "auto":
        # the north-star configs at N ranks: configs[3] = the full DR12Q count split
        # over the ranks, and configs[2] end to end on files with every rank writing its own chunks
        alt = {}
        if not args.no_configs3:
            alt["configs3"] = configs3_alternative(dev, world, rank, dist, args.rehearsal)
        if not args.no_e2e:
            alt["e2e"] = e2e_alternative(args, world, rank, dist, dev)
    elif alt is not None and not args.no_configs2:
        # BASELINE configs[2]: the full DR12Q count on this GPU, driver-timed (north star "< 60 s")
        alt["configs2"] = configs2_alternative(dev)
    if world == 1 and alt is not None and not args.no_e2e:
        alt["e2e"] = e2e_alternative(args, 1, 0, None, dev)

    q_total = Q
    if world > 1:  # spectra over all ranks (LPT shards of configs[3] differ in size)
        import torch
        qt = torch.tensor([Q], dtype=torch.int64)
        dist.all_reduce(qt, op=dist.ReduceOp.SUM)
        q_total = int(qt.item())
    evals_total = q_total * S * args.steps
    value = evals_total / elapsed
    launches = max(st["likelihood_launches"], 1)
    avg_ms = st["likelihood_ms"] / launches
    evals_per_launch = Q * (S + 1) * args.steps / launches  # incl. the null-model evaluation
    flops_launch = algorithmic_flops_per_eval(n_mean, args.k) * evals_per_launch
    achieved_tf = flops_launch / (avg_ms * 1e-3) / 1e12
    eff_gbs = effective_bytes_per_eval(n_mean, args.k) * evals_per_launch / (avg_ms * 1e-3) / 1e9

    traffic, traffic_src = profiled_traffic(Q, S, args.k, path)
    roof = {"bound": "mfma", "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": ROOFLINE_KERNEL.get(path, path).format(k=args.k),
            "avg_launch_ms": avg_ms,
            "flops_per_eval": algorithmic_flops_per_eval(n_mean, args.k),
            "evals_per_launch": evals_per_launch,
            # int8 panel paths: the int8 GEMM kernel's own roofline (overrides the fields above)
            **(i8_roofline(st, n_mean, args.k, Q, S, args.steps, path) if path.startswith("panel-GEMM-int8")
               else f64_gemm_roofline(st, n_mean, args.k, Q, S, args.steps) if path == "panel-GEMM"
               else {})}
    if alone is not None:
        roof.update(panel_roofline_streams(roof, alone, args.panel_streams))
    rehearsal = world > 1 and distinct < world
    result = {
        "metric": "(spectrum x DLA-sample) log-evidence evals/sec",
        "value": None if rehearsal else value,
        "unit": "evals/s",
        "n_gpus": world,
        "world_size": dist.get_world_size() if world > 1 else 1,
        "ranks": ranks,
        "distinct_devices": distinct,
        "imbalance": imbalance,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": {"fused": "f64", "panel-GEMM": "f64",
                  "panel-GEMM-int8-24": "f64+i8+f32 (Gram contraction exact in int8/int32 over 24-bit-quantised "
                                        "operands, u over 32-bit, raw Voigt profiles in fp32, fp64 elsewhere; "
                                        "fp32-class, ~2.5e-7 from fp64)"}.get(
                     path, "f64+i8 (Gram/u contraction exact in int8/int32 over 32-bit-quantised operands, fp64 elsewhere)"),
        "data": "synthetic (seeded; SURVEY.md 8d model/spectra, unscrambled Halton samples)"
                + ("; DR12Q-shaped pool of 4096 spectra tiled to the count" if wl["dr12q"] else ""),
        "config": {"workload": f"{wl['label']}; this rank: {Q} spectra, mean n={n_mean:.0f}, 3 Lyman lines",
                   "spectra_per_gpu": Q, "num_samples": S, "k": args.k, "n_pixels": n_mean,
                   "likelihood_path": path, "parallelism": f"spectrum-shard x{world}"},
        "roofline": roof,
        "dram": dram_record(traffic, roof["avg_launch_ms"], traffic_src, path),
        "streamed_panel_equiv": {"gbs": eff_gbs, "bytes_per_eval": effective_bytes_per_eval(n_mean, args.k),
                                 "note": "SURVEY.md 8d's streamed-panel accounting (B_eval bytes per evaluation / "
                                         "kernel time): what a kernel re-reading the n x (k+5) panel per sample would "
                                         "move.  Not DRAM traffic and not a roofline fraction: this fused kernel reads "
                                         "each panel once per 64 samples (see dram)."},
        "kernel_ms": {"prep": st["prep_ms"] / max(st["prep_launches"], 1), "likelihood": avg_ms,
                      "reduce": st["reduce_ms"] / max(st["reduce_launches"], 1)},
        "invariant_calc_cddf_246": inv,
        "checks_ok": ok,
    }
    if rehearsal:
        result["rehearsal"] = {"value_if_counted": value, "distinct_devices": distinct,
                               "note": f"--rehearsal: {world} ranks shared {distinct} GPU(s); not a {world}-GPU point"}
    if cpu is not None:
        result["cpu_baseline"] = cpu
    if alt is not None:
        result["alternatives"] = alt
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        with _stdout_to_stderr():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
