"""Throughput of the widened rows on the device, for the measurement bar the hot
path has: the DLA-sample generator at BASELINE's sample counts and preload_qsos's numeric stage over
the DR12Q count (162,861 full BOSS coadds, a pool of 4,096 distinct spectra tiled), host copies
included, with the kernels' own times from a rocprofv3 kernel trace of the same command:

    python tools/bench_ingest.py [out.json]
    rocprofv3 --kernel-trace --stats -d gpurun_out/<dir> -o ingest -- python3 tools/bench_ingest.py

Algorithmic bytes of the ingest kernels (HBM-bound elementwise work): the scan reads 12 B per input
pixel (loglam, ivar, and_mask: single / int32; flux only in the 1310-1325 A window); the write pass
reads 16 B and writes 13 B (wavelength, flux, noise variance, mask) per selected pixel.  A single
fused pass could not do with less than 12 B per input pixel + 17 B per selected one ("fused_ideal")."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gp_dla_detection_amd import dla_samples as DS  # noqa: E402
from gp_dla_detection_amd import ingest as I  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402


def boss_pool(npool, seed=31):
    rng = np.random.default_rng(seed)
    zp = rng.uniform(2.15, 5.5, npool)
    return zp, [syn.make_boss_coadd_columns(rng, z) for z in zp]


def main(out=None):
    res = {}
    rng = np.random.default_rng(5)
    log_nhis = np.r_[rng.normal(20.55, 0.3, 800), rng.uniform(20.3, 21.8, 200)]
    for S in (10_000, 100_000):
        DS.generate_dla_samples(log_nhis, S)                    # warm-up
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            DS.generate_dla_samples(log_nhis, S)
        res[f"dla_samples_S{S}"] = {"wall_ms": (time.perf_counter() - t0) / reps * 1e3, "samples": S,
                                    "note": "gpdla_generate_dla_samples_f64, host buffers in and out"}
    Qt, npool = 162861, 4096
    zp, pool = boss_pool(npool)
    sel = np.arange(Qt) % npool
    flags = np.zeros(Qt, np.uint8)
    batch = 16384
    wr = I.preload_batch(zp[:256], flags[:256], [pool[i] for i in range(256)])  # warm-up (one launch each)
    warm = {"pixels_in": sum(pool[i][0].size for i in range(256)),
            "pixels_out": sum(c.size for c in wr["all_wavelengths"])}
    t0 = time.perf_counter()
    t_dev = 0.0
    npx = nsel = 0
    for b0 in range(0, Qt, batch):
        idx = sel[b0:b0 + batch]
        cols = [pool[i] for i in idx]
        t1 = time.perf_counter()
        r = I.preload_batch(zp[idx], flags[b0:b0 + batch], cols)
        t_dev += time.perf_counter() - t1
        npx += sum(c[0].size for c in cols)
        nsel += sum(c.size for c in r["all_wavelengths"])
    wall = time.perf_counter() - t0
    res["preload_qsos_dr12q"] = {
        "spectra": Qt, "pixels_in": npx, "pixels_out": nsel, "wall_s": wall, "preload_batch_s": t_dev,
        "batches": -(-Qt // batch), "warmup": warm,
        "algorithmic_bytes": {"scan": 12 * npx, "write": 29 * nsel, "fused_ideal": 12 * npx + 17 * nsel},
        "note": "preload_batch = host packing of the CSR + H2D + both kernels + D2H + splitting into cells, "
                "16,384 spectra per call; the kernels' own times are in the rocprofv3 trace of this command"}
    print(json.dumps(res), flush=True)
    if out:
        Path(out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
