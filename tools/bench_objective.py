"""Time the GPU training objective (objective.m) on a DR9-training-set-sized synthetic problem:
Q spectra x 1217 rest pixels, k = 20, ~30% missing pixels.  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gp_dla_detection_amd import training as T  # noqa: E402


def main(Q=5000, P=1217, k=20, reps=5):
    rng = np.random.default_rng(3)
    y = 0.3 * rng.standard_normal((Q, P))
    y[rng.uniform(size=y.shape) < 0.3] = np.nan
    lya = rng.uniform(2.5, 4.5, (Q, P))
    nv = rng.uniform(0.01, 0.1, (Q, P))
    x = np.concatenate([0.05 * rng.standard_normal(P * k), np.log(0.15) + 0.1 * rng.standard_normal(P),
                        [np.log(0.1), np.log(0.0023), np.log(3.65)]])
    with T.Objective(y, lya, nv, k) as obj:
        obj(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            f, g = obj(x)
        dt = (time.perf_counter() - t0) / reps
    flops = Q * np.mean((~np.isnan(y[:64])).sum(axis=1)) * (k * (k + 1) + 4 * k * k + 8 * k)
    print(json.dumps(dict(what="objective.m f+g on the GPU", spectra=Q, pixels=P, k=k, ms_per_eval=dt * 1e3,
                          spectra_per_s=Q / dt, approx_gflops=flops / dt / 1e9, f=f)))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
