"""Timing-only A/B of libgpdla builds on the configs[4] GEMM launch (GPU box):

    python tools/diag/time_c5_gemm.py <a.so|head> [<b.so|head> ...]

Each build runs in its own subprocess (GPDLA_LIB) on 32 configs[4] spectra (k = 50, 10^5 samples,
panel_gemm_i8_24), 2 timed passes after one warm-up; prints the average GEMM launch time (HIP events,
gpdla_stats.contraction_ms) and the batch time.  Numeric errors of timing-only variants (whose results
are wrong on purpose) are ignored."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CHILD = r'''
import sys; sys.path.insert(0, sys.argv[1])
import numpy as np
from gp_dla_detection_amd import _lib as L, synthetic as syn
from gp_dla_detection_amd.engine import Engine
from gp_dla_detection_amd.parameters import set_parameters
Q, S, k = 32, 100000, 50
model = syn.make_model(k=k); samples = syn.make_samples(S)
packed = syn.pack_spectra([syn.make_spectrum(model, q) for q in range(Q)])
t = {key: L.DeviceArray.from_numpy(packed[key]) for key in ("wavelengths", "flux", "noise_variance", "pixel_mask", "z_qsos")}
o1, o2, o3 = L.DeviceArray(0, Q, np.float64), L.DeviceArray(0, Q, np.float64), L.DeviceArray(0, (Q, S), np.float64)
with Engine(model, samples, set_parameters(k=k), path="panel_gemm_i8_24") as eng:
    def step():
        eng.process_device(packed["offsets"], t["wavelengths"].ptr, t["flux"].ptr, t["noise_variance"].ptr,
                           t["pixel_mask"].ptr, t["z_qsos"].ptr, o1.ptr, o2.ptr, o3.ptr, S)
    def sync():
        try:
            eng.synchronize()
        except L.GpdlaNumericError:
            pass
    step(); sync(); eng.reset_stats()
    for _ in range(2):
        step()
    sync()
    st = eng.stats()
print(f"gemm {st['contraction_ms'] / max(st['contraction_launches'], 1):.4f} ms/launch  "
      f"batch {st['likelihood_ms'] / max(st['likelihood_launches'], 1):.3f} ms", flush=True)
'''
for lib in sys.argv[1:]:
    env = dict(os.environ)
    env.pop("GPDLA_LIB", None)
    if lib != "head":
        env["GPDLA_LIB"] = str(Path(lib).resolve())
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], env=env, capture_output=True, text=True, timeout=600)
    print(f"{Path(lib).name:12s}", r.stdout.strip() or r.stderr.strip()[-300:], flush=True)
