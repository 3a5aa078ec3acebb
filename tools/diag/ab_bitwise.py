"""Bitwise A/B of two libgpdla builds on one panel path at a configs[4]-shaped size (GPU box):

    python tools/diag/ab_bitwise.py <a.so|head> <b.so|head> [path] [spectra] [samples]

Each build runs in its own subprocess (GPDLA_LIB), on DR12Q-like k = 50 spectra; the sample
log-likelihoods are compared bit for bit."""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
CHILD = r'''
import sys; sys.path.insert(0, sys.argv[1])
import numpy as np
from gp_dla_detection_amd import synthetic as syn
from gp_dla_detection_amd.engine import Engine
from gp_dla_detection_amd.parameters import set_parameters
path, nq, ns, out = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
model = syn.make_model(k=50, seed=7)
samples = syn.make_samples(ns)
packed = syn.pack_spectra(syn.make_dr12q_like_spectra(model, nq, seed=3, mask_fraction=0.05))
with Engine(model, samples, set_parameters(k=50), path=path) as eng:
    o = eng.process(packed)
np.savez(out, sll=o["sample_log_likelihoods_dla"], null=o["log_likelihoods_no_dla"])
'''


def run(lib, path, nq, ns, out):
    env = dict(os.environ)
    env.pop("GPDLA_LIB", None)
    if lib != "head":
        env["GPDLA_LIB"] = str(Path(lib).resolve())
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), path, str(nq), str(ns), out], check=True, env=env,
                   timeout=600)
    return np.load(out)


if __name__ == "__main__":
    a, b = sys.argv[1], sys.argv[2]
    path = sys.argv[3] if len(sys.argv) > 3 else "panel_gemm_i8_24"
    nq = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    ns = int(sys.argv[5]) if len(sys.argv) > 5 else 100000
    with tempfile.TemporaryDirectory() as d:
        A = run(a, path, nq, ns, f"{d}/a.npz")
        B = run(b, path, nq, ns, f"{d}/b.npz")
        for key in ("sll", "null"):
            x, y = A[key], B[key]
            same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
            diff = float(np.nanmax(np.abs(x - y))) if not same else 0.0
            print(f"{path} {key}: {'BITWISE EQUAL' if same else 'DIFFER max abs %.3e' % diff} "
                  f"({x.size} values, finite {bool(np.all(np.isfinite(x)))})", flush=True)
