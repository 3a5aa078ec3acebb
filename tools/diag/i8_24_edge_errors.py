"""Per-spectrum error of the int8 panel paths against the fp64 panel path on the edge-case spectra of
tests/test_gpu_i8.py::test_panel_gemm_i8_edge_cases (n = 1..65), split by error kind."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402

model = syn.make_model(k=50, seed=3)
samples = syn.make_samples(67)
base = syn.make_spectrum(model, 0, z_qso=2.8, n_target=None, mask_fraction=0.1)
spectra = []
sizes = (1, 3, 9, 33, 65)
for npx in sizes:
    sl = slice(100, 100 + npx)
    s = {kk: (v[sl] if isinstance(v, np.ndarray) else v) for kk, v in base.items()}
    s["pixel_mask"] = np.zeros(npx, dtype=bool)
    spectra.append(s)
packed = syn.pack_spectra(spectra)


def run(path):
    with Engine(model, samples, set_parameters(k=50), path=path) as eng:
        return eng.process(packed)


ref = run("panel_gemm")
for path in ("panel_gemm_i8", "panel_gemm_i8_24"):
    out = run(path)
    for q, n in enumerate(sizes):
        r, g = ref["sample_log_likelihoods_dla"][q], out["sample_log_likelihoods_dla"][q]
        abs_err = np.abs(g - r)
        rel = abs_err / np.maximum(np.abs(r), 1.0)
        i = int(np.argmax(rel))
        print(f"{path:18s} n={n:3d} npix={out['num_pixels'][q]:3d} max rel {rel.max():.3e} at s={i} "
              f"(ll {r[i]:.6f}, abs {abs_err[i]:.3e}); null rel "
              f"{abs(out['log_likelihoods_no_dla'][q] - ref['log_likelihoods_no_dla'][q]) / max(abs(ref['log_likelihoods_no_dla'][q]), 1):.3e}"
              f" (ll {ref['log_likelihoods_no_dla'][q]:.4f}); median |ll| {np.median(np.abs(r)):.3f}", flush=True)
