"""Per-spectrum error of the int8 panel paths against the fp64 panel path.

    python tools/diag/i8_24_edge_errors.py            short spectra (n = 1..65: tests/test_gpu_i8.py::
                                                      test_panel_gemm_i8_edge_cases), both int8 paths
    python tools/diag/i8_24_edge_errors.py above      the 24-bit path just above its 32-bit cutover
                                                      (internal.h i8_spectrum_nd: <= 128 pixels take 32-bit
                                                      digits): n = 129..512 over 3 seeds, and the margin of
                                                      the worst spectrum against the tests' 5e-7 bar
                                                      

The 24-bit scheme's error is absolute (~2^-24 of the Gram's scale), so relative to max(|ll|, 1) it is
largest where |ll| is small: short spectra."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402

BAR = 5e-7


def spectra_of(model, sizes, seed, start):
    base = syn.make_spectrum(model, seed, z_qso=2.8, n_target=None, mask_fraction=0.1)
    out = []
    for npx in sizes:
        sl = slice(start, start + npx)
        s = {kk: (v[sl] if isinstance(v, np.ndarray) else v) for kk, v in base.items()}
        s["pixel_mask"] = np.zeros(npx, dtype=bool)
        out.append(s)
    return out


def run(model, samples, packed, path):
    with Engine(model, samples, set_parameters(k=50), path=path) as eng:
        return eng.process(packed)


def report(model, samples, sizes, seed, start, paths):
    packed = syn.pack_spectra(spectra_of(model, sizes, seed, start))
    ref = run(model, samples, packed, "panel_gemm")
    worst = 0.0
    for path in paths:
        out = run(model, samples, packed, path)
        for q, n in enumerate(sizes):
            r, g = ref["sample_log_likelihoods_dla"][q], out["sample_log_likelihoods_dla"][q]
            abs_err = np.abs(g - r)
            rel = abs_err / np.maximum(np.abs(r), 1.0)
            i = int(np.argmax(rel))
            null_rel = (abs(out["log_likelihoods_no_dla"][q] - ref["log_likelihoods_no_dla"][q])
                        / max(abs(ref["log_likelihoods_no_dla"][q]), 1))
            worst = max(worst, float(rel.max()), float(null_rel)) if path.endswith("_24") else worst
            print(f"{path:18s} seed={seed} n={n:3d} npix={out['num_pixels'][q]:3d} max rel {rel.max():.3e} at s={i} "
                  f"(ll {r[i]:.6f}, abs {abs_err[i]:.3e}); null rel {null_rel:.3e} "
                  f"(ll {ref['log_likelihoods_no_dla'][q]:.4f}); median |ll| {np.median(np.abs(r)):.3f}", flush=True)
    return worst


if __name__ == "__main__":
    model = syn.make_model(k=50, seed=3)
    if len(sys.argv) > 1 and sys.argv[1] == "above":
        samples = syn.make_samples(1000)
        worst = max(report(model, samples, (129, 160, 193, 256, 320, 384, 448, 512), seed, 20, ("panel_gemm_i8_24",))
                    for seed in (0, 1, 2))
        print(f"24-bit path, n = 129..512, 3 seeds x 8 lengths x 1,001 evaluations: worst relative error "
              f"{worst:.3e}, margin {BAR / worst:.1f}x against the {BAR:.0e} bar", flush=True)
    else:
        report(model, syn.make_samples(67), (1, 3, 9, 33, 65), 0, 100, ("panel_gemm_i8", "panel_gemm_i8_24"))
