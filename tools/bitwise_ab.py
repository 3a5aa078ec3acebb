"""Bitwise A/B of two library builds on the panel paths (run on the GPU box).

    GPDLA_LIB=<a.so> python tools/bitwise_ab.py run a.npz [samples] [paths]
    GPDLA_LIB=<b.so> python tools/bitwise_ab.py run b.npz [samples] [paths]
    python tools/bitwise_ab.py compare a.npz b.npz

`run` evaluates 8 DR12Q-like spectra x 3,000 samples (or [samples]) at k = 50 on every panel path and
k = 20 on the fused paths (or the comma-separated [paths]) and saves the sample log-likelihoods; `compare` reports, per path, whether the two
builds agree bit for bit (and the largest difference if not).
"""
import sys

import numpy as np


def run(out, nsamples=3000, only=None):
    sys.path.insert(0, ".")
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    res = {}
    for k, paths in ((50, ("panel_gemm", "panel_gemm_i8", "panel_gemm_i8_24")), (20, ("fused", "fused_i8"))):
        model = syn.make_model(k=k, seed=7)
        samples = syn.make_samples(nsamples)
        packed = syn.pack_spectra(syn.make_dr12q_like_spectra(model, 8, seed=3, mask_fraction=0.05))
        for p in paths:
            if only and p not in only:
                continue
            with Engine(model, samples, set_parameters(k=k), path=p) as eng:
                o = eng.process(packed)
            res[p] = o["sample_log_likelihoods_dla"]
            res[p + "_null"] = o["log_likelihoods_no_dla"]
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for key in A.files:
        x, y = A[key], B[key]
        same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
        print(f"{key:24s} {'bitwise equal' if same else 'differ: max rel %.3g' % np.max(np.abs(x - y) / np.maximum(np.abs(y), 1))}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3000,
            sys.argv[4].split(",") if len(sys.argv) > 4 else None)
    else:
        compare(sys.argv[2], sys.argv[3])
