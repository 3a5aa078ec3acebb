"""Line centres on the padded grid: the Voigt zones of the batched sweeps at their edges.

Every kernel path evaluates the damping wing branch-free and recomputes, per batch of pixels, only
the lanes within kOuterX = 32 Doppler units of a Lyman line, and there only the nearest line
(device_common.h nearest_line / raw_profile3_batch, kernels.hip likelihood_kernel).  Here the DLA
samples are placed so that the Lya, Lyb and Lyg centres fall exactly on padded-grid wavelengths
(x = 0 up to rounding), and at x = +-5, +-9, +-20, +-32 and +-40 from one (core, the core/inner-wing
edge, inner wing, the fix-up edge, outer wing), at the extreme column densities 1e20 and 1e23, and
each path is checked against the oracle (voigt.c:282-299 with scipy's voigt_profile,
process_qsos.m:184-197).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from gp_dla_detection_amd import _lib as L  # noqa: E402
from gp_dla_detection_amd import synthetic as syn  # noqa: E402
from gp_dla_detection_amd.engine import Engine  # noqa: E402
from gp_dla_detection_amd.parameters import set_parameters  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def require_device():
    lib = L.load()
    assert lib.gpdla_device_count() > 0, "no HIP device: GPU tests must run on the MI355X box"


def _centred_samples(prep, O):
    """Offsets putting line j's centre at padded wavelength i shifted by dx Doppler units."""
    padded, zmin, zmax = prep["padded"], prep["zmin"], prep["zmax"]
    c_over = O.C_CGS / (O.SIGMA * np.sqrt(2.0))        # x = c_over (lam / (lam_j (1 + z)) - 1)
    offs, nhis = [], []
    for j in range(3):
        lam_j = O.TRANSITION_WAVELENGTHS[j] * 1e8
        for i in range(0, padded.size, 97):
            for dx in (0.0, 5.0, -5.0, 9.0, -9.0, 20.0, -20.0, 32.0, -32.0, 40.0, -40.0):
                z = padded[i] / (lam_j * (1.0 + dx / c_over)) - 1.0
                off = (z - zmin) / (zmax - zmin)
                if 0.0 <= off <= 1.0:
                    for N in (1e20, 1e23):
                        offs.append(off)
                        nhis.append(N)
    return dict(offset_samples=np.array(offs), nhi_samples=np.array(nhis),
                log_nhi_samples=np.log10(np.array(nhis)))


@pytest.fixture(scope="module")
def centred_case():
    from oracle import gpdla_oracle as O
    model = syn.make_model(k=20, seed=11)
    spec = syn.make_spectrum(model, 0, z_qso=3.2, n_target=None, mask_fraction=0.05)
    prep = O.prepare_spectrum(spec["wavelengths"], spec["flux"], spec["noise_variance"], spec["pixel_mask"],
                              spec["z_qso"], model)
    samples = _centred_samples(prep, O)
    assert samples["offset_samples"].size >= 64
    ref = O.process_spectrum(spec["wavelengths"], spec["flux"], spec["noise_variance"], spec["pixel_mask"],
                             spec["z_qso"], model, samples["offset_samples"], samples["nhi_samples"])
    return model, spec, samples, ref


@pytest.mark.parametrize("path,tol", [("fused", 1e-9), ("panel_gemm", 1e-9), ("fused_i8", 1e-8),
                                      ("panel_gemm_i8", 1e-8), ("panel_gemm_i8_24", 5e-7)])
def test_line_centres_on_the_padded_grid(centred_case, path, tol):
    model, spec, samples, ref = centred_case
    with Engine(model, samples, set_parameters(k=20), path=path) as eng:
        out = eng.process(syn.pack_spectra([spec]))
    got, want = out["sample_log_likelihoods_dla"][0], ref["sample_log_likelihoods_dla"]
    assert np.all(np.isfinite(got))
    err = np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0))
    assert err < tol, (path, err)
    assert abs(out["log_likelihoods_no_dla"][0] - ref["log_likelihood_no_dla"]) < tol * max(
        abs(ref["log_likelihood_no_dla"]), 1.0)
