"""The MATLAB gateways in matlab/ (the reference-side bindings of INTEGRATION.md), driven through an
in-process MEX runtime (tests/support/mex_api/mex_mock.c; no MATLAB here):

* gpdla_mex.c      'create' / 'process' / 'destroy' -- replaces process_qsos.m:88-220;
* voigt_mex.c      voigt(lambdas, z, N[, num_lines])  -- voigt.c:253-304;
* log_mvnpdf_low_rank_mex.c                           -- log_mvnpdf_low_rank.m:5-33;
* objective_gpu_mex.c  [f, g] = objective_gpu(...)     -- objective.m.

CPU: every gateway loads and rejects bad calls with a MATLAB error (and, without a device, the
engine's GPDLA_EDEVICE message).  GPU: each gateway's outputs equal the Python binding's bit for
bit on the same inputs -- the gateway's CSR packing, MATLAB Q x S orientation and argument order
are what is checked; the numerics are the engine's, pinned elsewhere."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

from gp_dla_detection_amd import _lib as L

MOCK = Path(__file__).parent / "support" / "mex_api"
DOUBLE, SINGLE, LOGICAL, CHAR, CELL, UINT64, INT32 = 6, 7, 3, 4, 1, 15, 12


IN_TREE_LIB = str((Path(L.__file__).parent / "libgpdla.so").resolve())   # what the mocks' rpath names


def _mapped_libgpdla() -> set:
    """Paths of every libgpdla.so mapped into this process (/proc/self/maps)."""
    out = set()
    for line in Path("/proc/self/maps").read_text().splitlines():
        parts = line.split(maxsplit=5)
        if len(parts) == 6 and Path(parts[5]).name == "libgpdla.so":
            out.add(str(Path(parts[5]).resolve()))
    return out


class Gateway:
    """One gateway linked with the mock MEX runtime; Python values <-> mxArrays."""

    def __init__(self, name):
        L.load()                                  # libgpdla first (one instance, torch-free)
        path = MOCK / f"lib{name}_mock.so"
        if not path.exists():
            pytest.skip(f"{path.name} not built (gp_dla_detection_amd.build.build_mex_mocks)")
        lib = C.CDLL(str(path))
        # The mock resolves libgpdla through its rpath (the in-tree build); L.load() honours GPDLA_LIB.
        # A "bitwise equal to the Python engine" check is only meaningful when both are one file.
        maps = _mapped_libgpdla()
        assert IN_TREE_LIB in maps, (IN_TREE_LIB, maps)
        if L.LIB_PATH.resolve() != Path(IN_TREE_LIB):
            pytest.skip(f"GPDLA_LIB={L.LIB_PATH} is not the in-tree {IN_TREE_LIB} the gateway links: "
                        "the two would run different builds")
        vp = C.c_void_p
        for fn, res, args in (("mock_numeric", vp, [C.c_int, C.c_size_t, C.c_size_t, vp]),
                              ("mock_string", vp, [C.c_char_p]), ("mock_cell", vp, [C.c_size_t, C.POINTER(vp)]),
                              ("mock_data", vp, [vp]), ("mock_m", C.c_size_t, [vp]), ("mock_n", C.c_size_t, [vp]),
                              ("mock_class", C.c_int, [vp]), ("mock_free", None, [vp]),
                              ("mock_error", C.c_char_p, []), ("mock_locks", C.c_int, []),
                              ("mock_call", C.c_int, [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp)])):
            f = getattr(lib, fn)
            f.restype, f.argtypes = res, args
        self.lib = lib

    def mx(self, v):
        lib = self.lib
        if isinstance(v, str):
            return lib.mock_string(v.encode())
        if isinstance(v, list):                               # n x 1 cell
            elems = (C.c_void_p * max(len(v), 1))(*[self.mx(e) for e in v])
            return lib.mock_cell(len(v), elems)
        a = np.asarray(v)
        cls = {np.dtype(bool): LOGICAL, np.dtype(np.uint64): UINT64, np.dtype(np.int32): INT32,
               np.dtype(np.float32): SINGLE}.get(a.dtype, DOUBLE)
        if cls == DOUBLE:
            a = a.astype(np.float64)
        m, n = (a.size, 1) if a.ndim <= 1 else a.shape
        buf = np.asfortranarray(a.reshape(m, n)).astype(a.dtype, copy=False)
        raw = np.ascontiguousarray(buf.ravel(order="F"))
        return lib.mock_numeric(cls, m, n, raw.ctypes.data_as(C.c_void_p))

    def py(self, p):
        lib = self.lib
        m, n, cls = lib.mock_m(p), lib.mock_n(p), lib.mock_class(p)
        dt = {DOUBLE: np.float64, UINT64: np.uint64, INT32: np.int32, LOGICAL: np.bool_}[cls]
        a = np.ctypeslib.as_array(C.cast(lib.mock_data(p), C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                  shape=(m * n,)).copy()
        return a.reshape((m, n), order="F")

    def __call__(self, nlhs, *args):
        prhs = (C.c_void_p * max(len(args), 1))(*[self.mx(a) for a in args])
        plhs = (C.c_void_p * max(nlhs, 1))()
        rc = self.lib.mock_call(nlhs, plhs, len(args), prhs)
        if rc:
            raise RuntimeError(self.lib.mock_error().decode())
        return [self.py(plhs[i]) for i in range(max(nlhs, 1)) if plhs[i]]


def _create_args(model, samples, params, path="auto", mode=0):
    p = params
    return ("create", 0.0, model["rest_wavelengths"], model["mu"], model["M"], model["log_omega"],
            model["log_c_0"], model["log_tau_0"], model["log_beta"], samples["offset_samples"],
            samples["nhi_samples"], p.num_lines, p.width, p.pixel_spacing, p.min_lambda, p.max_lambda,
            p.lya_wavelength, p.lyman_limit, p.min_z_cut, p.max_z_cut, float(mode), path)


@pytest.mark.parametrize("name", ["gpdla_mex", "voigt_mex", "log_mvnpdf_low_rank_mex", "objective_gpu_mex"])
def test_gateways_reject_bad_calls(name):
    g = Gateway(name)
    with pytest.raises(RuntimeError, match="gpdla:"):
        g(1, "bogus" if name == "gpdla_mex" else np.zeros(2))


def test_engine_gateway_command_checks():
    g = Gateway("gpdla_mex")
    with pytest.raises(RuntimeError, match="gpdla:args: first argument"):
        g(1, 3.0)
    with pytest.raises(RuntimeError, match="gpdla:args: create"):
        g(1, "create", 0.0)
    with pytest.raises(RuntimeError, match="gpdla:handle"):
        g(6, "process", np.uint64(12345), [], [], [], [], np.zeros(0))
    with pytest.raises(RuntimeError, match="gpdla:handle"):
        g(0, "destroy", np.uint64(12345))


def test_engine_gateway_needs_a_device():
    if L.load().gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.parameters import set_parameters
    g = Gateway("gpdla_mex")
    with pytest.raises(RuntimeError, match="no HIP device"):
        g(1, *_create_args(syn.make_model(k=8), syn.make_samples(8), set_parameters(k=8)))


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["auto", "panel_gemm_i8_24"])
def test_engine_gateway_matches_python_engine(path):
    """gpdla_mex('create' | 'process' | 'destroy') against Engine(...).process on the same inputs:
    bitwise equal outputs, the sample matrix as MATLAB's Q x S, masked pixels given as logical."""
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    k = 20 if path == "auto" else 12
    model = syn.make_model(k=k)
    samples = syn.make_samples(96)
    spectra = syn.make_dr12q_like_spectra(model, 7, seed=4, mask_fraction=0.05)
    params = set_parameters(k=k)
    with Engine(model, samples, params, path=path) as eng:
        ref = eng.process(syn.pack_spectra(spectra))
    g = Gateway("gpdla_mex")
    (h,) = g(1, *_create_args(model, samples, params, path))
    assert g.lib.mock_locks() == 1
    outs = g(6, "process", h, [s["wavelengths"] for s in spectra], [s["flux"] for s in spectra],
             [s["noise_variance"] for s in spectra], [np.asarray(s["pixel_mask"], bool) for s in spectra],
             np.array([s["z_qso"] for s in spectra]))
    g(0, "destroy", h)
    assert g.lib.mock_locks() == 0
    names = ("log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla", "min_z_dlas",
             "max_z_dlas", "num_pixels")
    assert outs[1].shape == (7, 96)                     # MATLAB's Q x S (process_qsos.m:79)
    for name, got in zip(names, outs):
        want = np.asarray(ref[name])
        np.testing.assert_array_equal(got.reshape(want.shape), want, err_msg=name)


@pytest.mark.gpu
def test_voigt_and_mvn_gateways_match_python_bindings():
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import log_mvnpdf_low_rank, voigt
    lam = np.linspace(3700.0, 3900.0, 406)
    gv = Gateway("voigt_mex")
    for z, N, nl in ((2.1, 10 ** 20.5, 3.0), (2.05, 1e22, None)):
        args = (lam, z, N) + (() if nl is None else (nl,))
        (got,) = gv(1, *args)
        assert got.shape == (400, 1)
        np.testing.assert_array_equal(got[:, 0], voigt(lam, z, N, 31 if nl is None else int(nl)))
    with pytest.raises(RuntimeError, match="num_lines"):
        gv(1, lam, 2.1, 1e20, 40.0)
    rng = np.random.default_rng(2)
    n, k = 300, 20
    y, mu, d = rng.standard_normal(n), rng.standard_normal(n), rng.uniform(0.1, 0.5, n)
    M = syn.make_model(k=k)["M"][:n] * 3
    gm = Gateway("log_mvnpdf_low_rank_mex")
    (got,) = gm(1, y, mu, M, d)
    assert got[0, 0] == log_mvnpdf_low_rank(y, mu, M, d)


@pytest.mark.gpu
def test_objective_gateway_matches_python_binding():
    from gp_dla_detection_amd.training import Objective
    rng = np.random.default_rng(3)
    Qn, P, k = 9, 64, 4
    F = rng.standard_normal((Qn, P))
    F[rng.uniform(size=F.shape) < 0.1] = np.nan
    lya = rng.uniform(3.0, 4.0, (Qn, P))
    nv = rng.uniform(0.01, 0.1, (Qn, P))
    x = np.r_[0.1 * rng.standard_normal(P * k), np.log(0.2) + 0.1 * rng.standard_normal(P), np.log(0.1),
              np.log(0.0023), np.log(3.65)]
    obj = Objective(F, lya, nv, k)
    f_ref, g_ref = obj(x)
    obj.close()
    go = Gateway("objective_gpu_mex")
    # MATLAB passes the transposes of the num_quasars x num_pixels matrices (column-major = row-major here)
    f, g = go(2, x, F.T, lya.T, nv.T)
    assert f[0, 0] == f_ref
    np.testing.assert_array_equal(g[:, 0], g_ref)
    f2, _ = go(2, x, F.T, lya.T, nv.T)             # cached handle, same data
    assert f2[0, 0] == f_ref


# ------------------------------------------------------------------ single-precision inputs
def test_gateways_accept_single_inputs():
    """Single arrays pass the gateways' type checks (they are widened, mex_widen.h): without a
    device the call gets as far as the engine's GPDLA_EDEVICE; other classes are still refused."""
    if L.load().gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.parameters import set_parameters
    lam = np.linspace(3700.0, 3900.0, 406, dtype=np.float32)
    with pytest.raises(RuntimeError, match="no HIP device"):
        Gateway("voigt_mex")(1, lam, np.float32(2.1), 1e20)
    with pytest.raises(RuntimeError, match="must be real double or single"):
        Gateway("voigt_mex")(1, np.arange(10, dtype=np.int32), 2.1, 1e20)
    n = 40
    y = np.ones(n, np.float32)
    with pytest.raises(RuntimeError, match="no HIP device"):
        Gateway("log_mvnpdf_low_rank_mex")(1, y, y, np.ones((n, 3), np.float32), y)
    model = {k: (v.astype(np.float32) if isinstance(v, np.ndarray) else v) for k, v in syn.make_model(k=8).items()}
    with pytest.raises(RuntimeError, match="no HIP device"):
        Gateway("gpdla_mex")(1, *_create_args(model, syn.make_samples(8), set_parameters(k=8)))


def _m_call_args(text, call):
    """The argument names of the first ``call(...)`` in MATLAB source (continuations joined)."""
    import re
    src = re.sub(r"\.\.\.[^\n]*\n", " ", text)
    i = src.index(call + "(")
    depth, j = 0, i + len(call)
    while True:
        depth += {"(": 1, ")": -1}.get(src[j], 0)
        if depth == 0:
            break
        j += 1
    return [a.strip() for a in src[i + len(call) + 1:j].split(",")]


def test_process_qsos_gpu_script_matches_the_gateway():
    """matlab/process_qsos_gpu.m passes gpdla_mex('create') the arguments in the order gpdla_mex.c
    reads them (the order the GPU tests drive), 'process' the preloaded cells, and saves the 22
    variables of process_qsos.m:235-249 (process.PROCESSED_VARIABLES)."""
    import re
    from gp_dla_detection_amd.process import PROCESSED_VARIABLES
    root = Path(__file__).resolve().parents[1]
    script = (root / "matlab" / "process_qsos_gpu.m").read_text()
    create = _m_call_args(script, "gpdla_mex")
    assert create == ["'create'", "gpu_device", "rest_wavelengths", "mu", "M", "log_omega", "log_c_0", "log_tau_0",
                      "log_beta", "offset_samples", "nhi_samples", "num_lines", "width", "pixel_spacing",
                      "min_lambda", "max_lambda", "lya_wavelength", "lyman_limit", "min_z_cut", "max_z_cut",
                      "absorption_mode", "likelihood_path"]
    gateway = (root / "matlab" / "gpdla_mex.c").read_text()
    doc = gateway[gateway.index("eng = gpdla_mex('create',") + 25:gateway.index("[, absorption_mode [, path]])")]
    assert ["gpu_device"] + re.findall(r"[A-Za-z_0-9]+", doc)[1:] == create[1:20]
    proc = script[script.index("gpdla_mex('process'"):]
    assert _m_call_args(proc, "gpdla_mex") == ["'process'", "eng", "all_wavelengths", "all_flux",
                                               "all_noise_variance", "all_pixel_mask", "z_qsos"]
    saved = re.findall(r"'([a-z_0-9]+)'", script[script.index("variables_to_save = {"):script.index("};")])
    assert tuple(saved) == tuple(PROCESSED_VARIABLES) and len(saved) == 22
    for v in saved:   # every saved variable is set by the script or by set_parameters / the caller
        assert re.search(rf"\b{v}\b\s*(=|,|\])", script) or v in (
            "training_release", "training_set_name", "dla_catalog_name", "release", "test_set_name",
            "prior_z_qso_increase", "max_z_cut", "num_lines"), v


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["auto", "panel_gemm_i8_24"])
def test_engine_gateway_single_cells(path):
    """process_qsos_gpu.m's engine calls on single cells (the class of the reference's
    preloaded_qsos.mat cells): bitwise equal to the Python engine on the exactly widened doubles."""
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import Engine
    from gp_dla_detection_amd.parameters import set_parameters
    k = 20 if path == "auto" else 12
    model = syn.make_model(k=k)
    samples = syn.make_samples(80)
    spectra = syn.make_dr12q_like_spectra(model, 6, seed=8, mask_fraction=0.05)
    cells = {key: [np.asarray(s[key], np.float32) for s in spectra] for key in ("wavelengths", "flux", "noise_variance")}
    widened = [dict(wavelengths=cells["wavelengths"][q].astype(np.float64), flux=cells["flux"][q].astype(np.float64),
                    noise_variance=cells["noise_variance"][q].astype(np.float64), pixel_mask=s["pixel_mask"],
                    z_qso=s["z_qso"]) for q, s in enumerate(spectra)]
    params = set_parameters(k=k)
    with Engine(model, samples, params, path=path) as eng:
        ref = eng.process(syn.pack_spectra(widened))
    g = Gateway("gpdla_mex")
    (h,) = g(1, *_create_args(model, samples, params, path))
    outs = g(5, "process", h, cells["wavelengths"], cells["flux"], cells["noise_variance"],
             [np.asarray(s["pixel_mask"], bool) for s in spectra], np.array([s["z_qso"] for s in spectra]))
    g(0, "destroy", h)
    for name, got in zip(("log_likelihoods_no_dla", "sample_log_likelihoods_dla", "log_likelihoods_dla",
                          "min_z_dlas", "max_z_dlas"), outs):
        want = np.asarray(ref[name])
        np.testing.assert_array_equal(got.reshape(want.shape), want, err_msg=name)
    assert np.all(np.isfinite(outs[2]))


@pytest.mark.gpu
def test_voigt_and_mvn_gateways_single_inputs():
    from gp_dla_detection_amd import synthetic as syn
    from gp_dla_detection_amd.engine import log_mvnpdf_low_rank, voigt
    lam = np.linspace(3700.0, 3900.0, 406).astype(np.float32)
    (got,) = Gateway("voigt_mex")(1, lam, 2.1, 10 ** 20.5, 3.0)
    np.testing.assert_array_equal(got[:, 0], voigt(lam.astype(np.float64), 2.1, 10 ** 20.5, 3))
    rng = np.random.default_rng(5)
    n, k = 300, 20
    y, mu, d = (rng.standard_normal(n).astype(np.float32), rng.standard_normal(n).astype(np.float32),
                rng.uniform(0.1, 0.5, n).astype(np.float32))
    M = (syn.make_model(k=k)["M"][:n] * 3).astype(np.float32)
    (got,) = Gateway("log_mvnpdf_low_rank_mex")(1, y, mu, M, d)
    assert got[0, 0] == log_mvnpdf_low_rank(*(a.astype(np.float64) for a in (y, mu, M, d)))


@pytest.mark.gpu
def test_voigt_gateway_integer_class_scalars():
    """voigt.c:263-266 reads z, N and num_lines with mxGetScalar, so voigt(lam, z, N, int32(3)) and a
    logical or int32 N work with the original; the drop-in reads them the same way."""
    from gp_dla_detection_amd.engine import voigt
    lam = np.linspace(3700.0, 3900.0, 406)
    g = Gateway("voigt_mex")
    (got,) = g(1, lam, 2.1, 10 ** 20.5, np.array([3], np.int32))
    np.testing.assert_array_equal(got[:, 0], voigt(lam, 2.1, 10 ** 20.5, 3))
    (got,) = g(1, lam, np.float32(2.5), np.array([10 ** 9], np.int32), np.array([True]))
    np.testing.assert_array_equal(got[:, 0], voigt(lam, float(np.float32(2.5)), 1e9, 1))


def test_voigt_gateway_scalar_classes_without_device():
    """CPU: integer-class scalars pass the gateway's argument reading (mxGetScalar, as voigt.c:263-266)
    and reach the engine, which reports that there is no device; empty or cell scalars are refused."""
    if L.load().gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    lam = np.linspace(3700.0, 3900.0, 406)
    g = Gateway("voigt_mex")
    with pytest.raises(RuntimeError, match="no HIP device"):
        g(1, lam, 2.1, 1e20, np.array([3], np.int32))
    with pytest.raises(RuntimeError, match="num_lines must be a numeric scalar"):
        g(1, lam, 2.1, 1e20, np.zeros(0))
    with pytest.raises(RuntimeError, match="z must be a numeric scalar"):
        g(1, lam, [np.zeros(1)], 1e20)
