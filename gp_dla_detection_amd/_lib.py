"""ctypes binding of ``libgpdla.so`` (include/gpdla.h).

The library is built in-tree (``__graft_entry__.build()`` / ``python -m gp_dla_detection_amd.build``).
There is no CPU fallback: if the library is missing or no HIP device is present, compute calls
raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("GPDLA_LIB") or Path(__file__).resolve().parent / "libgpdla.so")

GPDLA_OK = 0
GPDLA_ENUMERIC = 1
GPDLA_EINVAL = -1
GPDLA_EDEVICE = -2
GPDLA_ENOMEM = -3
GPDLA_EUNSUPPORTED = -4
MEM_HOST = 0
MEM_DEVICE = 1
ABSORPTION_REFERENCE = 0
ABSORPTION_UNMASKED = 1
PATH_AUTO = 0
PATH_FUSED = 1
PATH_PANEL_GEMM = 2
PATH_FUSED_I8 = 3
PATH_PANEL_GEMM_I8 = 4
PATH_PANEL_GEMM_I8_24 = 5

dp = C.POINTER(C.c_double)
i64p = C.POINTER(C.c_int64)
u8p = C.POINTER(C.c_uint8)
i32p = C.POINTER(C.c_int32)
fp = C.POINTER(C.c_float)


class Model(C.Structure):
    _fields_ = [("num_rest", C.c_int32), ("k", C.c_int32), ("rest_wavelengths", dp), ("mu", dp),
                ("M", dp), ("log_omega", dp), ("log_c_0", C.c_double), ("log_tau_0", C.c_double),
                ("log_beta", C.c_double)]


class Samples(C.Structure):
    _fields_ = [("num_samples", C.c_int64), ("offset_samples", dp), ("nhi_samples", dp)]


class Params(C.Structure):
    _fields_ = [("num_lines", C.c_int32), ("width", C.c_int32), ("pixel_spacing", C.c_double),
                ("min_lambda", C.c_double), ("max_lambda", C.c_double),
                ("lya_wavelength", C.c_double), ("lyman_limit", C.c_double),
                ("min_z_cut", C.c_double), ("max_z_cut", C.c_double),
                ("absorption_mode", C.c_int32), ("max_batch_spectra", C.c_int32),
                ("path", C.c_int32)]


class Spectra(C.Structure):
    _fields_ = [("memory", C.c_int32), ("num_spectra", C.c_int64), ("offsets", i64p),
                ("wavelengths", dp), ("flux", dp), ("noise_variance", dp), ("pixel_mask", u8p),
                ("z_qsos", dp)]


class Results(C.Structure):
    _fields_ = [("memory", C.c_int32), ("log_likelihoods_no_dla", dp),
                ("sample_log_likelihoods_dla", dp), ("sample_ld", C.c_int64),
                ("log_likelihoods_dla", dp), ("min_z_dlas", dp), ("max_z_dlas", dp),
                ("num_pixels", i32p)]


class Stats(C.Structure):
    _fields_ = [("prep_ms", C.c_double), ("likelihood_ms", C.c_double), ("reduce_ms", C.c_double),
                ("prep_launches", C.c_int64), ("likelihood_launches", C.c_int64),
                ("reduce_launches", C.c_int64), ("spectra", C.c_int64), ("sample_evals", C.c_int64),
                ("contraction_ms", C.c_double), ("contraction_launches", C.c_int64)]


class DlaPrior(C.Structure):
    _fields_ = [("alpha", C.c_double), ("uniform_min", C.c_double), ("uniform_max", C.c_double),
                ("fit_min", C.c_double), ("fit_max", C.c_double), ("fit_upper", C.c_double)]


class PreloadParams(C.Structure):
    _fields_ = [("normalization_min_lambda", C.c_double), ("normalization_max_lambda", C.c_double),
                ("min_lambda", C.c_double), ("max_lambda", C.c_double),
                ("loading_min_lambda", C.c_double), ("loading_max_lambda", C.c_double),
                ("min_num_pixels", C.c_int32), ("brightsky_bit", C.c_int32)]


# every symbol include/gpdla.h declares, with its ctypes signature
SIGNATURES = {
    "gpdla_engine_create": (C.c_int, [C.c_int32, C.POINTER(Model), C.POINTER(Samples), C.POINTER(Params), C.POINTER(C.c_void_p)]),
    "gpdla_engine_process": (C.c_int, [C.c_void_p, C.POINTER(Spectra), C.POINTER(Results)]),
    "gpdla_engine_synchronize": (C.c_int, [C.c_void_p]),
    "gpdla_engine_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gpdla_engine_set_panel_streams": (C.c_int, [C.c_void_p, C.c_int32]),
    "gpdla_engine_use_null_stream": (C.c_int, [C.c_void_p]),
    "gpdla_engine_get_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "gpdla_engine_get_stats_n": (C.c_int, [C.c_void_p, C.POINTER(Stats), C.c_int64]),
    "gpdla_engine_reset_stats": (C.c_int, [C.c_void_p]),
    "gpdla_engine_destroy": (None, [C.c_void_p]),
    "gpdla_voigt_f64": (C.c_int, [dp, C.c_int64, C.c_double, C.c_double, C.c_int32, dp]),
    "gpdla_voigt_batch_f64": (C.c_int, [dp, C.c_int64, dp, dp, C.c_int64, C.c_int32, dp]),
    "gpdla_log_mvnpdf_low_rank_f64": (C.c_int, [dp, dp, dp, dp, C.c_int64, C.c_int32, dp]),
    "gpdla_objective_create": (C.c_int, [C.c_int32, C.c_int64, C.c_int64, C.c_int32, dp, dp, dp, C.c_int32,
                                         C.POINTER(C.c_void_p)]),
    "gpdla_objective_eval": (C.c_int, [C.c_void_p, dp, dp, dp]),
    "gpdla_objective_destroy": (None, [C.c_void_p]),
    "gpdla_spectrum_loss_f64": (C.c_int, [dp, dp, dp, dp, dp, C.c_int64, C.c_int32, C.c_double, C.c_double,
                                          C.c_double, dp, dp, dp, dp, dp, dp]),
    "gpdla_halton_rr2_f64": (C.c_int, [C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.POINTER(C.c_int32), C.c_int32, dp]),
    "gpdla_generate_dla_samples_f64": (C.c_int, [C.c_int32, dp, C.c_int64, C.c_int64, C.POINTER(DlaPrior), dp, dp, dp,
                                                 dp]),
    "gpdla_read_spec_f32": (C.c_int, [C.c_int32, C.c_int64, fp, fp, i32p, fp, fp, u8p]),
    "gpdla_preload_qsos_f32": (C.c_int, [C.c_int32, C.c_int64, i64p, fp, fp, fp, i32p, dp, C.POINTER(PreloadParams),
                                         u8p, i64p, fp, fp, fp, u8p, dp, fp]),
    "gpdla_diag_faddeeva_w": (C.c_int, [C.c_double, C.c_double, dp, dp]),
    "gpdla_diag_line_table_error": (C.c_int, [C.c_int32, dp]),
    "gpdla_diag_raw_profile3": (C.c_int, [dp, C.c_int64, C.c_double, C.c_double, C.c_int32, dp]),
    "gpdla_device_malloc": (C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_void_p)]),
    "gpdla_device_free": (C.c_int, [C.c_int32, C.c_void_p]),
    "gpdla_memcpy_htod": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64]),
    "gpdla_memcpy_dtoh": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64]),
    "gpdla_last_error": (C.c_char_p, []),
    "gpdla_version": (C.c_int32, []),
    "gpdla_last_call_kernel_ms": (C.c_int, [C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_int32)]),
    "gpdla_device_count": (C.c_int32, []),
    "gpdla_device_pci_bus_id": (C.c_int, [C.c_int32, C.c_char_p, C.c_int32]),
}

# GPDLA_ABI_VERSION of include/gpdla.h this binding is written against
ABI_VERSION = 5

_lib = None


class GpdlaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gpdla error {code}: {msg}")
        self.code = code


class GpdlaNumericError(GpdlaError):
    pass


def load() -> C.CDLL:
    """Load libgpdla.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build() "
                              "(there is no CPU fallback for the GP-DLA hot path)")
        lib = C.CDLL(str(LIB_PATH))
        missing = [name for name in SIGNATURES if getattr(lib, name, None) is None]
        if missing:
            raise ImportError(f"{LIB_PATH} lacks {', '.join(missing)}: a stale or foreign build "
                              "(rebuild with __graft_entry__.build())")
        lib.gpdla_version.restype = C.c_int32
        if lib.gpdla_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH} has ABI version {lib.gpdla_version()}, this binding needs "
                              f"{ABI_VERSION} (rebuild with __graft_entry__.build())")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def pci_bus_id(device: int) -> str:
    """PCI bus id of a HIP device (which physical GPU a rank drives)."""
    buf = C.create_string_buffer(64)
    check(load().gpdla_device_pci_bus_id(device, buf, len(buf)))
    return buf.value.decode()


def last_call_kernel_ms() -> list[float]:
    """Per-launch kernel times (ms) of this thread's last ingest / sampler call (gpdla_last_call_kernel_ms)."""
    buf = (C.c_double * 8)()
    n = C.c_int32(0)
    check(load().gpdla_last_call_kernel_ms(buf, 8, C.byref(n)))
    return [buf[i] for i in range(min(n.value, 8))]


def check(rc: int) -> int:
    if rc == GPDLA_OK:
        return rc
    msg = load().gpdla_last_error().decode(errors="replace")
    if rc == GPDLA_ENUMERIC:
        raise GpdlaNumericError(rc, msg)
    raise GpdlaError(rc, msg)


def ptr(arr, ctype=C.c_double):
    """ctypes pointer to a numpy array's data (None -> NULL)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(C.POINTER(ctype))


def dev_ptr(addr: int, ctype=C.c_double):
    """ctypes pointer from a raw device address (e.g. torch ``tensor.data_ptr()``)."""
    if addr is None:
        return None
    return C.cast(C.c_void_p(addr), C.POINTER(ctype))


class DeviceArray:
    """A device buffer owned by libgpdla (hipMalloc on the library's HIP runtime)."""

    def __init__(self, device: int, shape, dtype):
        import numpy as np
        self.device, self.shape, self.dtype = device, tuple(np.atleast_1d(shape)), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        check(load().gpdla_device_malloc(device, self.nbytes, C.byref(p)))
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, arr, device: int = 0):
        import numpy as np
        arr = np.ascontiguousarray(arr)
        out = cls(device, arr.shape, arr.dtype)
        check(load().gpdla_memcpy_htod(device, C.c_void_p(out.ptr), arr.ctypes.data_as(C.c_void_p), out.nbytes))
        return out

    def numpy(self, rows: int | None = None, start: int = 0):
        """Copy to host; ``rows`` limits the copy to that many rows from row ``start`` (C order)."""
        import numpy as np
        nrow = self.shape[0] - start if rows is None else min(rows, self.shape[0] - start)
        shape = (max(nrow, 0),) + self.shape[1:]
        out = np.empty(shape, dtype=self.dtype)
        row_bytes = int(self.nbytes // self.shape[0]) if self.shape[0] else 0
        src = C.c_void_p(int(self.ptr) + int(start) * row_bytes)
        check(load().gpdla_memcpy_dtoh(self.device, out.ctypes.data_as(C.c_void_p), src, out.nbytes))
        return out

    def free(self):
        if self.ptr:
            load().gpdla_device_free(self.device, C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
