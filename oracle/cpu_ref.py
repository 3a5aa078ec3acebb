"""ctypes binding of oracle/liboracle_cpu.so (oracle/cpu_ref.cpp, built by oracle/Makefile) --
TEST INFRASTRUCTURE AND CPU BASELINE ONLY (tests/, smoke(), bench.py's cpu_baseline leg).

The C++ OpenMP restatement of process_qsos.m:184-198 + voigt.c:253-304 +
log_mvnpdf_low_rank.m:5-33 in MATLAB operation order; the per-spectrum preparation comes from
the numpy oracle (gpdla_oracle.prepare_spectrum)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle_cpu.so"
_lib = None
dp = C.POINTER(C.c_double)


def build(force: bool = False) -> Path:
    src = HERE / "cpu_ref.cpp"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(str(LIB))
        lib.gpdla_cpu_threads.restype = C.c_int
        lib.gpdla_cpu_voigt.argtypes = [dp, C.c_int64, C.c_double, C.c_double, C.c_int32, dp]
        lib.gpdla_cpu_faddeeva_w.argtypes = [C.c_double, C.c_double, dp, dp]
        lib.gpdla_cpu_log_mvnpdf_low_rank.argtypes = [dp, dp, dp, dp, C.c_int64, C.c_int32, dp]
        lib.gpdla_cpu_sample_lls.argtypes = [C.c_int64, C.c_int32, dp, dp, dp, dp, dp, C.c_int64, dp,
                                             C.POINTER(C.c_int64), C.c_double, C.c_double, C.c_int64, dp, dp,
                                             C.c_int32, C.c_int32, dp]
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(dp)


def threads() -> int:
    return int(load().gpdla_cpu_threads())


def faddeeva_w(x: float, y: float) -> complex:
    re, im = C.c_double(), C.c_double()
    load().gpdla_cpu_faddeeva_w(float(x), float(y), C.byref(re), C.byref(im))
    return complex(re.value, im.value)


def voigt(lambdas, z, N, num_lines=31) -> np.ndarray:
    lam = np.ascontiguousarray(lambdas, dtype=np.float64)
    out = np.empty(lam.size - 6)
    if load().gpdla_cpu_voigt(_p(lam), lam.size, float(z), float(N), int(num_lines), _p(out)):
        raise ValueError("bad voigt arguments")
    return out


def log_mvnpdf_low_rank(y, mu, M, d) -> float:
    y, mu, d = (np.ascontiguousarray(a, dtype=np.float64) for a in (y, mu, d))
    M = np.asarray(M, dtype=np.float64)
    n, k = M.shape
    Mf = np.ascontiguousarray(M.ravel(order="F"))
    out = np.empty(1)
    load().gpdla_cpu_log_mvnpdf_low_rank(_p(y), _p(mu), _p(Mf), _p(d), n, k, _p(out))
    return float(out[0])


def sample_lls(prep: dict, offsets, nhi, num_lines: int = 3, nthreads: int = 0) -> np.ndarray:
    """All sample log-likelihoods of one prepared spectrum (gpdla_oracle.prepare_spectrum)."""
    y, noise, mu, om2 = (np.ascontiguousarray(prep[k], dtype=np.float64) for k in ("y", "noise", "mu", "omega2"))
    M = np.ascontiguousarray(np.asarray(prep["M"], dtype=np.float64).ravel(order="F"))
    pad = np.ascontiguousarray(prep["padded"], dtype=np.float64)
    aind = np.ascontiguousarray(prep["absorption_index"], dtype=np.int64)
    off = np.ascontiguousarray(offsets, dtype=np.float64)
    nh = np.ascontiguousarray(nhi, dtype=np.float64)
    n, k = np.asarray(prep["M"]).shape
    out = np.empty(off.size)
    load().gpdla_cpu_sample_lls(n, k, _p(y), _p(noise), _p(mu), _p(M), _p(om2), int(prep["m"]), _p(pad),
                                aind.ctypes.data_as(C.POINTER(C.c_int64)), float(prep["zmin"]),
                                float(prep["zmax"]), off.size, _p(off), _p(nh), int(num_lines), int(nthreads),
                                _p(out))
    return out
