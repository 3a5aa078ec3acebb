"""Python handle on the native engine (``gpdla_engine_*`` in include/gpdla.h)."""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib as L
from .parameters import Parameters, set_parameters


def _model_struct(model: dict, keep: list) -> L.Model:
    lam = np.ascontiguousarray(model["rest_wavelengths"], dtype=np.float64).ravel()
    mu = np.ascontiguousarray(model["mu"], dtype=np.float64).ravel()
    M = np.asfortranarray(model["M"], dtype=np.float64)
    lom = np.ascontiguousarray(model["log_omega"], dtype=np.float64).ravel()
    if M.shape[0] != lam.size or mu.size != lam.size or lom.size != lam.size:
        raise ValueError("model arrays disagree on the rest-grid size")
    Mflat = M.ravel(order="F")  # MATLAB column-major
    keep += [lam, mu, Mflat, lom]
    return L.Model(num_rest=lam.size, k=M.shape[1], rest_wavelengths=L.ptr(lam), mu=L.ptr(mu),
                   M=L.ptr(Mflat), log_omega=L.ptr(lom), log_c_0=float(np.ravel(model["log_c_0"])[0]),
                   log_tau_0=float(np.ravel(model["log_tau_0"])[0]),
                   log_beta=float(np.ravel(model["log_beta"])[0]))


_PATHS = {"auto": L.PATH_AUTO, "fused": L.PATH_FUSED, "panel_gemm": L.PATH_PANEL_GEMM,
          "fused_i8": L.PATH_FUSED_I8, "panel_gemm_i8": L.PATH_PANEL_GEMM_I8,
          "panel_gemm_i8_24": L.PATH_PANEL_GEMM_I8_24}


def _params_struct(p: Parameters, max_batch_spectra: int = 0, path: str = "auto") -> L.Params:
    return L.Params(num_lines=p.num_lines, width=p.width, pixel_spacing=p.pixel_spacing,
                    min_lambda=p.min_lambda, max_lambda=p.max_lambda,
                    lya_wavelength=p.lya_wavelength, lyman_limit=p.lyman_limit,
                    min_z_cut=p.min_z_cut, max_z_cut=p.max_z_cut,
                    absorption_mode=(L.ABSORPTION_REFERENCE if p.absorption_mode == "reference"
                                     else L.ABSORPTION_UNMASKED),
                    max_batch_spectra=max_batch_spectra, path=_PATHS[path])


def host_empty(shape: tuple, dtype=np.float64) -> np.ndarray:
    """An uninitialised host array for outputs the engine writes in full: the 13 GB full-DR12Q Q x S
    sample array is not NaN-filled first (a whole extra pass over it; the D2H copies touch each page
    once).  From 256 MB up it is an anonymous map advised for transparent huge pages where the host
    enables them (fewer first-touch faults)."""
    import math
    import mmap
    nbytes = math.prod(shape) * np.dtype(dtype).itemsize
    if nbytes < (1 << 28):
        return np.empty(shape, dtype=dtype)
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m.madvise(mmap.MADV_HUGEPAGE)
    except (AttributeError, OSError):  # no THP on this host: plain pages
        pass
    return np.frombuffer(m, dtype=dtype).reshape(shape)


class Engine:
    """One engine per device: resident model, DLA samples and line-profile tables.

    ``path``: "auto" (fused single-kernel sweep for ranks 1..24 -- compiled for 4 8 10 12 16 20 24, a
    rank in between runs on the next one with M zero-padded, exactly -- else the panel-GEMM path),
    "fused", or "panel_gemm" (weights kernel + dgemm + batched LDL^T; ranks 1..64)."""

    def __init__(self, model: dict, samples: dict, params: Parameters | None = None,
                 device: int = 0, max_batch_spectra: int = 0, path: str = "auto"):
        self.lib = L.load()
        self.params = params or set_parameters(k=np.asarray(model["M"]).shape[1])
        if self.params.k != np.asarray(model["M"]).shape[1]:
            raise ValueError("params.k disagrees with the model's M")
        keep: list = []
        ms = _model_struct(model, keep)
        off = np.ascontiguousarray(samples["offset_samples"], dtype=np.float64).ravel()
        nhi = np.ascontiguousarray(samples["nhi_samples"], dtype=np.float64).ravel()
        if off.size != nhi.size:
            raise ValueError("offset_samples and nhi_samples differ in length")
        ss = L.Samples(num_samples=off.size, offset_samples=L.ptr(off), nhi_samples=L.ptr(nhi))
        if path not in _PATHS:
            raise ValueError(f"path must be one of {sorted(_PATHS)}")
        ps = _params_struct(self.params, max_batch_spectra, path)
        h = C.c_void_p()
        L.check(self.lib.gpdla_engine_create(device, C.byref(ms), C.byref(ss), C.byref(ps), C.byref(h)))
        self._h = h
        self.num_samples = off.size
        self.device = device

    # -------------------------------------------------------------------------------- host path
    def process(self, packed: dict, want_samples: bool = True, raise_numeric: bool = False,
                timings: dict | None = None) -> dict:
        """Run the hot path on CSR-packed host spectra (see synthetic.pack_spectra).  ``timings``
        (optional) receives the host output allocation and the engine call times."""
        t0 = time.perf_counter()
        offsets = np.ascontiguousarray(packed["offsets"], dtype=np.int64)
        Q = offsets.size - 1
        wl = np.ascontiguousarray(packed["wavelengths"], dtype=np.float64)
        fl = np.ascontiguousarray(packed["flux"], dtype=np.float64)
        nv = np.ascontiguousarray(packed["noise_variance"], dtype=np.float64)
        mk = np.ascontiguousarray(packed["pixel_mask"], dtype=np.uint8)
        zq = np.ascontiguousarray(packed["z_qsos"], dtype=np.float64)
        if not (wl.size == fl.size == nv.size == mk.size and offsets[-1] <= wl.size and zq.size == Q):
            raise ValueError("inconsistent spectra arrays")
        out = dict(log_likelihoods_no_dla=np.full(Q, np.nan), log_likelihoods_dla=np.full(Q, np.nan),
                   min_z_dlas=np.full(Q, np.nan), max_z_dlas=np.full(Q, np.nan),
                   num_pixels=np.zeros(Q, dtype=np.int32))
        if want_samples:  # every row is written by the engine (NaN rows for unusable spectra)
            out["sample_log_likelihoods_dla"] = host_empty((Q, self.num_samples))
        sp = L.Spectra(memory=L.MEM_HOST, num_spectra=Q, offsets=L.ptr(offsets, C.c_int64),
                       wavelengths=L.ptr(wl), flux=L.ptr(fl), noise_variance=L.ptr(nv),
                       pixel_mask=L.ptr(mk, C.c_uint8), z_qsos=L.ptr(zq))
        sll = out.get("sample_log_likelihoods_dla")
        rs = L.Results(memory=L.MEM_HOST, log_likelihoods_no_dla=L.ptr(out["log_likelihoods_no_dla"]),
                       sample_log_likelihoods_dla=L.ptr(sll), sample_ld=self.num_samples,
                       log_likelihoods_dla=L.ptr(out["log_likelihoods_dla"]),
                       min_z_dlas=L.ptr(out["min_z_dlas"]), max_z_dlas=L.ptr(out["max_z_dlas"]),
                       num_pixels=L.ptr(out["num_pixels"], C.c_int32))
        t1 = time.perf_counter()
        rc = self.lib.gpdla_engine_process(self._h, C.byref(sp), C.byref(rs))
        if timings is not None:
            timings["host_alloc_s"] = t1 - t0
            timings["engine_process_s"] = time.perf_counter() - t1
        if rc == L.GPDLA_ENUMERIC and not raise_numeric:
            out["numeric_warning"] = self.lib.gpdla_last_error().decode()
        else:
            L.check(rc)
        return out

    # ------------------------------------------------------------------------- device path
    def process_device(self, offsets: np.ndarray, wl_ptr: int, flux_ptr: int, noise_ptr: int,
                       mask_ptr: int, z_ptr: int, ll_null_ptr: int, ll_dla_ptr: int,
                       sample_ptr: int | None = None, sample_ld: int = 0,
                       zmin_ptr: int | None = None, zmax_ptr: int | None = None,
                       npix_ptr: int | None = None) -> None:
        """Enqueue the hot path on device-resident inputs/outputs (raw device addresses).
        ``offsets`` is host int64 [Q+1].  Returns after enqueueing; call ``synchronize()``."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self._keep_offsets = offsets
        Q = offsets.size - 1
        sp = L.Spectra(memory=L.MEM_DEVICE, num_spectra=Q, offsets=L.ptr(offsets, C.c_int64),
                       wavelengths=L.dev_ptr(wl_ptr), flux=L.dev_ptr(flux_ptr),
                       noise_variance=L.dev_ptr(noise_ptr), pixel_mask=L.dev_ptr(mask_ptr, C.c_uint8),
                       z_qsos=L.dev_ptr(z_ptr))
        rs = L.Results(memory=L.MEM_DEVICE, log_likelihoods_no_dla=L.dev_ptr(ll_null_ptr),
                       sample_log_likelihoods_dla=L.dev_ptr(sample_ptr), sample_ld=sample_ld or self.num_samples,
                       log_likelihoods_dla=L.dev_ptr(ll_dla_ptr), min_z_dlas=L.dev_ptr(zmin_ptr),
                       max_z_dlas=L.dev_ptr(zmax_ptr), num_pixels=L.dev_ptr(npix_ptr, C.c_int32))
        L.check(self.lib.gpdla_engine_process(self._h, C.byref(sp), C.byref(rs)))

    def synchronize(self) -> None:
        L.check(self.lib.gpdla_engine_synchronize(self._h))

    def set_stream(self, stream_handle: int | None) -> None:
        """Order the engine's kernels on an external hipStream_t handle (e.g. torch's
        ``current_stream().cuda_stream``).  Handle 0 is the null stream (torch's default stream,
        gpdla_engine_use_null_stream), since the C ABI reads a NULL handle as "restore".  None restores
        the engine's own stream, as ``restore_stream()`` does; before round 6, 0 meant "restore" too, so a
        caller passing 0 for that now gets the null stream -- a warning says so."""
        if stream_handle == 0:
            import warnings
            warnings.warn("Engine.set_stream(0) selects the null stream (torch's default stream); use "
                          "restore_stream() or set_stream(None) for the engine's own stream", stacklevel=2)
            L.check(self.lib.gpdla_engine_use_null_stream(self._h))
        elif stream_handle is None:
            self.restore_stream()
        else:
            L.check(self.lib.gpdla_engine_set_stream(self._h, C.c_void_p(stream_handle)))

    def restore_stream(self) -> None:
        """Back to the engine's own (non-blocking) stream."""
        L.check(self.lib.gpdla_engine_set_stream(self._h, C.c_void_p(0)))

    def set_panel_streams(self, n: int) -> None:
        """Panel-GEMM paths: spectra of a batch alternate over n (1..4) compute streams."""
        L.check(self.lib.gpdla_engine_set_panel_streams(self._h, int(n)))

    def stats(self) -> dict:
        s = L.Stats()
        L.check(self.lib.gpdla_engine_get_stats(self._h, C.byref(s)))
        return {name: getattr(s, name) for name, _ in L.Stats._fields_}

    def reset_stats(self) -> None:
        L.check(self.lib.gpdla_engine_reset_stats(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.gpdla_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def voigt(lambdas, z, N, num_lines=31) -> np.ndarray:
    """MEX ``voigt(lambdas, z, N, num_lines)`` (voigt.c:253-304) on the GPU."""
    lib = L.load()
    lam = np.ascontiguousarray(lambdas, dtype=np.float64).ravel()
    out = np.empty(lam.size - 6)
    L.check(lib.gpdla_voigt_f64(L.ptr(lam), lam.size, float(z), float(N), int(num_lines), L.ptr(out)))
    return out


def voigt_batch(lambdas, zs, Ns, num_lines=31) -> np.ndarray:
    lib = L.load()
    lam = np.ascontiguousarray(lambdas, dtype=np.float64).ravel()
    zs = np.ascontiguousarray(zs, dtype=np.float64).ravel()
    Ns = np.ascontiguousarray(Ns, dtype=np.float64).ravel()
    out = np.empty((zs.size, lam.size - 6))
    L.check(lib.gpdla_voigt_batch_f64(L.ptr(lam), lam.size, L.ptr(zs), L.ptr(Ns), zs.size,
                                      int(num_lines), L.ptr(out)))
    return out


def log_mvnpdf_low_rank(y, mu, M, d) -> float:
    """``log_mvnpdf_low_rank(y, mu, M, d)`` (log_mvnpdf_low_rank.m:5-33) on the GPU."""
    lib = L.load()
    y = np.ascontiguousarray(y, dtype=np.float64).ravel()
    mu = np.ascontiguousarray(mu, dtype=np.float64).ravel()
    d = np.ascontiguousarray(d, dtype=np.float64).ravel()
    M = np.asarray(M, dtype=np.float64)
    if M.ndim == 1:
        M = M[:, None]
    n, k = M.shape
    Mf = np.asfortranarray(M).ravel(order="F")
    out = np.empty(1)
    L.check(lib.gpdla_log_mvnpdf_low_rank_f64(L.ptr(y), L.ptr(mu), L.ptr(Mf), L.ptr(d), n, k, L.ptr(out)))
    return float(out[0])
