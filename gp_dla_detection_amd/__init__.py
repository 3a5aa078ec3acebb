"""gp_dla_detection_amd -- MI355X-native GP DLA-detection likelihood engine.

The hot path of sbird/gp_dla_detection (process_qsos.m's per-sample Voigt absorption x
log_mvnpdf_low_rank) runs as hand-written HIP kernels for gfx950 in
libgpdla.so, behind the C ABI in include/gpdla.h.  This package is the Python host that mirrors
the reference's call surface (set_parameters / process_qsos / .mat output).
"""
from .parameters import Parameters, set_parameters  # noqa: F401

__all__ = ["Parameters", "set_parameters", "Engine", "process_qsos", "save_processed_qsos",
           "voigt", "voigt_batch", "log_mvnpdf_low_rank"]


def __getattr__(name):
    if name in ("Engine", "voigt", "voigt_batch", "log_mvnpdf_low_rank"):
        from . import engine
        return getattr(engine, name)
    if name in ("process_qsos", "save_processed_qsos"):
        from . import process
        return getattr(process, name)
    raise AttributeError(name)
