"""C-ABI library checks that need no GPU: it loads, exports every symbol include/gpdla.h declares,
its host-side Faddeeva/table builder is accurate, and compute entry points fail loudly without a
device (there is no CPU fallback)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest
from scipy.special import wofz

from gp_dla_detection_amd import _lib as L

HEADER = Path(__file__).resolve().parents[1] / "include" / "gpdla.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(gpdla_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = L.load()
    names = declared_functions()
    assert len(names) >= 14
    for name in names:
        assert hasattr(lib, name), name
        assert name in L.SIGNATURES, f"{name} missing from the ctypes binding"
    assert lib.gpdla_version() == L.ABI_VERSION == 5   # 2: gpdla_stats grew; 3: pci bus id; 4: samples + ingest; 5: kernel times


def test_faddeeva_host_matches_scipy():
    lib = L.load()
    re_, im_ = C.c_double(), C.c_double()
    xs = np.concatenate([np.linspace(0, 12, 241), np.geomspace(12.01, 2e4, 60), -np.linspace(0.1, 9, 17)])
    for y in (4.717e-4, 1.205e-4, 4.895e-5, 0.0, 0.3):
        for x in xs:
            assert lib.gpdla_diag_faddeeva_w(x, y, C.byref(re_), C.byref(im_)) == 0
            ref = wofz(x + 1j * y)
            assert abs(re_.value - ref.real) <= 2e-14 * abs(ref.real) + 1e-27, (x, y)
            assert abs(im_.value - ref.imag) <= 2e-14 * abs(ref.imag) + 1e-300, (x, y)


@pytest.mark.parametrize("line", list(range(31)))
def test_line_tables_accurate(line):
    err = C.c_double()
    assert L.load().gpdla_diag_line_table_error(line, C.byref(err)) == 0
    assert err.value < 2e-15  # measured max over all 31 lines: 5.5e-16


def test_no_cpu_fallback_without_device():
    lib = L.load()
    if lib.gpdla_device_count() > 0:
        pytest.skip("a HIP device is present")
    lam = np.linspace(3600, 3700, 20)
    out = np.zeros(14)
    rc = lib.gpdla_voigt_f64(L.ptr(lam), 20, 2.0, 1e20, 3, L.ptr(out))
    assert rc == L.GPDLA_EDEVICE
    raw = np.zeros(20)
    assert lib.gpdla_diag_raw_profile3(L.ptr(lam), 20, 2.0, 1e20, 1, L.ptr(raw)) == L.GPDLA_EDEVICE
    with pytest.raises(L.GpdlaError):
        L.pci_bus_id(0)
    assert b"no HIP device" in lib.gpdla_last_error()
    from gp_dla_detection_amd.engine import log_mvnpdf_low_rank
    with pytest.raises(L.GpdlaError):
        log_mvnpdf_low_rank(np.ones(5), np.zeros(5), np.ones((5, 2)), np.ones(5))


def test_invalid_arguments_rejected():
    lib = L.load()
    out = np.zeros(4)
    lam = np.linspace(3600, 3700, 10)
    assert lib.gpdla_voigt_f64(L.ptr(lam), 10, 2.0, 1e20, 0, L.ptr(out)) == L.GPDLA_EINVAL
    assert lib.gpdla_voigt_f64(L.ptr(lam), 10, 2.0, 1e20, 32, L.ptr(out)) == L.GPDLA_EINVAL
    assert lib.gpdla_voigt_f64(L.ptr(lam), 6, 2.0, 1e20, 3, L.ptr(out)) == L.GPDLA_EINVAL
