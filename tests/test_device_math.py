"""Host emulation of the fused sweep's scalar device math (device_common.h), IEEE-exact per operation:
exp_tab128_nc (128-entry 2^(j/128) table, degree-4 minimax polynomial, no clamp) and batch_rcp4
(four reciprocals from one, Montgomery's trick).  The constants are read from the header itself, so
a change there is checked here without a GPU.  The GPU suite checks the kernels end to end against
the oracle (tests/test_gpu_*.py)."""
import math
import re
from fractions import Fraction
from pathlib import Path

import numpy as np
import pytest

HDR = (Path(__file__).resolve().parents[1] / "gp_dla_detection_amd" / "csrc" / "device_common.h").read_text()


def _fma(a, b, c):
    """Correctly rounded a * b + c (exact rational arithmetic, one rounding)."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _exp128_constants():
    body = HDR[HDR.index("__device__ inline double exp_tab128_nc"):]
    body = body[:body.index("\n}\n")]
    num = r"(0x[0-9a-fA-Fp.+-]+|[0-9.]+(?:e[+-]?[0-9]+)?)"
    def val(name):
        s = re.search(rf"{name} = {num};", body).group(1)
        return float.fromhex(s) if s.startswith("0x") else float(s)
    poly = re.findall(r"fma\(r, ([0-9.e-]+), ([0-9.e-]+)\)", body)[0]
    rest = re.findall(r"fma\(p, r, ([0-9.e-]+)\)", body)
    return val("kInvL"), val("kLhi"), val("kLlo"), [float(poly[0]), float(poly[1])] + [float(x) for x in rest]


def _exp128(v, tab, kInvL, kLhi, kLlo, c):
    kd = _fma(v, kInvL, float.fromhex("0x1.8p52"))
    ki = int(Fraction(kd) - Fraction(float.fromhex("0x1.8p52")))   # the low word, as an int
    k = kd - float.fromhex("0x1.8p52")
    r = _fma(-k, kLhi, v)
    r = _fma(-k, kLlo, r)
    p = _fma(r, c[0], c[1])
    for ci in c[2:]:
        p = _fma(p, r, ci)
    return math.ldexp(p * tab[ki & 127], ki >> 7)


def test_exp_tab128_nc_accuracy():
    kInvL, kLhi, kLlo, c = _exp128_constants()
    assert len(c) == 5 and kInvL == pytest.approx(128 / math.log(2), rel=1e-15)
    # the split of ln2/128: kLhi exact for |k| < 2^20 (33 significant bits), kLhi + kLlo = ln2/128
    assert Fraction(kLhi).numerator.bit_length() <= 33
    assert abs(kLhi + kLlo - math.log(2) / 128) < 1e-30
    tab = [2.0 ** (j / 128) for j in range(128)]   # engine.hip rounds 2^(j/128) from long double
    rng = np.random.default_rng(0)
    worst = 0.0
    for v in np.concatenate([-rng.random(3000) * 745.0, -rng.random(1000) * 1e-3, [0.0, -1e-300]]):
        got = _exp128(float(v), tab, kInvL, kLhi, kLlo, c)
        ref = math.exp(v)
        worst = max(worst, abs(got - ref) / ref)
    assert worst < 6e-16, worst            # a few ulp (table and polynomial rounding)
    # past -745 the result underflows to +0 like exp, down to the bound the sweep guarantees
    for v in (-750.0, -1100.0, -1e5, -1.1e7):
        assert _exp128(v, tab, kInvL, kLhi, kLlo, c) == 0.0


def test_batch_rcp4_matches_four_reciprocals():
    """batch_rcp4: 1/q_i from one Newton-refined reciprocal of q_0 q_1 q_2 q_3 (v_rcp_f64 modelled as
    1/P with a 2^-26 relative error, its documented accuracy)."""
    rng = np.random.default_rng(1)
    worst = 0.0
    for _ in range(2000):
        q = [float(x) for x in 10.0 ** rng.uniform(-15, 15, 4)]
        q01, q23 = q[0] * q[1], q[2] * q[3]
        P = q01 * q23
        R = (1.0 / P) * (1.0 + rng.uniform(-1, 1) * 2.0 ** -26)
        R = _fma(R, _fma(-P, R, 1.0), R)
        R23, R01 = R * q23, R * q01
        iq = [R23 * q[1], R23 * q[0], R01 * q[3], R01 * q[2]]
        for qi, ii in zip(q, iq):
            worst = max(worst, abs(ii * qi - 1.0))
    assert worst < 1e-15, worst
