"""CPU checks of the int8 Ozaki digit scheme used by kernels_i8.hip / gemm_i8.hip (DESIGN.md
section 10): the digit identities are exact, the balanced panel digits stay in int8 range, and the
level <= 3 truncation error stays inside its bound.  Pure integer arithmetic (Python ints)."""
import numpy as np

from support.emulate_i8 import digits_balanced


def offset_digits(U):
    """Weights: X_A + offset read as 4 bytes, XOR 0x80 -> signed digits d_i = b_i - 128."""
    return [((U >> (8 * (3 - i))) & 255) - 128 for i in range(4)]


def test_balanced_digits_are_exact_and_in_range():
    rng = np.random.default_rng(0)
    X = rng.integers(-127 * 2 ** 24, 127 * 2 ** 24 + 1, size=20000, dtype=np.int64)
    X = np.concatenate([X, [0, 127 * 2 ** 24, -127 * 2 ** 24, 1, -1, 128, -128, 2 ** 24 - 1]])
    d = digits_balanced(X)
    for di in d:
        assert di.min() >= -128 and di.max() <= 127
    rebuilt = sum(di.astype(object) * (2 ** (8 * (3 - i))) for i, di in enumerate(d))
    assert np.array_equal(rebuilt.astype(np.int64), X)


def test_pair_sum_identity_exact_for_gram_and_u_offsets():
    """sum_slot X_A X_B = sum_{i,j} 2^(8(6-i-j)) sum_slot dA_i dB_j + c * sum_slot X_B, with
    c = 0x80808080 for unsigned Gram weights (X_A = U) and 0x808080 for u (X_A = U - 2^31)."""
    rng = np.random.default_rng(1)
    n = 777
    XB = rng.integers(-127 * 2 ** 24, 127 * 2 ** 24 + 1, size=n, dtype=np.int64)
    dB = digits_balanced(XB)
    for signed in (False, True):
        if signed:
            XA = rng.integers(-(2 ** 31 - 256), 2 ** 31 - 256, size=n, dtype=np.int64)
            U = XA + 2 ** 31
            c = 0x808080
        else:
            U = XA = rng.integers(0, 2 ** 32 - 256, size=n, dtype=np.int64)
            c = 0x80808080
        dA = offset_digits(U)
        exact = int(sum(int(a) * int(b) for a, b in zip(XA, XB)))
        total = sum((2 ** (8 * (6 - i - j))) * int(np.dot(dA[i].astype(object), dB[j].astype(object)))
                    for i in range(4) for j in range(4))
        total += c * int(XB.sum())
        assert total == exact


def test_level3_truncation_bound_and_int32_level_sums():
    """Dropping the digit pairs of level >= 4 changes each slot's product by at most
    3 * 2^8 * 128^2 + 2 * 128^2 + 128^2 (levels 4..6) relative to 2^60-scale operands, and the
    kept level sums stay exact in int32 up to the kI8MaxSlots = 30,000 slot bound."""
    bound_per_slot = (3 * 2 ** 16 + 2 * 2 ** 8 + 1) * 128 ** 2
    assert bound_per_slot / 2.0 ** 60 < 2 ** -28
    # level l has at most 4 digit pairs, each |dA dB| <= 2^14
    assert 4 * 30000 * 2 ** 14 < 2 ** 31
    rng = np.random.default_rng(2)
    n = 500
    XB = rng.integers(-127 * 2 ** 24, 127 * 2 ** 24 + 1, size=n, dtype=np.int64)
    U = rng.integers(0, 2 ** 32 - 256, size=n, dtype=np.int64)
    dA, dB = offset_digits(U), digits_balanced(XB)
    full = sum((2 ** (8 * (6 - i - j))) * int(np.dot(dA[i].astype(object), dB[j].astype(object)))
               for i in range(4) for j in range(4))
    kept = sum((2 ** (8 * (6 - i - j))) * int(np.dot(dA[i].astype(object), dB[j].astype(object)))
               for i in range(4) for j in range(4) if i + j <= 3)
    assert abs(full - kept) <= n * bound_per_slot


def test_fp32_raw_profile_adds_little_to_the_24_bit_scheme():
    """The 24-bit panel path evaluates its weights' raw Voigt profiles in packed fp32 (gemm_i8.hip
    raw_profile3_pair_f32; x_j stays fp64).  Emulated on configs[4]-shaped spectra (k = 50, 10^5
    samples): against the fp64 oracle the fp32 profiles add less than 5e-8 to the scheme's own
    log-likelihood error, which stays under 2e-7 (the GPU tests' bar is 5e-7)."""
    from gp_dla_detection_amd import synthetic as syn
    from support.emulate_f32_profile import worst_errors
    model = syn.make_model(k=50)
    samples = syn.make_samples(100000)
    rng = np.random.default_rng(3)
    spectra = [syn.make_spectrum(model, q) for q in range(2)]
    picks = [(q, int(s)) for q in range(2) for s in rng.choice(100000, 6, replace=False)]
    w = worst_errors(model, spectra, samples, picks)
    assert w["f64"] < 2e-7
    assert w["f32"] - w["f64"] < 5e-8
    assert w["f32"] < 2e-7
