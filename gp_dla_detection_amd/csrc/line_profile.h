// Tabulated Voigt line profiles for the DLA absorption model.
//
// The reference evaluates, per padded pixel and Lyman line j (voigt.c:282-292),
//     V_j(v) = libcerf voigt(v, sigma, gamma_j) = Re w((v + i gamma_j) / (sigma sqrt 2)) / (sigma sqrt(2 pi))
// and accumulates  total -= lc_j * V_j(v).  With x = v / (sigma sqrt 2) and the line's fixed
// y_j = gamma_j / (sigma sqrt 2) (4.7e-4 ... 7e-8), f_j(x) = lc_j V_j is a 1-D function of x.
// A GPU lane evaluates it with 5 to 16 FMAs and no complex arithmetic:
//
//   |x| <  kCoreX : per-line piecewise polynomial (kPieces pieces of width kPieceW),
//                   u = |x| - (p + 1/2) kPieceW,   f = sum_{n <= kCoreDeg} core_j[p][n] u^n
//   |x| >= kCoreX : damping wing, T = 1/x^2 in (0, 1/kCoreX^2]:
//                   f = T * sum_{n <= kWingDeg} wing_j[n] T^n
//                   one Chebyshev fit per line of f_j(x) x^2 (smooth in T, -> lc_j y_j/pi^.5/(sigma
//                   sqrt(2 pi)) as T -> 0); the factored T keeps the RELATIVE error at rounding
//                   level however far out the wing is (max 5.6e-16 over |x| in [9, 3e7]).
//   |x| >= kOuterX: the same function fitted again on T in (0, 1/kOuterX^2] at degree kOuterDeg
//                   (max 9.9e-16 relative, 4 FMAs fewer per line): the batched sweeps evaluate it
//                   branch-free and recompute the rare lanes with |x| < kOuterX (core or wing).
//   Both wing polynomials of line j share one kWingStride block: wing at 0, outer at kOuterOff.
//
// All coefficients are fitted on the host from a long-double Faddeeva function
// (faddeeva_host.cpp) at engine creation; accuracy is checked in the tests against
// scipy.special.voigt_profile (the stand-in for libcerf).
#pragma once

#include <cmath>

#include "lyman_series.h"

#ifndef __HIPCC__
#define GPDLA_HD inline
#else
#define GPDLA_HD __host__ __device__ inline
#endif

namespace gpdla {

constexpr double kCoreX = 9.0;
constexpr double kPieceW = 0.25;
constexpr int kPieces = 36;  // kCoreX / kPieceW
constexpr int kCoreDeg = 15;
constexpr int kCoreStride = 16;  // kCoreDeg + 1
constexpr int kCoreTable = kPieces * kCoreStride;  // doubles per line
constexpr int kWingDeg = 8;      // wing polynomial degree in T
// outer wing: degree 4 on T <= 1/32^2.  A/B on configs[1] (profiles/r3e): degree 6 beyond 14,
// 5 beyond 20, 4 beyond 32 -> 78.64, 77.95, 77.40 ms (the wider fix-up zone costs less than the
// FMAs saved); degree 3 needs |x| >= 64 for 2e-15
constexpr double kOuterX = 32.0;
constexpr int kOuterDeg = 4;
constexpr int kOuterOff = 10;    // kWingDeg + 1, padded to 16-byte pairs
constexpr int kWingStride = 16;  // doubles per line: wing (10) + outer (kOuterDeg + 1, padded)

GPDLA_HD double wing_eval(const double* __restrict__ c, double x) {
  const double x2 = x * x;
#ifdef __HIP_DEVICE_COMPILE__
  // v_rcp_f64 + one Newton step: within ~1 ulp of 1/x2 (x2 >= 81, finite)
  double T = __builtin_amdgcn_rcp(x2);
  T = fma(T, fma(-x2, T, 1.0), T);
#else
  const double T = 1.0 / x2;
#endif
  double f = c[kWingDeg];
#pragma unroll
  for (int n = kWingDeg - 1; n >= 0; --n) f = fma(f, T, c[n]);
  return T * f;
}

// Damping wing from a precomputed T = 1/x^2 (the batched sweeps share one reciprocal between
// the three lines, wing_T3 in device_common.h).
GPDLA_HD double wing_poly(const double* __restrict__ c, double T) {
  double f = c[kWingDeg];
#pragma unroll
  for (int n = kWingDeg - 1; n >= 0; --n) f = fma(f, T, c[n]);
  return T * f;
}

// Outer wing (|x| >= kOuterX) from T = 1/x^2; c is the line's kWingStride block.
GPDLA_HD double outer_poly(const double* __restrict__ c, double T) {
  c += kOuterOff;
  double f = c[kOuterDeg];
#pragma unroll
  for (int n = kOuterDeg - 1; n >= 0; --n) f = fma(f, T, c[n]);
  return T * f;
}

GPDLA_HD double core_eval(const double* __restrict__ core, double ax) {
  int p = (int)(ax * (1.0 / kPieceW));
  p = p > kPieces - 1 ? kPieces - 1 : p;
  const double u = ax - (p + 0.5) * kPieceW;
  const double* c = core + p * kCoreStride;
  double f = c[kCoreDeg];
#pragma unroll
  for (int n = kCoreDeg - 1; n >= 0; --n) f = fma(f, u, c[n]);
  return f;
}

// Full evaluation (host checks and generic paths).
GPDLA_HD double line_profile_eval(const double* __restrict__ core, const double* __restrict__ wing,
                                  double x) {
  const double ax = x < 0 ? -x : x;
  return ax < kCoreX ? core_eval(core, ax) : wing_eval(wing, x);
}

}  // namespace gpdla
