// Tabulated Voigt line profiles for the DLA absorption model.
//
// The reference evaluates, per padded pixel and Lyman line j (voigt.c:282-292),
//     V_j(v) = libcerf voigt(v, sigma, gamma_j) = Re w((v + i gamma_j) / (sigma sqrt 2)) / (sigma sqrt(2 pi))
// and accumulates  total -= lc_j * V_j(v).  For a fixed line the imaginary part
// y_j = gamma_j / (sigma sqrt 2) is a constant (4.7e-4 ... 2.3e-7), so lc_j V_j is a 1-D function of
// x = v / (sigma sqrt 2).  This file defines a compact per-line representation of that function
// that a GPU lane evaluates with ~15 FMAs and no complex arithmetic:
//
//   |x| <  kCoreX : piecewise polynomial, piece p = floor(|x| / kPieceW),
//                   u = |x| - (p + 1/2) kPieceW,   f = sum_{n<=kCoreDeg} core[p][n] u^n
//   |x| >= kCoreX : damping-wing polynomial in T = 1/x^2,   f = T * sum_{n<=kWingDeg} wing[n] T^n
//
// Coefficients are fitted at engine creation (faddeeva_host.cpp) from a long-double Faddeeva
// function, and carry the lc_j / (sigma sqrt(2 pi)) scale.  Accuracy is checked in the tests
// against scipy.special.voigt_profile (the stand-in for libcerf).
#pragma once

#ifndef __HIPCC__
#define GPDLA_HD inline
#else
#define GPDLA_HD __host__ __device__ inline
#endif

namespace gpdla {

constexpr double kCoreX = 7.0;
constexpr double kPieceW = 0.25;
constexpr int kPieces = 28;  // kCoreX / kPieceW
constexpr int kCoreDeg = 15;
constexpr int kCoreStride = 16;  // kCoreDeg + 1
constexpr int kWingDeg = 13;
constexpr int kWingStride = 16;  // padded

// Per-line table: kPieces * kCoreStride core coefficients, then kWingStride wing coefficients.
constexpr int kLineTableStride = kPieces * kCoreStride + kWingStride;

GPDLA_HD double line_profile_eval(const double* __restrict__ tab, double x) {
  const double ax = x < 0 ? -x : x;
  if (ax < kCoreX) {
    int p = (int)(ax * (1.0 / kPieceW));
    p = p > kPieces - 1 ? kPieces - 1 : p;
    const double u = ax - (p + 0.5) * kPieceW;
    const double* c = tab + p * kCoreStride;
    double f = c[kCoreDeg];
#pragma unroll
    for (int n = kCoreDeg - 1; n >= 0; --n) f = f * u + c[n];
    return f;
  }
  const double T = 1.0 / (x * x);
  const double* c = tab + kPieces * kCoreStride;
  double f = c[kWingDeg];
#pragma unroll
  for (int n = kWingDeg - 1; n >= 0; --n) f = f * T + c[n];
  return f * T;
}

}  // namespace gpdla
