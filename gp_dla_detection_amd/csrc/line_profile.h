// Tabulated Voigt line profiles for the DLA absorption model.
//
// The reference evaluates, per padded pixel and Lyman line j (voigt.c:282-292),
//     V_j(v) = libcerf voigt(v, sigma, gamma_j) = Re w((v + i gamma_j) / (sigma sqrt 2)) / (sigma sqrt(2 pi))
// and accumulates  total -= lc_j * V_j(v).  With x = v / (sigma sqrt 2) and the line's fixed
// y_j = gamma_j / (sigma sqrt 2) (4.7e-4 ... 7e-8), f_j(x) = lc_j V_j is a 1-D function of x.
// A GPU lane evaluates it with ~20 FMAs and no complex arithmetic:
//
//   |x| <  kCoreX : per-line piecewise polynomial (kPieces pieces of width kPieceW),
//                   u = |x| - (p + 1/2) kPieceW,   f = sum_{n <= kCoreDeg} core_j[p][n] u^n
//   |x| >= kCoreX : damping wing, T = 1/x^2:
//                   f = A_j T (g(T) + B_j T h(T)),  A_j = lc_j y_j / (sigma sqrt(2 pi)),  B_j = y_j^2
//                   where g, h are UNIVERSAL (line-independent): Re w(x+iy) x^2 / y = g(T) + y^2 T h(T)
//                   + O(y^4 T^2) (the O term is < 1e-17 relative for every Lyman line here).
//
// All coefficients are fitted on the host from a long-double Faddeeva function
// (faddeeva_host.cpp) at engine creation; accuracy is checked in the tests against
// scipy.special.voigt_profile (the stand-in for libcerf).
#pragma once

#include <cmath>

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
constexpr int kWingG = 10;  // g coefficients (degree 9 in T)
constexpr int kWingH = 5;   // h coefficients (degree 4 in T)

// Everything the lane needs besides the per-line core table, passed by value (SGPRs).
struct WingPoly {
  double g[kWingG];
  double h[kWingH];
};

GPDLA_HD double wing_eval(const WingPoly& w, double A, double B, double x) {
  const double x2 = x * x;
#ifdef __HIP_DEVICE_COMPILE__
  // v_rcp_f64 + one Newton step: within ~1 ulp of 1/x2 (x2 >= 81, finite)
  double T = __builtin_amdgcn_rcp(x2);
  T = fma(T, fma(-x2, T, 1.0), T);
#else
  const double T = 1.0 / x2;
#endif
  double g = w.g[kWingG - 1];
#pragma unroll
  for (int n = kWingG - 2; n >= 0; --n) g = fma(g, T, w.g[n]);
  double h = w.h[kWingH - 1];
#pragma unroll
  for (int n = kWingH - 2; n >= 0; --n) h = fma(h, T, w.h[n]);
  const double G = fma(B * T, h, g);
  return (A * T) * G;
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
GPDLA_HD double line_profile_eval(const double* __restrict__ core, const WingPoly& w, double A,
                                  double B, double x) {
  const double ax = x < 0 ? -x : x;
  return ax < kCoreX ? core_eval(core, ax) : wing_eval(w, A, B, x);
}

}  // namespace gpdla
