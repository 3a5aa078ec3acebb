// Device helpers shared by the fused path (kernels.hip) and the panel-GEMM path (gemm_path.hip):
// constants, block scans/reductions, model interpolation, the Voigt raw profile (voigt.c:282-292)
// and the table exp.  Header-only, internal linkage per translation unit.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "internal.h"

namespace gpdla {

namespace {

constexpr double kLog2Pi = 1.83787706640934534;  // log_mvnpdf_low_rank.m:7
constexpr double kLn2 = 0.693147180559945309417;

// ---------------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------------
__device__ inline double rcp_nr(double d) {
  // v_rcp_f64 (~2^-26) refined by two Newton steps -> within 1 ulp of 1/d
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// 1/d in the per-pixel sweeps (d = omega^2 a^2 + sigma^2 > 0, finite): v_rcp_f64 (~2^-26) and one
// Newton step (error ~2^-52, i.e. within a couple of ulp; the sums over n pixels are insensitive)
__device__ inline double rcp_sweep(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}

// 1/q_0 .. 1/q_3 from ONE v_rcp_f64 (+ Newton step) of the product q_0 q_1 q_2 q_3 (Montgomery's
// trick): the same instruction count as four rcp_sweep, three fewer quarter-rate reciprocals.  The
// product must stay a normal double (callers bound their q_i).
__device__ inline void batch_rcp4(const double (&q)[4], double (&iq)[4]) {
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double P = q01 * q23;
  double R = __builtin_amdgcn_rcp(P);
  R = fma(R, fma(-P, R, 1.0), R);
  const double R23 = R * q23, R01 = R * q01;
  iq[0] = R23 * q[1];
  iq[1] = R23 * q[0];
  iq[2] = R01 * q[3];
  iq[3] = R01 * q[2];
}

// batch_rcp4 for unbounded positive q_i (the per-pixel d = omega^2 a^2 + sigma^2): P = q_0 q_1 q_2 q_3;
// when P leaves [2^-1000, 2^1000] (some d outside ~[1e-75, 1e75]) the lane takes four rcp_sweep
// instead and the function returns false (the caller then also keeps its running product of the q_i
// in range one factor at a time).
__device__ inline bool batch_rcp4_guarded(const double (&q)[4], double (&iq)[4], double& P) {
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  P = q01 * q23;
  if (__builtin_expect(!(P > 0x1p-1000 && P < 0x1p1000), 0)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) iq[i] = rcp_sweep(q[i]);
    return false;
  }
  double R = __builtin_amdgcn_rcp(P);
  R = fma(R, fma(-P, R, 1.0), R);
  const double R23 = R * q23, R01 = R * q01;
  iq[0] = R23 * q[1];
  iq[1] = R23 * q[0];
  iq[2] = R01 * q[3];
  iq[3] = R01 * q[2];
  return true;
}

// global -> LDS DMA of one 1 KiB piece (64 lanes x 16 B, per-lane global byte offsets from a
// wave-uniform base), issued from inline asm so the compiler's waitcnt pass does not drain it before
// unrelated LDS reads; the consumer waits with an explicit s_waitcnt vmcnt + barrier.  s_nop 4: a
// fresh SGPR base read by a global_* op; s_nop 0: between the M0 write and the LDS-DMA reading it.
__device__ inline void dma_piece(const void* sbase, uint32_t voffset, uint32_t lds_dst) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(lds_dst), "v"(voffset), "s"(sbase) : "memory", "m0");
#pragma clang diagnostic pop
}

// ---- int8 Ozaki contraction helpers (kernels_i8.hip, gemm_i8.hip)
typedef int v4i __attribute__((ext_vector_type(4)));

// weight quantisation: Gram X_A = rint(w~ kI8ScaleG) in [0, 2^32) read directly as 4 offset bytes;
// u X_A = rint(u~ kI8ScaleU) stored as X_A + 2^31.  256 below the power of two keeps rint inside
// the range when w~ rounds a hair above 1.
constexpr double kI8ScaleG = 4294967040.0;  // 2^32 - 256
constexpr double kI8ScaleU = 2147483392.0;  // 2^31 - 256

// Static per-slot bound beta >= |a r / d| over a in [0, 1]: |a (y - mu a)| is a parabola in a
// (max at a = 1 or at its vertex y / (2 mu)), and d = omega^2 a^2 + sigma^2 >= sigma^2.
__device__ inline double u_bound(double y, double mu, double noise) {
  double f = fabs(y - mu);
  if (mu != 0.0) {
    const double av = y / (2 * mu);
    if (av > 0.0 && av < 1.0) f = fmax(f, fabs(y * av - mu * av * av));
  }
  const double b = 1.125 * f / noise;
  return (b > 0.0 && b < INFINITY) ? b : 1.0;
}

// digit plane i (byte 3 - i of each X) of 16 slots, packed 4 slots per dword in K order
__device__ inline v4i digit_plane(const uint32_t (&x)[16], int i) {
  const int sh = 8 * (3 - i);
  v4i r;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    r[m] = (int)(((x[4 * m] >> sh) & 0xffu) | (((x[4 * m + 1] >> sh) & 0xffu) << 8) |
                 (((x[4 * m + 2] >> sh) & 0xffu) << 16) | (((x[4 * m + 3] >> sh) & 0xffu) << 24));
  return r;
}

// exp(v) for v <= 0 (v = N * total, voigt.c:291): v = (64 m + j) ln2/64 + r, |r| <= ln2/128,
// exp(v) = 2^m * 2^(j/64) * e^r with 2^(j/64) from a 64-entry LDS table (host-rounded from long
// double) and e^r a degree-5 Taylor polynomial (truncation < 4e-17).  Underflows to +0 like exp.
__device__ inline double exp_tab64(double v, const double* __restrict__ tab) {
  constexpr double kInvL = 92.33248261689366;              // 64 / ln 2
  constexpr double kLhi = 0.010830424695086549;           // ln2/64 to 33 bits (k*kLhi exact)
  constexpr double kLlo = 1.162596423439437e-12;           // ln2/64 - kLhi
  v = fmax(v, -1100.0);                                    // keeps k in int range; exp(-1100) = 0
  // k = rint(v 64/ln2) by the 1.5 2^52 shifter: the fma rounds at the units place, the low
  // mantissa word is k as a two's-complement int (no f64 <-> int conversion instructions)
  const double kd = fma(v, kInvL, 0x1.8p52);
  const int ki = __double2loint(kd);
  const double k = kd - 0x1.8p52;
  double r = fma(-k, kLhi, v);
  r = fma(-k, kLlo, r);
  double p = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return __builtin_ldexp(p * tab[ki & 63], ki >> 6);
}

// exp_tab64 on a 128-entry table: v = (128 m + j) ln2/128 + r, |r| <= ln2/256, and e^r by a degree-4
// minimax polynomial on that interval (relative error 7.6e-17, Remez fit: tools/fit_exp_poly.py), one
// FMA fewer than exp_tab64.  No clamp of v: callers guarantee v >= -2^31 ln2/128 (k then fits an
// int; below -745 the ldexp underflows to +0 like exp).  The fused fp64 sweep clamps only its
// core-zone lanes, and every lane of a wave whose N_HI could take the wings alone past that bound.
__device__ inline double exp_tab128_nc(double v, const double* __restrict__ tab) {
  constexpr double kInvL = 184.6649652337873;              // 128 / ln 2
  constexpr double kLhi = 0x1.62e42fefp-8;                 // ln2/128 to 33 bits (k*kLhi exact)
  constexpr double kLlo = 5.812982117197185e-13;           // ln2/128 - kLhi
  const double kd = fma(v, kInvL, 0x1.8p52);
  const int ki = __double2loint(kd);
  const double k = kd - 0x1.8p52;
  double r = fma(-k, kLhi, v);
  r = fma(-k, kLlo, r);
  double p = fma(r, 0.04166665394028975, 0.16666674303258167);
  p = fma(p, r, 0.5000000000001633);
  p = fma(p, r, 0.99999999999986);
  p = fma(p, r, 1.0);
  return __builtin_ldexp(p * tab[ki & 127], ki >> 7);
}

// T_j = 1/x_j^2 of the three Lyman lines with ONE v_rcp_f64 (+ Newton step) on x0^2 x1^2 x2^2
// (< 1e26 over the spectral range) instead of three.  a_j = x_j^2 + 2^-1000 (an fma, as cheap as
// the multiply): bit-identical to x_j^2 for every x_j != 0 (|x_j| >= ~4e-12 on the path), and a lane
// exactly on a line centre (x_j = 0) still gets finite T of the other two lines instead of
// 0 * inf = NaN.  The core lanes' own T_j (huge) are discarded by the fix-up's core select.
__device__ inline void wing_T3(double x0, double x1, double x2, double& T0, double& T1, double& T2) {
  constexpr double kTiny = 0x1p-1000;
  const double a0 = fma(x0, x0, kTiny), a1 = fma(x1, x1, kTiny), a2 = fma(x2, x2, kTiny);
  const double p01 = a0 * a1;
  const double q = p01 * a2;
  double R = __builtin_amdgcn_rcp(q);
  R = fma(R, fma(-q, R, 1.0), R);
  const double r01 = R * a2;  // 1 / (a0 a1)
  T0 = a1 * r01;
  T1 = a0 * r01;
  T2 = p01 * R;
}

template <int SRC>
__device__ inline double quad_bcast_c(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_mov_dpp(lo, SRC * 0x55, 0xF, 0xF, false);
  hi = __builtin_amdgcn_mov_dpp(hi, SRC * 0x55, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// value of lane (quad_base + src) broadcast to the 4 lanes of each quad; src folds to a
// constant after unrolling
__device__ inline double quad_bcast(double v, int src) {
  switch (src & 3) {
    case 0: return quad_bcast_c<0>(v);
    case 1: return quad_bcast_c<1>(v);
    case 2: return quad_bcast_c<2>(v);
    default: return quad_bcast_c<3>(v);
  }
}

__device__ inline int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int t = __shfl_up(v, off);
    if (lane >= off) v += t;
  }
  return v;
}

// exclusive block scan over 256 threads; returns exclusive prefix, total via *total
__device__ inline int block_excl_scan(int v, int* lds4, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) lds4[wave] = inc;
  __syncthreads();
  int woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    int c = lds4[w];
    if (w < wave) woff += c;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return woff + inc - v;
}

__device__ inline double block_reduce_min(double v, double* lds4) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off));
  if (lane == 0) lds4[wave] = v;
  __syncthreads();
  double r = fmin(fmin(lds4[0], lds4[1]), fmin(lds4[2], lds4[3]));
  __syncthreads();
  return r;
}

__device__ inline double block_reduce_max(double v, double* lds4) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  if (lane == 0) lds4[wave] = v;
  __syncthreads();
  double r = fmax(fmax(lds4[0], lds4[1]), fmax(lds4[2], lds4[3]));
  __syncthreads();
  return r;
}

__device__ inline double block_reduce_sum(double v, double* lds4) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if (lane == 0) lds4[wave] = v;
  __syncthreads();
  double r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
  __syncthreads();
  return r;
}

// Gram pair e -> (r, c), row-major upper triangle (r <= c)
template <int K>
__device__ inline void gram_pair(int e, int& r, int& c) {
  int rr = 0, start = 0;
  while (rr < K - 1 && e >= start + (K - rr)) {
    start += K - rr;
    ++rr;
  }
  r = rr;
  c = rr + (e - start);
}

template <int K>
__device__ __host__ constexpr int gram_index(int r, int c) {
  return r * K - r * (r - 1) / 2 + (c - r);
}

// numpy.interp-style linear interpolation index on a strictly increasing grid
__device__ inline int interp_index(const double* xp, int G, double x) {
  int lo = 0, hi = G - 1;  // invariant xp[lo] <= x < xp[hi] (x inside the grid)
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (xp[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ inline double interp_eval(const double* xp, const double* fp, int G, int j, double x) {
  if (x >= xp[G - 1]) return fp[G - 1];
  const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
  return slope * (x - xp[j]) + fp[j];
}

// ---------------------------------------------------------------------------------------------
// Voigt raw profile at one padded wavelength: exp(N * total), total = -sum_j lc_j V_j(v_j)
// (voigt.c:282-292).  x_j = lambda * fac_j / (1+z) - c/(sigma sqrt 2) (voigt.c:278-279,287).
// ---------------------------------------------------------------------------------------------
constexpr double kC2 = kCcgs / (kSigma * 1.41421356237309504880);  // c / (sigma sqrt 2)

// generic: any number of lines, core tables in global memory
__device__ inline double raw_profile(double lam, double zfac, double N, int num_lines,
                                     const LineArgs& L) {
  double total = 0.0;
  for (int j = 0; j < num_lines; ++j) {
    const double x = fma(lam, L.buf[kLineBufFac + j] * zfac, -kC2);
    total -= line_profile_eval(L.buf + (size_t)j * kCoreTable,
                               L.buf + kLineBufWing + (size_t)j * kWingStride, x);
  }
  return exp(N * total);
}

// 3-line fast path (Lyman alpha, beta, gamma; set_parameters.m:63): the damping wing is
// evaluated branch-free for every lane with its coefficients read from LDS by broadcast
// (wing_lds), the core polynomial (LDS tables) only by the lanes with |x| < kCoreX.
// TAB = the exp table in exp_lds: 64 entries (exp_tab64) or 128 (exp_tab128_nc, clamped here).
template <int TAB = 64>
__device__ inline double raw_profile3(double lam, const double (&afac)[3], double N,
                                      const double* __restrict__ core_lds,
                                      const double* __restrict__ wing_lds,
                                      const double* __restrict__ exp_lds) {
  double total = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double x = fma(lam, afac[j], -kC2);
    const double ax = fabs(x);
    double f = wing_eval(wing_lds + j * kWingStride, x);
    if (ax < kCoreX) f = core_eval(core_lds + j * kCoreTable, ax);
    total -= f;
  }
  if constexpr (TAB == 128) return exp_tab128_nc(fmax(N * total, -1100.0), exp_lds);
  else return exp_tab64(N * total, exp_lds);
}

// The fix-up lanes of the batched sweeps (some |x_j| < kOuterX): the nearest line j, |x_j| and T_j,
// and its kWingStride block.  At most one line can be that close: the Lyman lines are >= 5% apart
// in wavelength (>= 16,000 km/s) and kOuterX is 32 Doppler units (411 km/s), so the other two
// lines' outer-wing values stand.
__device__ inline void nearest_line(double lam, const double (&afac)[3], double T0, double T1, double T2,
                                    const double* __restrict__ wing_lds, double& ax, double& T,
                                    const double*& wl, int& j) {
  const double a0 = fabs(fma(lam, afac[0], -kC2)), a1 = fabs(fma(lam, afac[1], -kC2)),
               a2 = fabs(fma(lam, afac[2], -kC2));
  const bool p1 = a1 < a0;
  ax = p1 ? a1 : a0;
  T = p1 ? T1 : T0;
  j = p1 ? 1 : 0;
  const bool p2 = a2 < ax;
  ax = p2 ? a2 : ax;
  T = p2 ? T2 : T;
  j = p2 ? 2 : j;
  wl = wing_lds + j * kWingStride;
}

// raw_profile3 with the three damping-wing T_j = 1/x_j^2 from ONE v_rcp_f64 (wing_T3) instead of
// three (+ their Newton steps) and the outer wing polynomial; lanes with |x_j| < kOuterX take the
// inner wing, lanes with |x_j| < kCoreX the core polynomial (their T_j may be inf/NaN and are
// discarded by the select)
__device__ inline double raw_profile3_t3(double lam, const double (&afac)[3], double N,
                                         const double* __restrict__ core_lds,
                                         const double* __restrict__ wing_lds,
                                         const double* __restrict__ exp_lds) {
  double x[3], T[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) x[j] = fma(lam, afac[j], -kC2);
  wing_T3(x[0], x[1], x[2], T[0], T[1], T[2]);
  double total = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ax = fabs(x[j]);
    double f = outer_poly(wing_lds + j * kWingStride, T[j]);
    if (ax < kOuterX) {
      f = wing_poly(wing_lds + j * kWingStride, T[j]);
      if (ax < kCoreX) f = core_eval(core_lds + j * kCoreTable, ax);
    }
    total -= f;
  }
  return exp_tab64(N * total, exp_lds);
}

// Raw profiles of NB pixels at once, the batched sweeps' scheme: branch-free outer damping wings for
// every lane and line (one basic block, so the NB chains interleave), ONE wave-level fix-up branch for
// lanes with some |x_j| < kOuterX (the nearest line only, nearest_line), then the NB table exps.
// Same arithmetic as the fused kernel's chunk (kernels.hip likelihood_kernel).
template <int NB>
__device__ inline void raw_profile3_batch(const double (&lam)[NB], const double (&afac)[3], double N,
                                          const double* __restrict__ core_lds,
                                          const double* __restrict__ wing_lds,
                                          const double* __restrict__ exp_lds, double (&out)[NB]) {
  double tot[NB], Tj[3][NB];
  uint32_t cm = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const double x0 = fma(lam[b], afac[0], -kC2), x1 = fma(lam[b], afac[1], -kC2), x2 = fma(lam[b], afac[2], -kC2);
    cm |= (((fabs(x0) < kOuterX) | (fabs(x1) < kOuterX) | (fabs(x2) < kOuterX)) ? 1u : 0u) << b;
    wing_T3(x0, x1, x2, Tj[0][b], Tj[1][b], Tj[2][b]);
    tot[b] = 0.0;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    int zoff;
    asm volatile("s_mov_b32 %0, 0" : "=s"(zoff));  // one line's coefficients live at a time
    const double* wl = wing_lds + zoff + j * kWingStride;
#pragma unroll
    for (int b = 0; b < NB; ++b) tot[b] -= outer_poly(wl, Tj[j][b]);
  }
  if (cm) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (cm & (1u << b)) {
        double ax, T;
        const double* wl;
        int j;
        nearest_line(lam[b], afac, Tj[0][b], Tj[1][b], Tj[2][b], wing_lds, ax, T, wl, j);
        if (ax >= kCoreX) {
          tot[b] += outer_poly(wl, T) - wing_poly(wl, T);
        } else {
          const double cf = core_eval(core_lds + j * kCoreTable, ax);
          double t = 0.0;
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) t -= jj == j ? cf : outer_poly(wing_lds + jj * kWingStride, Tj[jj][b]);
          tot[b] = t;
        }
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) out[b] = exp_tab64(N * tot[b], exp_lds);
}

// ---------------------------------------------------------------------------------------------
// Per-sample augmented LDL^T in registers, one quad of lanes per sample.
//   Lane jq of the quad owns Gram columns c = 4jj + jq (rows 0..4jj+3, A[jj][i]) and u rows
//   i = 4m + jq (U[m]); pivot rows are broadcast inside the quad with DPP.  [B u; u' q1] with
//   B = I + M'D^-1 M (log_mvnpdf_low_rank.m:22-24) is factored as L D L': log det B = sum log D_p
//   and r'K^-1 r = q1 - u'B^-1 u is the last pivot (log_mvnpdf_low_rank.m:26-32).  quad = sum r^2/d,
//   prod d = dm 2^de.
// ---------------------------------------------------------------------------------------------
template <int K>
__device__ inline double ldl_factor(double (&A)[(K + 3) / 4][4 * ((K + 3) / 4)], double (&U)[(K + 3) / 4],
                                    double quad, double dm, double de, int jq, int n, bool& bad_out) {
  constexpr int NJJ = (K + 3) / 4;
  double pb = 1.0;
  int eb = 0;
  bool bad = false;
#pragma unroll
  for (int p = 0; p < K; ++p) {
    const double Dp = quad_bcast(A[p >> 2][p], p & 3);
    bad |= !(Dp > 0.0) || !(Dp < INFINITY);
    // v_rcp_f64 + two Newton steps (within an ulp of 1/Dp) instead of the IEEE division sequence;
    // a pivot that is not positive and finite is flagged above and the result discarded
    double invD = __builtin_amdgcn_rcp(Dp);
    invD = fma(invD, fma(-Dp, invD, 1.0), invD);
    invD = fma(invD, fma(-Dp, invD, 1.0), invD);
    pb *= Dp;
    if ((p & 3) == 3) {
      int ex;
      pb = frexp(pb, &ex);
      eb += ex;
    }
    const double up = quad_bcast(U[p >> 2], p & 3);
    const double upinv = up * invD;
    double rowp[K];
#pragma unroll
    for (int i = p + 1; i < K; ++i) rowp[i] = quad_bcast(A[i >> 2][p], i & 3);
#pragma unroll
    for (int jj = p >> 2; jj < NJJ; ++jj) {
      const double sc = A[jj][p] * invD;
#pragma unroll
      for (int i = p + 1; i < 4 * jj + 4 && i < K; ++i) A[jj][i] = fma(-rowp[i], sc, A[jj][i]);
    }
#pragma unroll
    for (int mm = 0; mm < NJJ; ++mm) {
      if (4 * mm + 3 > p) {
        const bool cnd = (4 * mm + jq) > p;
        U[mm] = cnd ? fma(-A[mm][p], upinv, U[mm]) : U[mm];
      }
    }
    quad = fma(-up, upinv, quad);
  }
  const double logdet_b = log(pb) + eb * kLn2;
  const double logdet_d = log(dm) + de * kLn2;
  const double ll = -0.5 * (quad + (logdet_d + logdet_b) + n * kLog2Pi);  // log_mvnpdf_low_rank.m:30-32
  bad_out = bad || !(fabs(ll) < INFINITY);
  return bad_out ? NAN : ll;
}

// The quad's matrix from a sample row in memory (Layout<K>::kES doubles): Gram entries (r, c),
// r <= c, at gram_index(r, c); u_i at 4 kGT + i; sum r^2/d, prod-d mantissa and exponent at
// 4 kTiles + {0,1,2}.
template <int K>
__device__ inline double ldl_log_likelihood(const double* srow, int jq, int n, bool& bad_out) {
  using Lay = Layout<K>;
  constexpr int kTiles = Lay::kTiles;
  constexpr int kGT = Lay::kGT;
  constexpr int NJJ = (K + 3) / 4;
  double A[NJJ][4 * NJJ];
  double U[NJJ];
#pragma unroll
  for (int jj = 0; jj < NJJ; ++jj) {
    const int c = 4 * jj + jq;
#pragma unroll
    for (int i = 0; i < 4 * jj + 4; ++i) {
      double v = 0.0;
      if (i <= c && c < K) {
        v = srow[gram_index<K>(i, c)];
        if (i == c) v += 1.0;  // B = I + M' D^-1 M (log_mvnpdf_low_rank.m:23)
      }
      A[jj][i] = v;
    }
    U[jj] = (c < K) ? srow[4 * kGT + c] : 0.0;
  }
  return ldl_factor<K>(A, U, srow[4 * kTiles], srow[4 * kTiles + 1], srow[4 * kTiles + 2], jq, n, bad_out);
}

// lane jq of each quad gets x from lane (jq + ROT) & 3 of its quad (DPP quad_perm)
template <int ROT>
__device__ inline double quad_rot(double v) {
  if constexpr ((ROT & 3) == 0) {
    return v;
  } else {
    constexpr int sel = ((0 + ROT) & 3) | (((1 + ROT) & 3) << 2) | (((2 + ROT) & 3) << 4) | (((3 + ROT) & 3) << 6);
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), sel, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), sel, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
  }
}

// The quad's matrix straight from the v_mfma_f64_4x4x4_4b accumulators (no memory): lane jq of a
// quad holds entry 4t + jq of its sample in acc[t], so entry (i, c = 4jj + jq) = e = b + jq with
// b = gram_index(i, 4jj) sits in lane (jq + b) & 3 of register (b >> 2) + ((jq + (b & 3)) >> 2):
// a quad rotation by b & 3 of registers b >> 2 and b >> 2 + 1, then a select.  All indices are
// compile-time; u_c = entry 4 kGT + c is already in lane jq.
template <int K, int I, int JJ>
__device__ inline double gram_entry_from_acc(const double (&acc)[Layout<K>::kTiles], int jq) {
  constexpr int kTiles = Layout<K>::kTiles;
  constexpr int b = I * K - I * (I - 1) / 2 - I + 4 * JJ;  // gram_index(I, 4 JJ), extended linearly
  constexpr int G = b >> 2, gam = b & 3;
  const double v0 = quad_rot<gam>(acc[G < kTiles ? G : kTiles - 1]);
  if constexpr (gam == 0) {
    return v0;
  } else {
    const double v1 = quad_rot<gam>(acc[G + 1 < kTiles ? G + 1 : kTiles - 1]);
    return (jq + gam >= 4) ? v1 : v0;
  }
}

template <int K, int JJ, int I>
__device__ inline void fill_column_block(double (&A)[(K + 3) / 4][4 * ((K + 3) / 4)],
                                         const double (&acc)[Layout<K>::kTiles], int jq) {
  if constexpr (I < 4 * JJ + 4) {
    const int c = 4 * JJ + jq;
    const double v = gram_entry_from_acc<K, I, JJ>(acc, jq);
    A[JJ][I] = (I <= c && c < K) ? v + (I == c ? 1.0 : 0.0) : 0.0;  // B = I + M' D^-1 M (.m:23)
    fill_column_block<K, JJ, I + 1>(A, acc, jq);
  }
}

template <int K, int JJ>
__device__ inline void fill_from_acc(double (&A)[(K + 3) / 4][4 * ((K + 3) / 4)], double (&U)[(K + 3) / 4],
                                     const double (&acc)[Layout<K>::kTiles], int jq) {
  if constexpr (JJ < (K + 3) / 4) {
    fill_column_block<K, JJ, 0>(A, acc, jq);
    U[JJ] = (4 * JJ + jq < K) ? acc[Layout<K>::kGT + JJ] : 0.0;
    fill_from_acc<K, JJ + 1>(A, U, acc, jq);
  }
}

}  // namespace

}  // namespace gpdla
