// Panel-GEMM path with the Gram/u contraction on the int8 matrix cores (path panel_gemm_i8, any
// rank 1..kGemmMaxK; BASELINE configs[4]: k = 50, 10^5 samples, quoted in fp32).  Same numerics as
// the fused int8 kernel (kernels_i8.hip), as a GEMM:
//   convert_gemm_i8_kernel  panel entries P~ (Khatri-Rao / (omega^2 + sigma^2), M beta) -> 4
//                           balanced base-256 digit planes per entry, K-contiguous, + scales
//   weights_i8_kernel       Voigt x pixel terms (process_qsos.m:186-197) -> the quantised weights
//                           w~, u~ as 4 offset-byte digit planes per sample, K-contiguous, and the
//                           sum r^2/d, sum log d partials of the fp64 weights kernel
//   gemm_i8_kernel          C[s][e] = sum_slot X_A X_B exactly (10 digit pairs of level <= 3 on
//                           v_mfma_i32_16x16x64_i8, int32 per level), fp64 epilogue -> Gram / u
// followed by the fp64 augmented LDL^T of gemm_path.hip (log_mvnpdf_low_rank.m:22-32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "internal.h"

#include <utility>

namespace {
// f(std::integral_constant<int, i>{}) for i = 0 .. N - 1, each i a compile-time constant (inline-asm
// immediates and register-set indices need that; #pragma unroll only folds them after the fact)
template <int N, typename F, int... I>
__device__ inline void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ inline void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}
}  // namespace

namespace gpdla {

namespace {

#define MFMA_I8(A, B, C) __builtin_amdgcn_mfma_i32_16x16x64_i8((A), (B), (C), 0, 0, 0)

// Epilogue of the exact int8 contraction: the ND level sums C_l (digit pairs of level l, weight
// 2^(48 - 8 l)) are folded as t = sum_l 256^(ND - 1 - l) C_l in fp64 (integer-valued, exact while it
// stays below 2^53, which covers every configs[4]-sized K), then value = (2^(48 - 8 (ND - 1)) t + off0)
// sc as ONE fma with the column's constants scl = 2^(48 - 8 (ND - 1)) sc and offl = off0 sc: 7 VALU
// per output instead of 9 (round 5: the epilogue was 16% of the Gram launch, profiles/round5/r10o)
template <int ND>
__device__ inline double i8_level_value(const v4i (&lv)[ND], int r, double scl, double offl) {
  double t = (double)lv[0][r];
#pragma unroll
  for (int l = 1; l < ND; ++l) t = fma(t, 256.0, (double)lv[l][r]);
  return fma(t, scl, offl);
}
template <int ND>
__host__ __device__ constexpr double i8_level_scale() { return (double)(1ull << (48 - 8 * (ND - 1))); }

// --------------------------------------------------------------------------------------------
// convert: grid (entries / 64, spectra), 256 threads = 64 entries x 4 segments
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void convert_gemm_i8_kernel(ConvertGemmI8Args a) {
  __shared__ double s_mx[4][64];
  __shared__ long long s_cs[4][64];
  __shared__ uint16_t s_rc[64];                  // Gram entry -> (r, c) of this block's 64 entries
  const int q = blockIdx.y;
  const SpecInfo inf = a.info[q];
  if (inf.J == 0) return;
  const int K = a.k;
  const int E = K * (K + 1) / 2;
  const int Ep = 64 * ((E + 63) / 64);
  const int NE = i8_gemm_entries(K);
  const int le = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + le;
  const bool is_u = e >= Ep;
  const int col = is_u ? e - Ep : e;
  const bool valid = is_u ? col < K : col < E;
  const int L = inf.L;
  const int Ls = ((L + kChunkSteps - 1) / kChunkSteps) * kChunkSteps;
  const int Ls16 = 16 * ((L + 15) / 16);
  const int64_t sb = a.slot_base[q];
  const int64_t kstride = i8_gemm_kstride(a.slot_cap[q]);
  const int nd = i8_spectrum_nd(a.nd, a.slot_cap[q]);  // short spectra: 4 planes on the 24-bit path too
  // the Gram entry col is the Khatri-Rao product M_r M_c of its (r, c) (gram_tile_index order, as
  // prep_kernel<0> would store it; formed here from the M rows instead of read as 8 B per entry and
  // slot: bit for bit the same products)
  if (threadIdx.x < 64) s_rc[threadIdx.x] = 0;
  __syncthreads();
  if (blockIdx.x * 64 < Ep)                      // a Gram entry tile: every (r, c) of it, 256 at a time
    for (int pr = threadIdx.x; pr < K * K; pr += 256) {
      const int r = pr / K, c = pr - r * K;
      const int ee = c >= r ? gram_tile_index(r, c, K) - blockIdx.x * 64 : -1;
      if (ee >= 0 && ee < 64) s_rc[ee] = (uint16_t)(r | (c << 8));
    }
  __syncthreads();
  const int rc = is_u ? 0 : s_rc[le];
  const int mr = is_u ? col : (rc & 255), mc = rc >> 8;
  auto value = [&](int t) -> double {
    if (!valid || t >= L) return 0.0;
    const int64_t row = sb + (int64_t)g * Ls + t;
    const double* sr = a.srow + row * 8;
    const double y = sr[1], noise = sr[2], mu = sr[3], om2 = sr[4];
    const double* m = a.panel_m + row * gemm_ldm(K);
    return is_u ? m[mr] * u_bound(y, mu, noise) : (m[mr] * m[mc]) / (om2 + noise);
  };
  double mx = 0.0;
  for (int t = 0; t < L; ++t) mx = fmax(mx, fabs(value(t)));
  s_mx[g][le] = mx;
  __syncthreads();
  mx = fmax(fmax(s_mx[0][le], s_mx[1][le]), fmax(s_mx[2][le], s_mx[3][le]));
  const double s_e = mx > 0.0 ? mx * (1.0 / (127.0 * 0x1p24)) : 1.0;  // |X_B| <= 127 2^24
  long long colsum = 0;
  // B layout (the GEMM's LDS image, pre-swizzled): [entry tile 64][K step][plane 4][row 64][64 B], K
  // granule gr of row r at 16-B slot (gr + 2 ((r >> 2) & 3)) & 3 -- one K step of an entry tile is a
  // contiguous 4 KiB per plane, so each 1-KiB DMA piece reads 8 whole cache lines
  const int64_t nksmax = kstride / 64;
  const int r = e & 63;
  uint8_t* tbase = a.bdig + a.bbase[q] + (int64_t)(e >> 6) * nksmax * 4 * 4096 + (int64_t)r * 64;
  const int rsw = 2 * ((r >> 2) & 3);
  for (int t0 = 0; t0 < Ls16; t0 += 16) {
    uint32_t pl[4][4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll
      for (int j = 0; j < 4; ++j) pl[j][w] = 0u;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        int X = (int)rint(value(t0 + 4 * w + b) / s_e);
        colsum += X;
        const int d3 = ((X + 128) & 255) - 128; X = (X - d3) >> 8;
        const int d2 = ((X + 128) & 255) - 128; X = (X - d2) >> 8;
        const int d1 = ((X + 128) & 255) - 128; X = (X - d1) >> 8;
        pl[0][w] |= (uint32_t)(X & 255) << (8 * b);
        pl[1][w] |= (uint32_t)(d1 & 255) << (8 * b);
        pl[2][w] |= (uint32_t)(d2 & 255) << (8 * b);
        pl[3][w] |= (uint32_t)(d3 & 255) << (8 * b);
      }
    }
    const int kk = g * Ls16 + t0, ks = kk >> 6, gr = (kk >> 4) & 3;
    uint8_t* dst = tbase + (int64_t)ks * 4 * 4096 + 16 * ((gr + rsw) & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < (is_u ? 4 : nd))  // u entries keep 4 digits (launch_gemm_i8)
        *reinterpret_cast<uint4*>(dst + j * 4096) = make_uint4(pl[j][0], pl[j][1], pl[j][2], pl[j][3]);
  }
  s_cs[g][le] = colsum;
  __syncthreads();
  if (g == 0) {
    const long long cs = s_cs[0][le] + s_cs[1][le] + s_cs[2][le] + s_cs[3][le];
    a.ent[(int64_t)q * 2 * NE + e] = s_e / (is_u ? kI8ScaleU : kI8ScaleG);
    a.ent[(int64_t)q * 2 * NE + NE + e] = (is_u ? 8421504.0 : 2155905152.0) * (double)cs;
  }
}

// --------------------------------------------------------------------------------------------
// Raw profiles of two padded positions in packed fp32 (the 24-bit path's weights, kF32 below).  x_j
// stays fp64 (lambda fac_j / (1 + z) - c / (sigma sqrt 2) cancels from ~2.3e4 to the few Doppler
// units that matter), then the three lines' damping wings (T_j = 1/x_j^2 from one reciprocal, the
// outer polynomial) and the exp run as v_pk_* fp32 on the pair.  Lanes with some |x_j| < kOuterX
// (core or inner wing; one wave-level branch per pair) recompute their total in fp64 as
// raw_profile3 does.  Emulated on configs[4] spectra: the log-likelihood error of the 24-bit path
// moves from 9.25e-8 to 9.9e-8 against fp64 (fp32 profile, instrument broadening and exp; DESIGN.md
// section 4.2); its Gram is quantised to 24 bits anyway.
// --------------------------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ inline double total3_f64(double x0, double x1, double x2, const double* __restrict__ core,
                                    const double* __restrict__ wing_lds) {
  const double xs[3] = {x0, x1, x2};
  double t = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ax = fabs(xs[j]);
    const double T = rcp_nr(fma(xs[j], xs[j], 0x1p-1000));
    double f = outer_poly(wing_lds + j * kWingStride, T);
    if (ax < kOuterX) f = wing_poly(wing_lds + j * kWingStride, T);
    if (ax < kCoreX) f = core_eval(core + j * kCoreTable, ax);
    t -= f;
  }
  return t;
}

__device__ inline f2v raw_profile3_pair_f32(double lam0, double lam1, const double (&afac)[3], float nl2e,
                                            const float (&oc)[3][kOuterDeg + 1],
                                            const double* __restrict__ core,
                                            const double* __restrict__ wing_lds) {
  double xd0[3], xd1[3];
  f2v x[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    xd0[j] = fma(lam0, afac[j], -kC2);
    xd1[j] = fma(lam1, afac[j], -kC2);
    x[j] = (f2v){(float)xd0[j], (float)xd1[j]};
  }
  const f2v tiny = (f2v){0x1p-60f, 0x1p-60f};
  const f2v a0 = x[0] * x[0] + tiny, a1 = x[1] * x[1] + tiny, a2 = x[2] * x[2] + tiny;
  const f2v p01 = a0 * a1, q = p01 * a2;
  const f2v R = (f2v){__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  const f2v r01 = R * a2;
  const f2v T[3] = {a1 * r01, a0 * r01, p01 * R};
  f2v tot = (f2v){0.0f, 0.0f};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    f2v f = (f2v){oc[j][kOuterDeg], oc[j][kOuterDeg]};
#pragma unroll
    for (int n = kOuterDeg - 1; n >= 0; --n) f = f * T[j] + (f2v){oc[j][n], oc[j][n]};
    tot = tot - T[j] * f;
  }
  const float m0 = fminf(fabsf(x[0].x), fminf(fabsf(x[1].x), fabsf(x[2].x)));
  const float m1 = fminf(fabsf(x[0].y), fminf(fabsf(x[1].y), fabsf(x[2].y)));
  const bool n0 = m0 < (float)kOuterX, n1 = m1 < (float)kOuterX;
  if (n0 || n1) {  // rare: a line's core or inner wing -- the whole total in fp64
    if (n0) tot.x = (float)total3_f64(xd0[0], xd0[1], xd0[2], core, wing_lds);
    if (n1) tot.y = (float)total3_f64(xd1[0], xd1[1], xd1[2], core, wing_lds);
  }
  const f2v v = tot * (f2v){nl2e, nl2e};  // N tot log2(e) <= 0
  return (f2v){__builtin_amdgcn_exp2f(v.x), __builtin_amdgcn_exp2f(v.y)};
}

// --------------------------------------------------------------------------------------------
// weights: one task = 64 consecutive samples (lane = sample) x one segment g x one quarter h of the
// segment's slots.  The wave walks its quarter (whole 16-slot groups) with the register sliding
// window, and stores each 16-slot group as 16 bytes per digit plane (K-contiguous rows: the GEMM's
// A operand).  core / wing_lds / exp_lds: the line cores, wing polynomials and 2^(j/64) table in LDS.
// kF32 (the 24-bit path, nd = 3): raw profiles and the 7-tap broadening in fp32 (pairs of positions
// in packed fp32, raw_profile3_pair_f32); everything from the broadened absorption on in fp64.
// --------------------------------------------------------------------------------------------
template <bool kF32>
__device__ inline void weights_i8_task(const WeightsI8Args& a, const double* __restrict__ srow, const SpecInfo& inf,
                                       int blk, int g, int h, int lane, const double* __restrict__ core,
                                       const double* __restrict__ wing_lds, const double* __restrict__ exp_lds) {
  using W = typename std::conditional<kF32, float, double>::type;
  constexpr int kB = kF32 ? 2 : kWB;              // raw profiles per batch
  const int sl = blk * 64 + lane;
  const bool active = sl < a.sc;
  const int64_t s = a.s0 + sl;
  const int L = inf.L;
  const int Ls = ((L + kChunkSteps - 1) / kChunkSteps) * kChunkSteps;
  const int Ls16 = 16 * ((L + 15) / 16);
  // quarter h: 16-slot groups h G16 / 4 .. (h + 1) G16 / 4 - 1 (balanced: 13 groups go 3, 3, 3, 4)
  const int G16 = Ls16 / 16;
  const int t0 = 16 * (h * G16 / kWeightQuarters), t1 = 16 * ((h + 1) * G16 / kWeightQuarters);
  const double off = (s < a.S) ? a.offsets[s] : 0.5;
  const double N = (s < a.S) ? a.nhi[s] : 0.0;  // null model / idle lanes: absorption exactly 1
  const double zdla = inf.zmin + (inf.zmax - inf.zmin) * off;  // process_qsos.m:163-165
  const double zfac = 1.0 / (1 + zdla);
  double afac[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) afac[j] = a.lines.buf[kLineBufFac + j] * zfac;
  float oc[3][kOuterDeg + 1];
  const float nl2e = (float)(N * 1.4426950408889634);
  if constexpr (kF32) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int n = 0; n <= kOuterDeg; ++n)  // wave-uniform: kept in SGPRs
        oc[j][n] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                       __builtin_bit_cast(int, (float)wing_lds[j * kWingStride + kOuterOff + n])));
  }
  const double* lamp = a.lam_pad + (int64_t)g * L + t0;  // padded positions g L + t0 + 0..5
  W w0, w1, w2, w3, w4, w5;
  if constexpr (kF32) {
    f2v p = raw_profile3_pair_f32(lamp[0], lamp[1], afac, nl2e, oc, core, wing_lds);
    w0 = p.x; w1 = p.y;
    p = raw_profile3_pair_f32(lamp[2], lamp[3], afac, nl2e, oc, core, wing_lds);
    w2 = p.x; w3 = p.y;
    p = raw_profile3_pair_f32(lamp[4], lamp[5], afac, nl2e, oc, core, wing_lds);
    w4 = p.x; w5 = p.y;
  } else {
    auto raw = [&](double lam) { return raw_profile3_t3(lam, afac, N, core, wing_lds, exp_lds); };
    w0 = raw(lamp[0]); w1 = raw(lamp[1]); w2 = raw(lamp[2]);
    w3 = raw(lamp[3]); w4 = raw(lamp[4]); w5 = raw(lamp[5]);
  }
  double q1 = 0.0, pm = 1.0;
  int pe = 0;
  // A layout (tile-major, like B): [type 2][sample tile 128][K step][plane 4][group 4][sample 128][16 B];
  // one K step of a sample tile is a contiguous 32 KiB (a lane's 16-byte store per group sits next to
  // its neighbours': coalesced runs of 1 KiB per wave)
  const int64_t nksmax = a.kstride / 64;
  const int64_t type_bytes = a.rows * a.kstride * 4;
  uint8_t* ag = a.adig + (((int64_t)(sl >> 7) * nksmax * 16) * 128 + (sl & 127)) * 16;
  uint8_t* au = ag + type_bytes;
  // byte offset of 16-slot group G (= K index / 16), plane i
  auto goff = [&](int G, int i) { return ((int64_t)((G >> 2) * 4 + i) * 4 + (G & 3)) * 2048; };
  for (int tg = t0; tg < t1; tg += 16) {
    // 16 slots' quantised weights collected for the digit planes, the raw profiles kB slots at a time
    // (one fix-up branch per batch; a task's 64 samples are consecutive in z)
    uint32_t xg[16], xu[16];
#pragma unroll
    for (int qb = 0; qb < 16 / kB; ++qb) {
      // neutral past the segment (quantisation scales as prep_kernel computes them for y = mu = om2 = 0,
      // noise = 1: u_bound = 1)
      double lam[kB];
      W w6v[kB];
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const int t = tg + kB * qb + b;
        lam[b] = t < L ? srow[((int64_t)g * Ls + t) * 8] : a.lam_pad[(int64_t)g * L + t + 2 * kWidth];
      }
      if constexpr (kF32) {
        const f2v p = raw_profile3_pair_f32(lam[0], lam[1], afac, nl2e, oc, core, wing_lds);
        w6v[0] = p.x;
        w6v[1] = p.y;
      } else {
        raw_profile3_batch<kB>(lam, afac, N, core, wing_lds, exp_lds, w6v);
      }
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const int e = kB * qb + b;
        const int t = tg + e;
        double y = 0.0, noise = 1.0, mu = 0.0, om2 = 0.0, su = kI8ScaleU, sg = kI8ScaleG;
        if (t < L) {
          const double* sr = srow + ((int64_t)g * Ls + t) * 8;
          y = sr[1]; noise = sr[2]; mu = sr[3]; om2 = sr[4]; su = sr[6]; sg = sr[7];
        }
        const W w6 = w6v[b];
        W abw = w0 * (W)kInstrumentProfile[0];  // voigt.c:297-299
        abw = fma(w1, (W)kInstrumentProfile[1], abw);
        abw = fma(w2, (W)kInstrumentProfile[2], abw);
        abw = fma(w3, (W)kInstrumentProfile[3], abw);
        abw = fma(w4, (W)kInstrumentProfile[4], abw);
        abw = fma(w5, (W)kInstrumentProfile[5], abw);
        abw = fma(w6, (W)kInstrumentProfile[6], abw);
        w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6;
        const double ab = (double)abw;
        const double r = fma(-mu, ab, y);  // process_qsos.m:191-197, log_mvnpdf_low_rank.m:11-15
        const double a2 = ab * ab;
        const double d = fma(om2, a2, noise);
        const double dinv = rcp_sweep(d);
        const double rd = r * dinv;
        q1 = fma(r, rd, q1);
        pm *= d;
        // rint to an integer in [0, 2^32) by the 1.5 2^52 shifter: one fma rounds at the units place
        // and the low mantissa word is the integer (v_rndne + v_cvt_u32 saved, twice per slot)
        xg[e] = (uint32_t)__double2loint(fma(a2 * dinv, sg, 0x1.8p52)) ^ 0x80808080u;
        xu[e] = (uint32_t)__double2loint(fma(ab * rd, su, 0x1.8p52 + 0x1p31)) ^ 0x80808080u;
        asm volatile("" : "+v"(xg[e]), "+v"(xu[e]), "+v"(q1), "+v"(pm));  // no sinking across slots
      }
    }
    {
      int ex;
      pm = frexp(pm, &ex);
      pe += ex;
    }
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int G = (g * Ls16 + tg) >> 4;
        if (i < a.nd) *reinterpret_cast<v4i*>(ag + goff(G, i)) = digit_plane(xg, i);
        *reinterpret_cast<v4i*>(au + goff(G, i)) = digit_plane(xu, i);  // 4 u digits
      }
    }
  }
  if (active) {
    a.q1p[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = q1;
    a.ldp[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = log(pm) + pe * kLn2;
  }
}

constexpr int kWingLds = 4 * ((3 * kWingStride + 3) / 4);

// grid (ceil(sc / 64), 4 quarters), 4 waves = the 4 segments of one task column
// srow separately and __restrict__: the kernel never writes the slot scalars, so their wave-uniform
// loads can be scalar (s_load into SGPRs) instead of 64-lane vector loads into VGPRs
template <bool kF32>
__global__ __launch_bounds__(256) void weights_i8_kernel(WeightsI8Args a, const double* __restrict__ srow) {
  __shared__ __attribute__((aligned(16))) double tables[3 * kCoreTable + kWingLds + 64];
  const SpecInfo inf = a.info[a.q];
  if (inf.J == 0) return;  // the LDL kernel writes NaN
  double* core_lds = tables;
  double* wing_lds = tables + 3 * kCoreTable;
  double* exp_lds = wing_lds + kWingLds;
  for (int i = threadIdx.x; i < 3 * kCoreTable; i += 256) core_lds[i] = a.lines.buf[i];
  if (threadIdx.x < 64) exp_lds[threadIdx.x] = a.lines.buf[kLineBufExp2 + threadIdx.x];
  if (threadIdx.x < 3 * kWingStride) wing_lds[threadIdx.x] = a.lines.buf[kLineBufWing + threadIdx.x];
  __syncthreads();
  weights_i8_task<kF32>(a, srow, inf, blockIdx.x, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), blockIdx.y,
                        threadIdx.x & 63, core_lds, wing_lds, exp_lds);
}

// --------------------------------------------------------------------------------------------
// Diagnostic (gpdla_diag_raw_profile3): the weights kernels' raw 3-line profiles exp(-N sum_j
// lc_j V_j) at given wavelengths, through the SAME device functions and LDS tables as
// weights_i8_kernel -- the packed-fp32 pair path of the 24-bit panel path (f32 = 1) or the fp64
// raw_profile3_t3 of the 32-bit one (f32 = 0).  Test infrastructure for the fp32 profile's error
// against the fp64 one (tests/test_gpu_i8.py); one thread per pair of wavelengths.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void diag_raw_profile_kernel(const double* __restrict__ lam, int64_t n, double z,
                                                               double N, int32_t f32, LineArgs lines,
                                                               double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double tables[3 * kCoreTable + kWingLds + 64];
  double* core_lds = tables;
  double* wing_lds = tables + 3 * kCoreTable;
  double* exp_lds = wing_lds + kWingLds;
  for (int i = threadIdx.x; i < 3 * kCoreTable; i += 256) core_lds[i] = lines.buf[i];
  if (threadIdx.x < 64) exp_lds[threadIdx.x] = lines.buf[kLineBufExp2 + threadIdx.x];
  if (threadIdx.x < 3 * kWingStride) wing_lds[threadIdx.x] = lines.buf[kLineBufWing + threadIdx.x];
  __syncthreads();
  const int64_t i0 = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (i0 >= n) return;
  const int64_t i1 = i0 + 1 < n ? i0 + 1 : i0;
  const double zfac = 1.0 / (1 + z);
  double afac[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) afac[j] = lines.buf[kLineBufFac + j] * zfac;
  double v0, v1;
  if (f32) {
    float oc[3][kOuterDeg + 1];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int m = 0; m <= kOuterDeg; ++m) oc[j][m] = (float)wing_lds[j * kWingStride + kOuterOff + m];
    const f2v p = raw_profile3_pair_f32(lam[i0], lam[i1], afac, (float)(N * 1.4426950408889634), oc, core_lds,
                                        wing_lds);
    v0 = p.x;
    v1 = p.y;
  } else {
    v0 = raw_profile3_t3(lam[i0], afac, N, core_lds, wing_lds, exp_lds);
    v1 = raw_profile3_t3(lam[i1], afac, N, core_lds, wing_lds, exp_lds);
  }
  out[i0] = v0;
  if (i0 + 1 < n) out[i0 + 1] = v1;
}

constexpr int kGTileS = 128, kGTileE = 64;

// --------------------------------------------------------------------------------------------
// GEMM: 128-sample x 64-entry tiles, 4 waves per block; wave w owns samples 32 w .. 32 w + 31 of the
// tile (2 row tiles) x all 64 entries (4 column tiles of v_mfma_i32_16x16x64_i8, the ND (ND + 1) / 2
// digit pairs of level <= ND - 1, int32 per level: 10 pairs for ND = 4, 6 for ND = 3).  The weight
// digits (A) go global -> VGPRs in the MFMA operand layout (each wave owns its 32 samples, so A has no
// reuse across the block's waves and LDS would only add traffic), prefetched one K step ahead; only
// the panel digits (B, shared by the 4 waves) are staged, by LDS-DMA into a double-buffered tile.
// Per K step a wave reads 4 ND B-operand granules from LDS for 8 ND (ND + 1) / 2 MFMAs (staging both
// operands through LDS cost 50% more LDS traffic per MFMA plus the A writes, which kept the matrix
// cores waiting on LDS bandwidth).
//
// Persistent blocks: a block walks its tiles as ONE stream of K steps, so the next tile's first step
// is prefetched behind the current tile's last MFMAs and epilogue stores (measured equal to one block
// per tile: the kernel is bound by L2 -> CU traffic -- a loads-only variant ran 0.77 ms of its 0.80,
// an MFMA-only one 0.51; profiles/r2/c5_ab).  Tile order is
// XCD-contiguous and entry-tile-fastest: the dispatcher deals linear block b to XCD b % 8, XCD x owns
// a contiguous run of (sample tile, entry tile) pairs, and its blocks advance through the run side by
// side -- a sample tile's A digits are read into that XCD's L2 once and reused by its entry tiles.
// --------------------------------------------------------------------------------------------
template <int ND>
// 3 blocks per CU for ND = 3 (168 VGPRs; +5% over 2), 2 for ND = 4 (222 VGPRs)
__global__ __launch_bounds__(256, ND == 3 ? 3 : 2) void gemm_i8_kernel(GemmI8Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t Bs[2][ND * kGTileE * 64];
  const SpecInfo inf = a.info[a.q];
  if (inf.J == 0) return;
  const int K = a.k;
  const int E = K * (K + 1) / 2;
  const int Ep = 64 * ((E + 63) / 64);
  const int NE = i8_gemm_entries(K);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  // this block's tiles.  The 8 XCDs form an SX x EX grid over (sample tiles, entry tiles): XCD x owns
  // sample-tile range x / EX and entry-tile range x % EX; its per blocks take local tiles j, j + per,
  // ... in entry-fastest order.  EX = 2 keeps an XCD's B digits (half the entries) closer to resident
  // in its L2 beside the A digits of the sample tiles in flight (-3% GEMM time against EX = 1, which
  // re-reads all of B per sample tile; EX = 4 -2%)
  const int ny = a.ny, nst = (a.sc + kGTileS - 1) / kGTileS;
  const int EX = ny >= 2 ? 2 : 1, SX = 8 / EX;  // (the u launch has one entry tile)
  const int per = gridDim.x / 8;  // blocks per XCD (1-D grid, a multiple of 8)
  const int x = blockIdx.x % 8;
  const int ex = x % EX, sx = x / EX;
  const int e0 = ny * ex / EX, e1 = ny * (ex + 1) / EX;       // entry tiles of this XCD
  const int s0 = nst * sx / SX, s1 = nst * (sx + 1) / SX;     // sample tiles of this XCD
  const int nye = e1 - e0;
  const int nloc = (s1 - s0) * nye;
  const int j0 = blockIdx.x / 8;
  if (j0 >= nloc) return;
  const int ntile = (nloc - j0 + per - 1) / per;
  const int nks = (16 * ((inf.L + 15) / 16)) / 16;  // 64-slot K steps: 4 Ls16 / 64
  const int nsteps = ntile * nks;
  const int64_t nksmax = a.kstride / 64, type_bytes = a.rows * a.kstride * 4;
  const int g = lane >> 4;
  // A: lane (row lane & 15, 16-slot group g of the K step) in the tile-major layout of
  // weights_i8_kernel: [type][sample tile][K step][plane 4][group 4][sample 128][16 B]
  const int64_t a_lane = ((int64_t)g * 128 + 32 * wave_s + (lane & 15)) * 16;
  const uint32_t bs_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&Bs[0][0];
  // B pieces (16 entry rows x 64 B per 1 KiB piece, 4 per plane; ND pieces per wave per K step) are
  // contiguous 1 KiB runs of the pre-swizzled global image (convert_gemm_i8_kernel): K granule g of
  // row `row` sits in 16-B slot (g + 2 ((row >> 2) & 3)) & 3 of its 64 B.  ds_read_b128 serves a wave
  // in the 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32); with row = lane & 15 and
  // g = lane >> 4 every group then hits 16 distinct 16-B slots of the 256-B bank row (the XOR form
  // g ^ ((row >> 2) & 3) paired lanes 0-3 with 20-23: 2-way conflicts)
  uint32_t boff[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) boff[i] = (uint32_t)((wave_s * ND + i) * 1024 + lane * 16);  // plane p at p 4 KiB
  auto tile_s = [&](int i) { return (s0 + (j0 + i * per) / nye) * kGTileS; };
  auto tile_e = [&](int i) { return (a.e_tile0 + e0 + (j0 + i * per) % nye) * kGTileE; };
  // global K step gs = tile i, step ks: B DMA into buffer buf and A loads into registers r
  auto prefetch = [&](int gs, v4i (&r)[2][ND], int buf) {
    const int i = gs / nks, ks = gs - i * nks;
    const int e_tile = tile_e(i);
    const uint8_t* B0 = a.bdig + ((int64_t)(e_tile >> 6) * nksmax + ks) * 4 * 4096;
#pragma unroll
    for (int pi = 0; pi < ND; ++pi)
      dma_piece(B0, boff[pi], bs_base + (uint32_t)(buf * (ND * kGTileE * 64) + (wave_s * ND + pi) * 1024));
    const uint8_t* A0 = a.adig + (e_tile >= Ep ? type_bytes : 0) +
                        ((int64_t)(tile_s(i) >> 7) * nksmax + ks) * 16 * 2048 + a_lane;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int p = 0; p < ND; ++p) r[rt][p] = *reinterpret_cast<const v4i*>(A0 + p * 8192 + rt * 256);
    __builtin_amdgcn_sched_barrier(0);  // the prefetch goes out before the step's MFMAs
  };
  v4i acc[ND][2][4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int l = 0; l < ND; ++l)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[l][rt][ct] = (v4i){0, 0, 0, 0};
  };
  // one K step's MFMAs on A registers Ar and LDS buffer buf
  auto compute = [&](const v4i (&Ar)[2][ND], int buf) {
    const uint8_t* Bc = Bs[buf];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int row = 16 * ct + (lane & 15);
      v4i Bd[ND];
#pragma unroll
      for (int p = 0; p < ND; ++p)
        Bd[p] = *reinterpret_cast<const v4i*>(Bc + p * (kGTileE * 64) + row * 64 + 16 * ((g + 2 * ((row >> 2) & 3)) & 3));
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        // level l = i + j: A digit i (most significant first) x B digit j
#pragma unroll
        for (int l = 0; l < ND; ++l)
#pragma unroll
          for (int i = 0; i <= l; ++i) acc[l][rt][ct] = MFMA_I8(Ar[rt][i], Bd[l - i], acc[l][rt][ct]);
      }
      __builtin_amdgcn_sched_barrier(0);  // one column tile's B reads + MFMAs at a time (registers)
    }
  };
  // epilogue of tile i: D lane map of 16x16x64: sample 4 (lane >> 4) + r, entry lane & 15
  auto epilogue = [&](int i) {
    const int s_tile = tile_s(i), e_tile = tile_e(i);
    const bool u_tile = e_tile >= Ep;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int e = e_tile + 16 * ct + (lane & 15);
      const int col = u_tile ? e - Ep : e;
      if (u_tile ? col >= K : col >= E) continue;
      const double sc = a.ent[e], off0 = a.ent[NE + e];
      const double scl = i8_level_scale<ND>() * sc, offl = off0 * sc;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        // the lane's 4 consecutive samples of entry col: one vector store in the quad_index layout
        // (every sample of the rows is stored; those past sc are never read)
        const int s4 = s_tile + 32 * wave + 16 * rt + 4 * (lane >> 4);
        v4i lv[ND];
#pragma unroll
        for (int l = 0; l < ND; ++l) lv[l] = acc[l][rt][ct];
        double v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = i8_level_value<ND>(lv, r, scl, offl);
        if (u_tile) {
          double2* d = reinterpret_cast<double2*>(a.U + quad_index(s4, col, K));
          d[0] = make_double2(v[0], v[1]);
          d[1] = make_double2(v[2], v[3]);
        } else if (a.G32) {
          // non-temporal: the fp32 Gram streams to the LDL^T kernel without being allocated in L2,
          // where it evicted the A digits the XCD's other entry tiles still read (A fetched from
          // beyond L2 1.66 -> 1.36 GB per launch, configs[4] +1.7%; profiles/r5e)
          typedef float f4v __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store((f4v){(float)v[0], (float)v[1], (float)v[2], (float)v[3]},
                                      reinterpret_cast<f4v*>(a.G32 + quad_index(s4, col, E)));
        } else {
          double2* d = reinterpret_cast<double2*>(a.G + quad_index(s4, col, E));
          d[0] = make_double2(v[0], v[1]);
          d[1] = make_double2(v[2], v[3]);
        }
      }
    }
    zero_acc();
  };
  // Wait for this wave's outstanding loads (the next step's B DMA, which the compiler cannot see, and
  // A loads into Ar), then hand Ar through an empty asm that "redefines" it: the compiler's waitcnt
  // pass would otherwise still count those loads as pending and, at the first MFMA reading Ar, insert
  // a vmcnt(N) that does not count the DMA issued after them -- draining the NEXT step's prefetch.
  // (The epilogue's stores are outstanding here too; the vmcnt(0) waits for them as well.)
  auto land = [&](v4i (&Ar)[2][ND]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int p = 0; p < ND; ++p) asm volatile("" : "+v"(Ar[rt][p]));
    __syncthreads();  // everyone's DMA landed; the other LDS buffer is free again
  };
  // Two A register sets used in turn (even / odd global steps) and the loop unrolled by two: no
  // register copies; the conditional prefetches are safe for the waitcnt pass because every path
  // goes through land() before the registers are read.
  zero_acc();
  v4i A0r[2][ND], A1r[2][ND];
  prefetch(0, A0r, 0);
  land(A0r);
  for (int gs = 0; gs < nsteps; gs += 2) {
    const bool m1 = gs + 1 < nsteps, m2 = gs + 2 < nsteps;
    if (m1) prefetch(gs + 1, A1r, 1);
    compute(A0r, 0);
    if ((gs + 1) % nks == 0) epilogue(gs / nks);
    land(A1r);
    if (m2) prefetch(gs + 2, A0r, 0);
    if (m1) {
      compute(A1r, 1);
      if ((gs + 2) % nks == 0) epilogue((gs + 1) / nks);
    }
    land(A0r);
  }
}

// --------------------------------------------------------------------------------------------
// B-stationary Gram GEMM (24-bit path, ND = 3): one 8-wave block per CU keeps the WHOLE K range of
// one 64-entry tile's panel digits in LDS (nks x 12 KiB, nks <= kBstMaxKs) and streams sample tiles
// past it.  gemm_i8_kernel re-reads an entry tile's B digits from L2 for every 128-sample tile (a
// third of its L2 -> CU bytes); here each block reads them once, and after the prologue there is no
// barrier at all: each wave walks its own 32 samples x 64 entries of ALL its sample tiles as one
// stream of K steps (same MFMAs, same per-accumulator order as gemm_i8_kernel<3>: bit for bit its
// int32 sums and epilogue).  Software pipeline (round 5, +2.3% configs[4] over the round-3/4 kernel
// of 12 waves with A one step ahead, bitwise equal; profiles/round5/r10e): the A digits are loaded
// TWO K steps ahead into three register sets in turn (three steps ahead measured equal), every column
// tile's B operands are read from LDS one column tile ahead (two register sets), the next tile's
// first A loads are in flight during the epilogue, and the epilogue's column scales come from LDS;
// 2 waves per SIMD at 203 VGPRs, no spills (the round-4 kernel spilled 52 B per lane).
// Work: XCD x owns entry tiles x % EX and sample tiles x / EX (EX = 2: each sample tile's A digits
// are read by the 2 XCDs of its range; EX = 4 / 8 measured -1.3% / -5%, profiles/r5j); its blocks
// form nye entry-tile columns x G groups (at k = 50: 10 x 3 of an XCD's 32); round r of group gi
// covers sample tiles s0 + 2 (r G + gi) .. + 1 (one per 4 waves), so all of an XCD's blocks sweep the
// same 2 G sample tiles together and their A lines stay in its L2.
// --------------------------------------------------------------------------------------------
constexpr int kBstMaxKs = 13;                    // 13 x 12 KiB = 156 KiB of LDS: spectra up to 832 slots
constexpr int kBstEX = GPDLA_BST_EX;

constexpr int kBstWaves = 8;
constexpr int kBstLds = kBstMaxKs * 3 * kGTileE * 64;  // the Gram role's B image (the u role uses 2/3)
constexpr float kBstUSpare = GPDLA_BST_USPARE;           // share of the u tiles the spare blocks take
constexpr int kBstUDepth = 2;  // the u role's A prefetch depth (K steps; 3 measured equal, profiles/round5/ab/r10n)

// One role of the B-stationary launch.  A unit is W = 16 NCT consecutive entries starting at global
// entry ebase, whose B digits (ND planes, the whole K range) sit in Bs; the block's waves walk the
// sample tiles s_lo + kTiles (gi + r G) + (wave >> 2), r = 0, 1, ... below s_hi.
//   (ND, NCT) = (3, 4): a Gram entry tile, 6 digit pairs (levels <= 2), fp32 Gram out;
//   (ND, NCT) = (4, 2): half of the u entry tile, 10 digit pairs (levels <= 3), fp64 u out.
template <int ND, int NCT, int DEPTH>  // DEPTH: K steps of A digits in flight ahead of the one multiplied
__device__ inline void bst_run(const GemmI8Args& a, const SpecInfo& inf, uint8_t* Bs, double (*s_ent)[kGTileE],
                               int ebase, int s_lo, int s_hi, int gi, int G) {
  constexpr int W = 16 * NCT;
  constexpr bool kU = ND == 4;
  constexpr int kStepBytes = ND * W * 64;        // one K step of the unit: ND planes x W rows x 64 B
  constexpr int kTiles = kBstWaves / 4;          // 128-sample tiles per block round
  const int K = a.k;
  const int E = K * (K + 1) / 2;
  const int Ep = 64 * ((E + 63) / 64);
  const int NE = i8_gemm_entries(K);
  const int lane = threadIdx.x & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nks = (16 * ((inf.L + 15) / 16)) / 16;
  const int64_t nksmax = a.kstride / 64;
  const uint32_t bs_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)Bs;
  auto valid_entry = [&](int e) { return kU ? e - Ep < K : e < E; };
  {
    // the unit's B digits for every K step: 1 KiB pieces (16 rows x 64 B of one plane), round-robin
    // over the waves; the global image is [entry tile][K step][plane 4][row 64][64 B]
    const uint8_t* B0 = a.bdig + (int64_t)(ebase >> 6) * nksmax * 4 * 4096 + (int64_t)(ebase & 63) * 64;
    const int npieces = nks * (kStepBytes / 1024);
    for (int pc = wave_s; pc < npieces; pc += kBstWaves) {
      const int ks = pc / (kStepBytes / 1024), w = pc - ks * (kStepBytes / 1024);
      const int p = w / NCT, sub = w - p * NCT;
      dma_piece(B0 + (int64_t)ks * 4 * 4096 + p * 4096 + sub * 1024, (uint32_t)(lane * 16),
                bs_base + (uint32_t)(pc * 1024));
    }
    // the epilogue's per-entry scale and offset from LDS: a global load there would make the waitcnt
    // pass drain the A prefetches in flight at every tile's end
    if (threadIdx.x < W) {  // the column's epilogue constants scl, offl (i8_level_value)
      const int c = threadIdx.x, e = ebase + c;
      const double sc = valid_entry(e) ? a.ent[e] : 0.0, off0 = valid_entry(e) ? a.ent[NE + e] : 0.0;
      s_ent[0][c] = i8_level_scale<ND>() * sc;
      s_ent[1][c] = off0 * sc;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int g = lane >> 4;
  const int wt = wave_s & 3;                     // the wave's 32 rows of its 128-sample tile
  const uint32_t a_lane = (uint32_t)((g * 128 + 32 * wt + (lane & 15)) * 16);  // the lane's byte offset
  const uint8_t* adig = a.adig + (kU ? a.rows * a.kstride * 4 : 0);  // [type (Gram, u)][...]
  // this wave's sample tiles: st_i = st0 + i span, i = 0 .. nt - 1
  const int span = kTiles * G;
  const int st0 = s_lo + kTiles * gi + (wave_s >> 2);
  const int nt = st0 < s_hi ? (s_hi - st0 + span - 1) / span : 0;
  const int total = nt * nks;                    // the wave's K steps over all its tiles
  if (total == 0) return;                        // (after the block's only barrier)
  const int last = total - 1;
  v4i acc[ND][2][NCT];
  auto zero_acc = [&]() {
#pragma unroll
    for (int l = 0; l < ND; ++l)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[l][rt][ct] = (v4i){0, 0, 0, 0};
  };
  // global step gs -> (tile i, step ks); the A digits of that step into r.  Issued from inline asm,
  // invisible to the compiler's waitcnt pass (which, around the guarded steps and the tile-end
  // stores, merged its queue model conservatively and drained the prefetch two steps ahead); land()
  // waits for them explicitly and hands the registers over through an empty "+v" asm.
  // The step's base address is wave-uniform (SGPR pair, saddr form); the lane's offset is one fixed
  // VGPR, so a prefetch needs no VGPR address of its own.
  auto load_a = [&](int gs, v4i (&r)[2][ND]) {
    const int i = gs / nks, ks = gs - i * nks;
    const uint8_t* A0 = adig + ((int64_t)(st0 + i * span) * nksmax + ks) * 16 * 2048;
#pragma unroll
    for (int p = 0; p < ND; ++p) {
      const uint8_t* ap = A0 + p * 8192;
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r[0][p]) : "v"(a_lane), "s"(ap) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, %2 offset:256" : "=v"(r[1][p]) : "v"(a_lane), "s"(ap) : "memory");
    }
  };
  // A(g) has landed once at most CNT newer vector-memory operations are outstanding: 2 ND per later
  // A step already issued (vmcnt is in order; a tile-end epilogue's stores in between make the wait
  // longer, never too short).  Every call site passes a compile-time count, and no prefetch is issued
  // under a condition (see the pipeline below): tools/isa_inflight.py checks the shipped ISA for a
  // register touched while its load is in flight, which a guarded prefetch beside a guarded wait
  // makes undecidable for it (and a prefetch whose value is never read is exactly the round-5 fault:
  // its registers are free to the compiler while the hardware may still write them).
  auto land = [&](auto cnt, v4i (&r)[2][ND]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(cnt)::value) : "memory");
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int p = 0; p < ND; ++p) asm volatile("" : "+v"(r[rt][p]));
  };
  // B operands of column tile ct (rows 16 ct .. + 15 of the unit): K granule g of a row sits in 16-B
  // slot (g + 2 ((row >> 2) & 3)) & 3 of its 64 B (convert_gemm_i8_kernel's swizzle; a unit starts at
  // a multiple of 32 rows of its entry tile, so the local row gives the same slot)
  // ((row >> 2) & 3) does not depend on ct, so the lane's part of the address is one offset for every
  // column tile and plane (the rest folds into the ds_read offset)
  const int b_lane = (lane & 15) * 64 + 16 * ((g + 2 * (((lane & 15) >> 2) & 3)) & 3);
  auto read_b = [&](int ks, int ct, v4i (&Bd)[ND]) {
    const uint8_t* Bc = Bs + ks * kStepBytes + b_lane;
#pragma unroll
    for (int p = 0; p < ND; ++p)
      Bd[p] = *reinterpret_cast<const v4i*>(Bc + p * (W * 64) + 16 * ct * 64);
  };
  auto mfmas = [&](const v4i (&Ar)[2][ND], const v4i (&Bd)[ND], int ct) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int l = 0; l < ND; ++l)
#pragma unroll
        for (int i = 0; i <= l; ++i) acc[l][rt][ct] = MFMA_I8(Ar[rt][i], Bd[l - i], acc[l][rt][ct]);
  };
  // D lane map of 16x16x64: sample 4 (lane >> 4) + r, entry lane & 15
  auto epilogue = [&](int s_tile) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      int c = 16 * ct + (lane & 15);
      asm volatile("" : "+v"(c));   // the column's addresses stay inside the loop (hoisted, they spilled)
      const int e = ebase + c;
      if (!valid_entry(e)) continue;
      const double scl = s_ent[0][c], offl = s_ent[1][c];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int s4 = s_tile + 32 * wt + 16 * rt + 4 * (lane >> 4);
        v4i lv[ND];
#pragma unroll
        for (int l = 0; l < ND; ++l) lv[l] = acc[l][rt][ct];
        double v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = i8_level_value<ND>(lv, r, scl, offl);
        if constexpr (kU) {
          double2* d = reinterpret_cast<double2*>(a.U + quad_index(s4, e - Ep, K));
          d[0] = make_double2(v[0], v[1]);
          d[1] = make_double2(v[2], v[3]);
        } else {
          typedef float f4v __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store((f4v){(float)v[0], (float)v[1], (float)v[2], (float)v[3]},
                                      reinterpret_cast<f4v*>(a.G32 + quad_index(s4, e, E)));
        }
      }
    }
  };
  // one K step: B of (ks, ct = 0) is in Bb[0] on entry, B of the next step's ct = 0 in Bb[0] on exit
  // (NCT is even, so the two register sets alternate in step)
  v4i Bb[2][ND];
  int ks = 0, tile = 0;
  auto step = [&](auto cnt, v4i (&Ar)[2][ND]) {
    const int ksn = ks + 1 == nks ? 0 : ks + 1;
    land(cnt, Ar);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      __builtin_amdgcn_sched_barrier(0);
      if (ct + 1 < NCT) read_b(ks, ct + 1, Bb[(ct + 1) & 1]);
      else read_b(ksn, 0, Bb[0]);
      mfmas(Ar, Bb[ct & 1], ct);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (ksn == 0) {
      epilogue((st0 + tile * span) * kGTileS);
      zero_acc();
      ++tile;
    }
    ks = ksn;
  };
  zero_acc();
  // DEPTH + 1 A register sets in turn, A(g) in set g % NS.  Streams shorter than NS + DEPTH steps go
  // one step at a time.  Otherwise: the prologue issues A(0 .. DEPTH - 1); each main-loop round issues
  // A(gs + u + DEPTH) and multiplies A(gs + u) for u < NS, all unconditionally (the loop runs while
  // the round's last prefetch exists), each wait retiring exactly the set about to be read; the tail
  // (R = total - gs in [DEPTH, NS - 1 + DEPTH] steps left, A(gs .. gs + DEPTH - 1) in flight) is one
  // straight-line sequence per R, its waits counting the prefetches that remain.  Same steps in the
  // same order as a single guarded loop: bit for bit the same sums.
  constexpr int NS = DEPTH + 1;
  v4i Ar[NS][2][ND];
  if (total < NS + DEPTH) {
    read_b(0, 0, Bb[0]);
    for (int g = 0; g < total; ++g) {
      load_a(g, Ar[0]);
      step(std::integral_constant<int, 0>{}, Ar[0]);
    }
    return;
  }
  static_for<DEPTH>([&](auto u) { load_a(decltype(u)::value, Ar[decltype(u)::value]); });
  read_b(0, 0, Bb[0]);
  int gs = 0;
  do {
    static_for<NS>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      load_a(gs + u + DEPTH, Ar[(u + DEPTH) % NS]);
      step(std::integral_constant<int, 2 * ND * DEPTH>{}, Ar[u]);
    });
    gs += NS;
  } while (gs + NS - 1 + DEPTH <= last);
  // tail: R = total - gs in [DEPTH, NS - 1 + DEPTH] steps left.  A(gs .. gs + DEPTH - 1) are in flight
  // in Ar[0 .. DEPTH - 1]; the rest are loaded one step at a time (the wave's last NS - 1 steps at
  // most), each load waited for before its registers are read.
  const int R = total - gs;
  static_for<NS - 1 + DEPTH>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    if constexpr (t < DEPTH) {
      constexpr int ahead = DEPTH - 1 - t;   // loads of A(gs + t + 1 .. gs + DEPTH - 1) still newer
      step(std::integral_constant<int, 2 * ND * ahead>{}, Ar[t]);
    } else if (t < R) {
      load_a(gs + t, Ar[t % NS]);
      step(std::integral_constant<int, 0>{}, Ar[t % NS]);
    }
  });
}

// The launch: per XCD, nye entry-tile columns x G groups of Gram blocks; when the u tile is fused
// (a.u_tile >= 0), the XCD's two spare blocks (32 - nye G = 2 at k = 50) take the two halves of the
// u tile over the XCD's share of its sample range (the two XCDs of a sample range split it), so the
// u contraction runs beside the Gram's instead of as a launch of its own.
__global__ __launch_bounds__(64 * kBstWaves, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void gemm_i8_bst_kernel(GemmI8Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t Bs[kBstLds];
  __shared__ double s_ent[2][kGTileE];
  const SpecInfo inf = a.info[a.q];
  if (inf.J == 0) return;
  const int ny = a.ny, nst = (a.sc + kGTileS - 1) / kGTileS;
  const int EX = kBstEX, SX = 8 / EX;
  const int per = gridDim.x / 8;
  const int x = blockIdx.x % 8;
  const int ex = x % EX, sx = x / EX;
  const int e0 = ny * ex / EX, e1 = ny * (ex + 1) / EX;
  const int s0 = nst * sx / SX, s1 = nst * (sx + 1) / SX;
  const int nye = e1 - e0;
  const int G = per / nye;
  const int j = blockIdx.x / 8;
  if (nye <= 0 || G <= 0) return;
  const int nks = (16 * ((inf.L + 15) / 16)) / 16;
  if (nks > kBstMaxKs) return;                   // never: the launch checks the bound (LDS safety)
  // the u work of this XCD: both halves of the u tile over its share [lo, hi) of the sample range; a
  // spare block per half takes the first kBstUSpare of the tiles (it starts at once), the Gram blocks
  // split the rest per half once their Gram columns are done.  A u tile takes a spare block ~2x the
  // time a Gram tile takes a Gram block (the u role is bound by its A stream: 4 digit planes for 2 x
  // 10 MFMA pairs), hence the split (tuning.h); the u launch this replaces cost 0.085 ms per
  // spectrum and 100,001 samples, the fused launch +0.03 ms over the Gram alone (profiles/round5)
  const int lo = s0 + (s1 - s0) * ex / EX, hi = s0 + (s1 - s0) * (ex + 1) / EX;
  const int mid = lo + (int)((hi - lo) * kBstUSpare + 0.5f);
  if (j < nye * G) {
    bst_run<3, 4, 2>(a, inf, Bs, s_ent, (a.e_tile0 + e0 + j % nye) * kGTileE, s0, s1, j / nye, G);
    if (a.u_tile >= 0 && nye * G >= 2) {
      __syncthreads();                           // every wave is done with the Gram B image
      const int half = j & 1, ngb = nye * G / 2;
      if (j / 2 < ngb) bst_run<4, 2, kBstUDepth>(a, inf, Bs, s_ent, a.u_tile * kGTileE + 32 * half, mid, hi, j / 2, ngb);
    }
  } else if (a.u_tile >= 0 && j < nye * G + 2) {
    const int half = j - nye * G;
    bst_run<4, 2, kBstUDepth>(a, inf, Bs, s_ent, a.u_tile * kGTileE + 32 * half, lo, mid, 0, 1);
  }
}

#undef MFMA_I8

}  // namespace

hipError_t launch_convert_gemm_i8(const ConvertGemmI8Args& a, int32_t q_count, hipStream_t s) {
  if (a.k < 1 || a.k > kGemmMaxK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(convert_gemm_i8_kernel, dim3((unsigned)(i8_gemm_entries(a.k) / 64), (unsigned)q_count),
                     dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_diag_raw_profile(const double* lam, int64_t n, double z, double N, int32_t f32,
                                   const LineArgs& lines, double* out, hipStream_t s) {
  if (n < 1) return hipSuccess;
  const unsigned blocks = (unsigned)(((n + 1) / 2 + 255) / 256);
  hipLaunchKernelGGL(diag_raw_profile_kernel, dim3(blocks), dim3(256), 0, s, lam, n, z, N, f32, lines, out);
  return hipGetLastError();
}

hipError_t launch_weights_i8(const WeightsI8Args& a, hipStream_t s) {
  // the 24-bit path (3 Gram digit planes) takes the fp32 raw profiles
  const dim3 grid((unsigned)((a.sc + 63) / 64), kWeightQuarters);
  if (a.nd == 3)
    hipLaunchKernelGGL(weights_i8_kernel<true>, grid, dim3(256), 0, s, a, a.srow);
  else
    hipLaunchKernelGGL(weights_i8_kernel<false>, grid, dim3(256), 0, s, a, a.srow);
  return hipGetLastError();
}

// nd = 4: one launch over all entry tiles.  nd = 3: the Gram tiles on the 3-digit kernel, then the u
// tiles on the 4-digit one (the u contraction carries most of the 24-bit scheme's error: emulated
// 2.1e-7 with 3 u digits, 7e-8 with 4, tests/support/emulate_i8.py; the u tiles are 1 of 21 at k = 50).
hipError_t launch_gemm_i8(const GemmI8Args& a0, hipStream_t s) {
  if (a0.k < 1 || a0.k > kGemmMaxK || a0.rows % kGTileS != 0 || a0.rows < a0.sc || a0.kstride % 64 != 0 ||
      (a0.nd != 3 && a0.nd != 4))
    return hipErrorInvalidValue;
  const int K = a0.k, Ep = 64 * ((K * (K + 1) / 2 + 63) / 64);
  const int ng = Ep / kGTileE, nu = i8_gemm_entries(K) / kGTileE - ng;
  const int nst = (a0.sc + kGTileS - 1) / kGTileS;
  // persistent grid: at most the resident blocks (3 or 2 per CU), a multiple of 8 (one run per XCD)
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  auto grid = [&](int ny, int per_cu) {
    const int nb = std::min(nst * ny, per_cu * ncu);
    return dim3((unsigned)((nb + 7) / 8 * 8));
  };
  GemmI8Args a = a0;
  if (a0.nd == 4) {
    a.e_tile0 = 0; a.ny = ng + nu;
    hipLaunchKernelGGL(gemm_i8_kernel<4>, grid(a.ny, 2), dim3(256), 0, s, a);
  } else {
    a.e_tile0 = 0; a.ny = ng;
    // B-stationary when the spectrum's K steps fit the block's LDS
    if (a0.ks_bound > 0 && a0.ks_bound <= kBstMaxKs && ng >= kBstEX && a0.G32 && ncu % 8 == 0) {
      // the u tile on the two spare blocks per XCD when the Gram columns leave them (k = 50: 10 x 3 of
      // 32) and there is one u tile (k <= 64)
      const int per = ncu / 8, nye_max = (ng + kBstEX - 1) / kBstEX, nye_min = ng / kBstEX;
      const bool fuse_u = nu == 1 && nye_min > 0 && per - nye_min * (per / nye_min) >= 2 &&
                          per - nye_max * (per / nye_max) >= 2;
      a.u_tile = fuse_u ? ng : -1;
      hipLaunchKernelGGL(gemm_i8_bst_kernel, dim3((unsigned)ncu), dim3(64 * kBstWaves), 0, s, a);
      if (fuse_u) return hipGetLastError();
    } else {
      hipLaunchKernelGGL(gemm_i8_kernel<3>, grid(a.ny, 3), dim3(256), 0, s, a);
    }
    a.e_tile0 = ng; a.ny = nu;
    hipLaunchKernelGGL(gemm_i8_kernel<4>, grid(a.ny, 2), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace gpdla
