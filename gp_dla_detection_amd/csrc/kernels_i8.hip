// Int8 (Ozaki-sliced) fused likelihood sweep for gfx950: the same per-(spectrum, sample) math as
// likelihood_kernel in kernels.hip (process_qsos.m:184-197, voigt.c:282-299,
// log_mvnpdf_low_rank.m:11-32), with the Khatri-Rao Gram/u contraction moved from the fp64 pipe
// to v_mfma_i32_16x16x64_i8.  The contraction is exact in integers; the only approximation is the
// 2^-30 quantisation of the weights and panel entries and the dropped digit levels >= 5
// (error budget).  Everything else (Voigt profile, modulation, residuals,
// sum r^2/d, log det D, the LDL^T) stays fp64 as in the fp64 kernel.
//
// The f64 VALU work per (sample, pixel) is unchanged, but the fp64 matrix pipe is no longer
// shared with it: the int8 MFMAs of a 64-slot chunk (13 digit pairs x kTiles tiles) take about
// half of the VALU time of the chunk.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

constexpr int kI8Levels = 4;  // digit levels i + j = 0..3 kept (10 of the 16 pairs)

// ---------------------------------------------------------------------------------------------
// convert: fp64 fused panel (prep_kernel<K>) -> int8 digit planes + slot records + entry scales.
// One block per spectrum, thread e = entry (kEnt <= 256).
// i8 slot (segment g, step t), t < 16 nch: chunk c = t / 16, MFMA K index k = 16 g + t % 16.
// Source fp64 row: g Ls4 + t for t < L (rows with position >= J are neutral there already),
// neutral for t >= L.
// ---------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void convert_i8_kernel(ConvertI8Args a) {
  using F = Layout<K>;
  using I = I8Layout<K>;
  static_assert(I::kEnt <= 256, "one thread per entry");
  const int q = blockIdx.x;
  const int e = threadIdx.x;
  const SpecInfo inf = a.info[q];
  if (inf.J == 0) return;
  const int L = inf.L;
  const int Ls4 = ((L + kChunkSteps - 1) / kChunkSteps) * kChunkSteps;
  const int nch = (L + 15) / 16;
  const double* panel = a.panel + inf.slot_base * F::kRow;
  const int64_t cb = a.chunk_base[q];

  int src = -1;
  bool is_u = false;
  if (e < F::kNGram) {
    src = (e & 3) * F::kJS + (e >> 2);
  } else if (e >= I::kUBase && e - I::kUBase < K) {
    const int kr = 4 * F::kGT + (e - I::kUBase);
    src = (kr & 3) * F::kJS + (kr >> 2);
    is_u = true;
  }
  auto value = [&](const double* row) -> double {
    if (src < 0) return 0.0;
    const double y = row[F::kY], noise = row[F::kNoise], mu = row[F::kMu], om2 = row[F::kOmega2];
    return is_u ? row[src] * u_bound(y, mu, noise) : row[src] / (om2 + noise);
  };

  // pass 1: per-entry max |P~| -> scale s_e = max / (127 2^24), so |X_B| <= 127 2^24 and the top
  // balanced digit stays within [-127, 127]
  double mx = 0.0;
  if (e < I::kEnt) {
    for (int g = 0; g < 4; ++g)
      for (int t = 0; t < L; ++t) mx = fmax(mx, fabs(value(panel + (int64_t)(g * Ls4 + t) * F::kRow)));
  }
  const double s_e = mx > 0.0 ? mx * (1.0 / (127.0 * 0x1p24)) : 1.0;

  // pass 2: balanced base-256 digits of X_B = rint(P~ / s_e), 16 slots per 16 B store
  int64_t colsum = 0;
  if (e < I::kEnt) {
    for (int g = 0; g < 4; ++g) {
      for (int c = 0; c < nch; ++c) {
        uint32_t pl[4][4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
#pragma unroll
          for (int j = 0; j < 4; ++j) pl[j][w] = 0u;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int t = 16 * c + 4 * w + b;
            const double v = t < L ? value(panel + (int64_t)(g * Ls4 + t) * F::kRow) : 0.0;
            int X = (int)rint(v / s_e);
            colsum += X;
            const int d3 = ((X + 128) & 255) - 128; X = (X - d3) >> 8;
            const int d2 = ((X + 128) & 255) - 128; X = (X - d2) >> 8;
            const int d1 = ((X + 128) & 255) - 128; X = (X - d1) >> 8;
            const int d0 = X;
            pl[0][w] |= (uint32_t)(d0 & 255) << (8 * b);
            pl[1][w] |= (uint32_t)(d1 & 255) << (8 * b);
            pl[2][w] |= (uint32_t)(d2 & 255) << (8 * b);
            pl[3][w] |= (uint32_t)(d3 & 255) << (8 * b);
          }
        }
        uint8_t* base = a.panel_i8 + (cb + c) * (int64_t)I::kChunkBytes + e * 64 + 16 * ((g + 2 * ((e >> 2) & 3)) & 3);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<uint4*>(base + j * I::kPlaneBytes) = make_uint4(pl[j][0], pl[j][1], pl[j][2], pl[j][3]);
      }
    }
    // epilogue constants: value = (sum_l 2^(8(6-l)) C_l + c colsum_e) s_e / scaleA, with the digit
    // offset c = 0x80808080 (Gram: X_A = U) or 0x808080 (u: X_A = U - 2^31)
    const bool u_tile = e >= I::kUBase;
    a.ent[(int64_t)q * 2 * I::kEnt + e] = s_e / (u_tile ? kI8ScaleU : kI8ScaleG);
    a.ent[(int64_t)q * 2 * I::kEnt + I::kEnt + e] = (u_tile ? 8421504.0 : 2155905152.0) * (double)colsum;
  }

  // slot records: lam at padded position + 6, y, noise, mu, om2, gscale, uscale
  const double* lamp = a.lam_pad + inf.lam_base;
  for (int id = threadIdx.x; id < 4 * 16 * nch; id += 256) {
    const int g = id / (16 * nch), t = id - g * 16 * nch;
    const int c = t >> 4, k = 16 * g + (t & 15);
    double* rec = a.scal + ((cb + c) * I::kChunkSlots + k) * I::kScal;
    double y = 0.0, noise = 1.0, mu = 0.0, om2 = 0.0;
    if (t < L) {
      const double* row = panel + (int64_t)(g * Ls4 + t) * F::kRow;
      y = row[F::kY]; noise = row[F::kNoise]; mu = row[F::kMu]; om2 = row[F::kOmega2];
    }
    rec[0] = lamp[g * L + t + 2 * kWidth];
    rec[1] = y;
    rec[2] = noise;
    rec[3] = mu;
    rec[4] = om2;
    rec[5] = (om2 + noise) * kI8ScaleG;
    rec[6] = kI8ScaleU / u_bound(y, mu, noise);
    rec[7] = 0.0;
  }
}

// LDS-DMA of `pieces` 1 KiB pieces from global src to LDS dst (M0), one global_load_lds_dwordx4
// per piece (same hazard notes as stage_chunk in kernels.hip).
__device__ inline void dma_pieces(const uint8_t* src, uint32_t dst, int pieces, uint32_t voff) {
  for (int h = 0; h < pieces; ++h) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(dst + h * 1024), "v"(voff), "s"(src + h * 1024) : "memory", "m0");
#pragma clang diagnostic pop
  }
}

#define MFMA_I8(A, B, C) __builtin_amdgcn_mfma_i32_16x16x64_i8((A), (B), (C), 0, 0, 0)

// ---------------------------------------------------------------------------------------------
// likelihood (int8 contraction): one spectrum x 64 samples per block (4 waves x 16), one block
// per CU (the double-buffered 64-slot chunks take ~150 KB of LDS).  Lane (sample s = lane & 15,
// segment g = lane >> 4) computes the weights of its 16 consecutive slots of the chunk; they are
// exactly its MFMA A-operand K range (k = 16 g + 0..15).
// ---------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256, 1) void likelihood_i8_kernel(LikelihoodI8Args a) {
  using F = Layout<K>;
  using I = I8Layout<K>;
  constexpr int NT = I::kTiles;
  constexpr int kWingLds = 4 * ((3 * kWingStride + 3) / 4);
  constexpr int kSBuf = I::kChunkSlots * I::kScal;  // doubles per slot-record buffer
  __shared__ __attribute__((aligned(16))) uint8_t ldsb[2 * I::kChunkBytes];
  __shared__ __attribute__((aligned(16))) double ldss[2 * kSBuf + 3 * kCoreTable + kWingLds + 64];
  double* core_lds = ldss + 2 * kSBuf;
  double* wing_lds = core_lds + 3 * kCoreTable;
  double* exp_lds = wing_lds + kWingLds;

  // XCD-aware block order, as likelihood_kernel
  const int64_t blocks_x = (a.S + 1 + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const int64_t per_xcd = gridDim.x / 8;
  const int64_t v = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (v >= blocks_x * a.q_count) return;
  const int q = (int)(v / blocks_x);
  const int64_t bx = v - (int64_t)q * blocks_x;
  const SpecInfo inf = a.info[q];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t s_base = bx * kSamplesPerBlock + wave * kSamplesPerWave;
  if (inf.J == 0) {
    const int64_t su = s_base + (lane >> 2);
    if ((lane & 3) == 0 && su < a.S && a.sample_ll) a.sample_ll[q * a.ld + su] = NAN;
    if ((lane & 3) == 0 && su == a.S) a.ll_null[q] = NAN;
    return;
  }
  const int L = inf.L;
  const int nch = (L + 15) / 16;
  const int64_t cb = a.chunk_base[q];
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t ldsb_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)ldsb;
  const uint32_t ldss_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)ldss;
  const uint32_t voff = (uint32_t)(lane * 16);
  constexpr int kBPieces = I::kChunkBytes / 1024 / kWavesPerBlock;  // per wave
  static_assert(I::kChunkBytes % (1024 * kWavesPerBlock) == 0, "B chunk splits into whole pieces");
  static_assert(I::kScalBytes == 1024 * kWavesPerBlock, "one record piece per wave");
  auto stage_b = [&](int c, int buf) {
    const uint8_t* bsrc = a.panel_i8 + (cb + c) * (int64_t)I::kChunkBytes + wave_s * kBPieces * 1024;
    dma_pieces(bsrc, ldsb_base + (uint32_t)(buf * I::kChunkBytes + wave_s * kBPieces * 1024), kBPieces, voff);
  };
  auto stage_rec = [&](int c, int buf) {
    const uint8_t* ssrc = reinterpret_cast<const uint8_t*>(a.scal + (cb + c) * kSBuf) + wave_s * 1024;
    dma_pieces(ssrc, ldss_base + (uint32_t)(buf * kSBuf * 8 + wave_s * 1024), 1, voff);
  };
  auto stage = [&](int c, int buf) {
    stage_b(c, buf);
    stage_rec(c, buf);
  };

  // software pipeline: iteration c computes chunk c's weights while its MFMAs contract chunk c-1
  // (digits kept from the previous iteration, B planes in buffer (c-1)&1; B(c) is staged into
  // buffer c&1 during iteration c).  Iteration 0 contracts an all-zero "chunk -1" (buffer 1).
  static_assert(I::kTiles == 16, "one tile per slot of the 16-slot stage");
  stage_rec(0, 0);
  for (int i = threadIdx.x; i < I::kChunkBytes / 16; i += 256)
    reinterpret_cast<uint4*>(ldsb + I::kChunkBytes)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = threadIdx.x; i < 3 * kCoreTable; i += 256) core_lds[i] = a.lines.buf[i];
  if (threadIdx.x < 64) exp_lds[threadIdx.x] = a.lines.buf[kLineBufExp2 + threadIdx.x];
  if (threadIdx.x < 3 * kWingStride) wing_lds[threadIdx.x] = a.lines.buf[kLineBufWing + threadIdx.x];

  const int g = lane >> 4;
  const int64_t s = s_base + (lane & 15);
  const double off = (s < a.S) ? a.offsets[s] : 0.5;
  const double N = (s < a.S) ? a.nhi[s] : 0.0;  // null model / idle lanes: absorption 1 exactly
  const double zdla = inf.zmin + (inf.zmax - inf.zmin) * off;  // process_qsos.m:163-165
  const double zfac = 1.0 / (1 + zdla);
  double afac[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) afac[j] = a.lines.buf[kLineBufFac + j] * zfac;
  const double* lamp = a.lam_pad + inf.lam_base + (int64_t)g * L;
  double lw[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) lw[i] = lamp[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // damping-wing coefficients from LDS (broadcast reads, lgkmcnt): vector loads from global
  // memory here would wait on vmcnt behind the next chunk's LDS-DMA and serialise it with compute
  const double* wing_g = wing_lds;
  auto raw = [&](double lam) { return raw_profile3(lam, afac, N, core_lds, wing_lds, exp_lds); };
  double w0 = raw(lw[0]), w1 = raw(lw[1]), w2 = raw(lw[2]);
  double w3 = raw(lw[3]), w4 = raw(lw[4]), w5 = raw(lw[5]);

  v4i acc[kI8Levels][NT];
#pragma unroll
  for (int l = 0; l < kI8Levels; ++l)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[l][t] = (v4i){0, 0, 0, 0};
  double q1 = 0.0, pm = 1.0;
  int pe = 0;

  v4i Apg[4], Apu[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) Apg[i] = Apu[i] = (v4i){0, 0, 0, 0};
  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) stage_rec(c + 1, cur ^ 1);
    stage_b(c, cur);
    const uint8_t* bp = ldsb + (cur ^ 1) * I::kChunkBytes;  // B planes of chunk c - 1
    auto load_bp = [&](int t, v4i (&Bt)[4]) {
      const int ent = 16 * t + (lane & 15);
      const int boff = ent * 64 + 16 * ((g + 2 * ((ent >> 2) & 3)) & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) Bt[j] = *reinterpret_cast<const v4i*>(bp + j * I::kPlaneBytes + boff);
    };
    v4i Bq[4];
    // ---- weights of this lane's 16 slots (fp64), quantised to X_A + 2^31, digits XOR 0x80
    const double* rec = ldss + cur * kSBuf + (16 * g) * I::kScal;
    // (1) line sums of the 16 slots, branch-free damping wings (one basic block: the scheduler
    //     interleaves the 16 independent chains), coefficients in SGPRs (uniform global loads)
    double tot[16];
    uint32_t cm = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const double lam = rec[e * I::kScal];
      double t = 0.0;
      const double x0 = fma(lam, afac[0], -kC2), x1 = fma(lam, afac[1], -kC2), x2 = fma(lam, afac[2], -kC2);
      cm |= (((fabs(x0) < kOuterX) | (fabs(x1) < kOuterX) | (fabs(x2) < kOuterX)) ? 1u : 0u) << e;
      double T0, T1, T2;
      wing_T3(x0, x1, x2, T0, T1, T2);
      t -= outer_poly(wing_g, T0);
      t -= outer_poly(wing_g + kWingStride, T1);
      t -= outer_poly(wing_g + 2 * kWingStride, T2);
      tot[e] = t;
    }
    // (2) rare fix-up (z-sorted samples: a few % of wave-chunks): the lanes with some |x| < kOuterX
    //     recomputed in raw_profile3's evaluation (core polynomial or inner wing)
    if (cm) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if (cm & (1u << e)) {
          const double lam = rec[e * I::kScal];
          double t = 0.0;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const double x = fma(lam, afac[j], -kC2);
            const double ax = fabs(x);
            double f = wing_eval(wing_g + j * kWingStride, x);
            if (ax < kCoreX) f = core_eval(core_lds + j * kCoreTable, ax);
            t -= f;
          }
          tot[e] = t;
        }
      }
    }
    // (3) the 16 table exps (their LDS lookups in flight together)
    double rw[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      rw[e] = exp_tab64(N * tot[e], exp_lds);  // voigt.c:291
    }
    // (4) 7-tap convolution, pixel terms, weights; slot records prefetched one slot ahead
    uint32_t xg[16], xu[16];
    double2 n01 = *reinterpret_cast<const double2*>(rec + 0);
    double2 n23 = *reinterpret_cast<const double2*>(rec + 2);
    double2 n45 = *reinterpret_cast<const double2*>(rec + 4);
    double nus = rec[6];
    load_bp(0, Bq);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      {  // tile e of chunk c - 1 (its 10 MFMAs run beside this slot's VALU work)
        const v4i B0 = Bq[0], B1 = Bq[1], B2 = Bq[2], B3 = Bq[3];
        if (e + 1 < 16) load_bp(e + 1, Bq);
        const v4i* A = e < I::kGT ? Apg : Apu;
        acc[0][e] = MFMA_I8(A[0], B0, acc[0][e]);
        acc[1][e] = MFMA_I8(A[0], B1, acc[1][e]);
        acc[1][e] = MFMA_I8(A[1], B0, acc[1][e]);
        acc[2][e] = MFMA_I8(A[0], B2, acc[2][e]);
        acc[2][e] = MFMA_I8(A[1], B1, acc[2][e]);
        acc[2][e] = MFMA_I8(A[2], B0, acc[2][e]);
        acc[3][e] = MFMA_I8(A[0], B3, acc[3][e]);
        acc[3][e] = MFMA_I8(A[1], B2, acc[3][e]);
        acc[3][e] = MFMA_I8(A[2], B1, acc[3][e]);
        acc[3][e] = MFMA_I8(A[3], B0, acc[3][e]);
      }
      const double y = n01.y, noise = n23.x, mu = n23.y, om2 = n45.x, gs = n45.y, us = nus;
      if (e + 1 < 16) {
        n01 = *reinterpret_cast<const double2*>(rec + (e + 1) * I::kScal);
        n23 = *reinterpret_cast<const double2*>(rec + (e + 1) * I::kScal + 2);
        n45 = *reinterpret_cast<const double2*>(rec + (e + 1) * I::kScal + 4);
        nus = rec[(e + 1) * I::kScal + 6];
      }
      const double w6 = rw[e];
      double ab = w0 * kInstrumentProfile[0];  // voigt.c:297-299
      ab = fma(w1, kInstrumentProfile[1], ab);
      ab = fma(w2, kInstrumentProfile[2], ab);
      ab = fma(w3, kInstrumentProfile[3], ab);
      ab = fma(w4, kInstrumentProfile[4], ab);
      ab = fma(w5, kInstrumentProfile[5], ab);
      ab = fma(w6, kInstrumentProfile[6], ab);
      w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6;
      const double r = fma(-mu, ab, y);  // process_qsos.m:191-197, log_mvnpdf_low_rank.m:11-15
      const double a2 = ab * ab;
      const double d = fma(om2, a2, noise);
      const double dinv = rcp_sweep(d);
      const double rd = r * dinv;
      const double wg = a2 * dinv;
      const double wu = ab * rd;
      q1 = fma(r, rd, q1);
      pm *= d;
      xg[e] = (uint32_t)__builtin_rint(wg * gs) ^ 0x80808080u;
      xu[e] = (uint32_t)__builtin_rint(fma(wu, us, 0x1p31)) ^ 0x80808080u;
    }
    {
      int ex;
      pm = frexp(pm, &ex);
      pe += ex;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Apg[i] = digit_plane(xg, i);
      Apu[i] = digit_plane(xu, i);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (rec c+1, B c) landed
    __syncthreads();
  }
  // drain: contract the last chunk
  {
    const v4i* Ag = Apg;
    const v4i* Au = Apu;
    const uint8_t* bb = ldsb + ((nch - 1) & 1) * I::kChunkBytes;
    // ---- exact int8 contraction: the 10 digit pairs of level i + j <= 3 per tile
    auto load_b = [&](int t, v4i (&Bt)[4]) {
      const int ent = 16 * t + (lane & 15);
      const int boff = ent * 64 + 16 * ((g + 2 * ((ent >> 2) & 3)) & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) Bt[j] = *reinterpret_cast<const v4i*>(bb + j * I::kPlaneBytes + boff);
    };
    v4i Bn[4];
    load_b(0, Bn);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // B digits of tile t were loaded one tile ahead (their LDS latency hides behind the
      // previous tile's MFMAs)
      const v4i B0 = Bn[0], B1 = Bn[1], B2 = Bn[2], B3 = Bn[3];
      if (t + 1 < NT) load_b(t + 1, Bn);
      const v4i* A = t < I::kGT ? Ag : Au;
      acc[0][t] = MFMA_I8(A[0], B0, acc[0][t]);
      acc[1][t] = MFMA_I8(A[0], B1, acc[1][t]);
      acc[1][t] = MFMA_I8(A[1], B0, acc[1][t]);
      acc[2][t] = MFMA_I8(A[0], B2, acc[2][t]);
      acc[2][t] = MFMA_I8(A[1], B1, acc[2][t]);
      acc[2][t] = MFMA_I8(A[2], B0, acc[2][t]);
      acc[3][t] = MFMA_I8(A[0], B3, acc[3][t]);
      acc[3][t] = MFMA_I8(A[1], B2, acc[3][t]);
      acc[3][t] = MFMA_I8(A[2], B1, acc[3][t]);
      acc[3][t] = MFMA_I8(A[3], B0, acc[3][t]);
      __builtin_amdgcn_sched_barrier(0);  // keep one tile's B digits live at a time
    }
  }

  // ---- combine the 4 segments of each sample (lanes l, l^16, l^32, l^48)
  q1 += __shfl_xor(q1, 16);
  q1 += __shfl_xor(q1, 32);
#pragma unroll
  for (int off2 = 16; off2 <= 32; off2 <<= 1) {
    const double pm2 = __shfl_xor(pm, off2);
    const int pe2 = __shfl_xor(pe, off2);
    int ex;
    pm = frexp(pm * pm2, &ex);
    pe += pe2 + ex;
  }

  // ---- epilogue: integer level sums -> fp64 Gram/u entries in the fp64 kernel's scratch-row
  //      layout (Layout<K>), then the same augmented LDL^T.
  //      D lane map of 16x16x64: sample 4 (lane >> 4) + r, entry 16 t + (lane & 15).
  double* scr = a.scratch + (v * kSamplesPerBlock + wave * kSamplesPerWave) * F::kES;
  const double* ent_q = a.ent + (int64_t)q * 2 * I::kEnt;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int ent = 16 * t + (lane & 15);
    int pos = -1;
    if (t < I::kGT) pos = ent < I::kNGram ? ent : -1;                            // gram_index order
    else pos = (ent - I::kUBase) < K ? 4 * F::kGT + (ent - I::kUBase) : -1;      // u_i
    if (pos >= 0) {
      const double sc = ent_q[ent];
      const double off0 = ent_q[I::kEnt + ent];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double val = (double)acc[3][t][r] * 0x1p24;
        val = fma((double)acc[2][t][r], 0x1p32, val);
        val = fma((double)acc[1][t][r], 0x1p40, val);
        val = fma((double)acc[0][t][r], 0x1p48, val);
        scr[(4 * (lane >> 4) + r) * F::kES + pos] = (val + off0) * sc;
      }
    }
  }
  if (lane < 16) {
    double* scl = scr + lane * F::kES + 4 * F::kTiles;
    scl[0] = q1;
    scl[1] = pm;
    scl[2] = (double)pe + inf.de_shift;  // prep's unit scaling (kernels.hip prep_kernel)
  }
  __syncthreads();
  const int jq = lane & 3, sq = lane >> 2;
  const int64_t s2 = s_base + sq;
  bool bad;
  const double ll = ldl_log_likelihood<K>(scr + sq * F::kES, jq, inf.n, bad);
  if (jq == 0 && s2 <= a.S) {
    if (bad) atomicOr(a.status, 1);
    if (s2 == a.S) a.ll_null[q] = ll;
    else if (a.sample_ll) a.sample_ll[q * a.ld + a.perm[s2]] = ll;
  }
}

#undef MFMA_I8

template <int K>
hipError_t launch_convert_i8_k(const ConvertI8Args& a, hipStream_t s) {
  hipLaunchKernelGGL(convert_i8_kernel<K>, dim3(a.q_count), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int K>
hipError_t launch_likelihood_i8_k(const LikelihoodI8Args& a, hipStream_t s) {
  const int64_t blocks_x = (a.S + 1 + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const int64_t nb = (blocks_x * a.q_count + 7) / 8 * 8;  // padded for the XCD remap
  if (nb > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(likelihood_i8_kernel<K>, dim3((unsigned)nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

#define GPDLA_FOR_EACH_I8_RANK(X) X(20)

bool i8_supported(int K) {
#define X(k) if (K == k) return true;
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return false;
}

// smallest compiled int8 fused rank >= k (0: none); lower ranks run zero-padded (fused_rank, kernels.hip;
// a zero panel column quantises to zero digits, so the padding stays exact here too)
int i8_fused_rank(int k) {
  if (k < 1) return 0;
#define X(kk) if (k <= kk) return kk;
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return 0;
}

int i8_chunk_bytes(int K) {
#define X(k) if (K == k) return I8Layout<k>::kChunkBytes;
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return 0;
}

int i8_entries(int K) {
#define X(k) if (K == k) return I8Layout<k>::kEnt;
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return 0;
}

hipError_t launch_convert_i8(int K, const ConvertI8Args& a, hipStream_t s) {
#define X(k) if (K == k) return launch_convert_i8_k<k>(a, s);
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_likelihood_i8(int K, const LikelihoodI8Args& a, hipStream_t s) {
#define X(k) if (K == k) return launch_likelihood_i8_k<k>(a, s);
  GPDLA_FOR_EACH_I8_RANK(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace gpdla
