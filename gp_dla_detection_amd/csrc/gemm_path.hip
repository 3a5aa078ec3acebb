// Panel-GEMM path for any rank k <= kGemmMaxK (BASELINE configs[4]: k = 50): the north star's
// "MFMA for the n x k panel contraction" branch.  Per (spectrum, chunk of samples):
//   weights_kernel    Voigt absorption x pixel terms (process_qsos.m:186-197) ->
//                     Wg[slot][s] = a^2/d, Wu[slot][s] = a r/d, per-segment sum r^2/d, sum log d
//   gemm_f64_kernel   Gram[s] = PG^T Wg[:, s] (Khatri-Rao panel, k(k+1)/2 columns) and
//                     u[s] = M^T Wu[:, s] on the f64 matrix cores (gemm_f64.hip), or the int8
//                     digit GEMM of gemm_i8.hip  -- log_mvnpdf_low_rank.m:13-23
//   ldl_mfma_kernel   augmented LDL^T of [[I + Gram, u], [u', sum r^2/d]] per sample -> logdet and
//                     r'K^-1 r (log_mvnpdf_low_rank.m:24-32), 4 samples per wave on the f64
//                     matrix cores.
// Slot layout, neutral padding rows and sample order are those of the fused path (kernels.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

// One wave per (segment g, quarter h) of the slot sweep (4 per block, blockIdx.y = h), lanes over
// 64 consecutive samples of the chunk; the wave walks its Ls/4 slots with the same register
// sliding window as the fused kernel (warmed up at its first slot).  Splitting each segment in
// four gives 16 waves per CU for a 16,384-sample chunk (4 with whole segments).  The weights go
// to gemm_f64's tile layout (a 32-sample tile's 32 values of a slot are one 256-B run), for
// every sample of the padded chunk (lanes past sc: the null model's N = 0, finite); slot scalars
// are wave-uniform loads; sum r^2/d and sum log d are left as kWeightParts partials per sample.
template <int NL>
__global__ __launch_bounds__(256) void weights_kernel(WeightsArgs a) {
  constexpr int kWingLds = 4 * ((3 * kWingStride + 3) / 4);
  __shared__ __attribute__((aligned(16))) double tables[NL == 3 ? 3 * kCoreTable + kWingLds + 64 : 1];
  const SpecInfo inf = a.info[a.q];
  if (inf.J == 0) return;  // unusable spectrum: the LDL kernel writes NaN
  const int lane = threadIdx.x & 63;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sl = blockIdx.x * 64 + lane;
  const bool active = sl < a.sc;
  const int64_t s = a.s0 + sl;
  double* core_lds = tables;
  double* wing_lds = tables + 3 * kCoreTable;
  double* exp_lds = wing_lds + kWingLds;
  if constexpr (NL == 3) {
    for (int i = threadIdx.x; i < 3 * kCoreTable; i += 256) core_lds[i] = a.lines.buf[i];
    if (threadIdx.x < 64) exp_lds[threadIdx.x] = a.lines.buf[kLineBufExp2 + threadIdx.x];
    if (threadIdx.x < 3 * kWingStride) wing_lds[threadIdx.x] = a.lines.buf[kLineBufWing + threadIdx.x];
    __syncthreads();
  }
  const int L = inf.L;
  const int Ls = ((L + kChunkSteps - 1) / kChunkSteps) * kChunkSteps;
  const int h = blockIdx.y;                       // quarter of the segment
  const int Lq = Ls / kWeightQuarters;            // Ls is a multiple of kChunkSteps = 4
  const int t0 = h * Lq;
  // null model (s == S) and idle lanes: N = 0, absorption exactly 1 (see kernels.hip)
  const double off = (s < a.S) ? a.offsets[s] : 0.5;
  const double N = (s < a.S) ? a.nhi[s] : 0.0;
  const double zdla = inf.zmin + (inf.zmax - inf.zmin) * off;  // process_qsos.m:163-165
  const double zfac = 1.0 / (1 + zdla);
  double afac[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) afac[j] = a.lines.buf[kLineBufFac + j] * zfac;
  auto raw = [&](double lam) {
    if constexpr (NL == 3) return raw_profile3(lam, afac, N, core_lds, wing_lds, exp_lds);
    else return raw_profile(lam, zfac, N, a.num_lines, a.lines);
  };
  // window at pixel-order position g L + t0: raw profile at padded positions +0..+5 (the tail
  // beyond the spectrum is replicated, so every position is finite)
  const double* lamp = a.lam_pad + (int64_t)g * L + t0;
  double w0 = raw(lamp[0]), w1 = raw(lamp[1]), w2 = raw(lamp[2]);
  double w3 = raw(lamp[3]), w4 = raw(lamp[4]), w5 = raw(lamp[5]);
  double q1 = 0.0, pm = 1.0;
  int pe = 0;
  const int64_t cap16 = gemm_f64_cap16(a.cap);
  const int sloc = sl & 31;
  double* wg_t = a.wg + (int64_t)(sl >> 5) * cap16 * 32 + 8 * (sloc & 3) + (sloc >> 2);
  double* wu_t = a.wu + (wg_t - a.wg);
  // the raw profiles go kWB slots at a time for the 3-line set (raw_profile3_batch: one fix-up branch
  // per batch); a batch past the quarter's last slot evaluates a valid wavelength and drops it
  constexpr int kB = NL == 3 ? kWB : 1;
  for (int t = t0; t < t0 + Lq; t += kB) {
    double lamb[kB], w6v[kB];
#pragma unroll
    for (int b = 0; b < kB; ++b) lamb[b] = t + b < t0 + Lq ? a.srow[((int64_t)g * Ls + t + b) * 8] : lamp[0];
    if constexpr (NL == 3) {
      raw_profile3_batch<kB>(lamb, afac, N, core_lds, wing_lds, exp_lds, w6v);
    } else {
      w6v[0] = raw(lamb[0]);
    }
#pragma unroll
    for (int b = 0; b < kB; ++b) {
      if (t + b >= t0 + Lq) break;
      const int64_t slot = (int64_t)g * Ls + t + b;
      const double* sr = a.srow + slot * 8;
      const double y = sr[1], noise = sr[2], mu = sr[3], om2 = sr[4];
      const double w6 = w6v[b];
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
      q1 = fma(r, rd, q1);
      pm *= d;
      if (((t + b - t0) & 3) == 3) {
        int ex;
        pm = frexp(pm, &ex);
        pe += ex;
      }
      wg_t[slot * 32] = a2 * dinv;
      wu_t[slot * 32] = ab * rd;
    }
  }
  // slots past the 4 segments (capacity slack, and the GEMM's padding to 16) are neutral: weight 0
  if (h == 0) {
    for (int64_t slot = 4 * (int64_t)Ls + g; slot < cap16; slot += 4) {
      wg_t[slot * 32] = 0.0;
      wu_t[slot * 32] = 0.0;
    }
  }
  if (active) {
    a.q1p[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = q1;
    a.ldp[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = log(pm) + pe * kLn2;
  }
}

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Batched augmented LDL^T on the f64 matrix cores: one wave per 4 samples, the 4 samples being the
// 4 independent blocks of v_mfma_f64_4x4x4_4b.  The augmented matrix [[I + Gram, u], [u', r'D^-1 r]]
// of rank k + 1 is padded with identity rows to N = 4 NT and held as its NT (NT + 1) / 2 upper
// 4 x 4 tiles S(L, I), L <= I, one double per lane per tile in the MFMA D layout (lane 16 i + 4 b +
// j holds S(4L + i, 4I + j) of sample b).  Right-looking block elimination, per block column J:
//   * the diagonal tile goes through LDS to the 16 lanes of its sample, each of which factors it
//     (4 x 4 LDL^T, pivots D_p -> log det / r'K^-1 r) and solves for its element of S_JJ^-1;
//   * X_L = S_JJ^-1 S(J, L) for every L > J                         (one MFMA each);
//   * S(L, I) -= X_L' S(J, I) for every J < L <= I                 (one MFMA each: the Schur
//     complement S_LI - S_LJ S_JJ^-1 S_JI, using S_LJ = S_JL').
// Operand maps of 4x4x4_4b (probed, tools/probe_layout.hip): A[i][k] at lane 16k + 4b + i,
// B[k][j] at 16k + 4b + j, D[i][j] at 16i + 4b + j -- so a D-layout register passed as B is the
// tile itself and passed as A is its transpose, which is what both products need.  After the NT
// block steps log det B = sum_{p<k} log D_p and r'K^-1 r = D_k (log_mvnpdf_low_rank.m:24-32).
template <typename GT> __device__ inline const GT* gram_of(const LdlArgs& a);
template <> __device__ inline const double* gram_of<double>(const LdlArgs& a) { return a.G; }
template <> __device__ inline const float* gram_of<float>(const LdlArgs& a) { return a.G32; }

// 1 / D_p for the pivots: v_rcp_f64 and two Newton steps (within an ulp) for the fp64 Gram, one step
// (~2^-50) for the fp32 Gram of the 24-bit path, whose entries carry 2^-24 already
template <typename GT>
__device__ inline double pivot_rcp(double d) {
  if constexpr (std::is_same<GT, float>::value) return rcp_sweep(d);
  else return rcp_nr(d);
}

template <int NT, typename GT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NT <= 13 ? 2 : 1))) void ldl_mfma_kernel(LdlArgs a) {
  constexpr int NTT = NT * (NT + 1) / 2;
  __shared__ __attribute__((aligned(16))) double diag_all[4][2][64];  // double-buffered by J parity
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = (lane >> 2) & 3, ti = lane >> 4, tj = lane & 3;
  const int sl = (blockIdx.x * 4 + wave) * 4 + b;  // this lane's sample within the chunk
  const bool live = sl < a.sc;
  const int K = a.k;
  const int64_t s = a.s0 + sl;
  const SpecInfo inf = a.info[a.q];
  const bool write = live && ti == 0 && tj == 0;
  auto emit = [&](double ll) {
    if (!write) return;
    if (s == a.S) *a.ll_null = ll;
    else if (a.sample_ll) a.sample_ll[a.perm[s]] = ll;
  };
  if (inf.J == 0) {  // no usable pixel: NaN outputs (as the fused path)
    emit(NAN);
    return;
  }
  const int64_t E = (int64_t)K * (K + 1) / 2;
  const int slc = live ? sl : 0;  // idle samples of the last wave compute on sample 0, discarded
  // quad_index layout (internal.h): entry e of this lane's sample at 4 e; the wave's 4 samples x 16
  // tile positions are 64 consecutive values per load
  const GT* Gs = gram_of<GT>(a) + quad_index(slc, 0, E);  // fp64, or fp32 on the 24-bit int8 path
  const double* Us = a.U + quad_index(slc, 0, K);
  // sum r^2/d and sum log d: the sample's 16 lanes load one partial each and add them up
  double q1 = a.q1p[(int64_t)slc * kWeightParts + 4 * ti + tj];
  double logdet_d = a.ldp[(int64_t)slc * kWeightParts + 4 * ti + tj];
#pragma unroll
  for (int m = 1; m <= 32; m <<= 1) {
    if (m == 4 || m == 8) continue;          // lane bits 2-3 are the sample
    q1 += __shfl_xor(q1, m);
    logdet_d += __shfl_xor(logdet_d, m);
  }
  logdet_d += inf.de_shift * kLn2;  // prep's unit scaling (kernels.hip prep_kernel); 0 unless scaled
  // Load the tiles: straight-line code (unconditional loads from valid addresses), all issued up
  // front in row order; a row's values are formed only when its step comes (below), so the
  // factorisation of row J runs while rows > J are still in flight (the compiler's vmcnt waits count
  // only the loads before them).  Since 4 (NT - 1) <= k, only the last tile column (I = NT - 1) holds
  // the u column (c = k), r'D^-1 r (r = c = k) and identity padding (c > k); every other tile is
  // Gram only.  Gram offsets follow gram_tile_index (internal.h): a compile-time tile base plus a
  // per-lane position inside the tile.
  const int di = min(ti, tj), dj = max(ti, tj);            // diagonal tiles: upper-triangle slot
  const int ldiag = di * 4 - di * (di - 1) / 2 + (dj - di), loff = 4 * ti + tj;
  const double done = ti == tj ? 1.0 : 0.0;
  const int w = K - 4 * (NT - 1);                           // Gram columns in the last tile column
  constexpr int base2 = 10 * (NT - 1) + 8 * (NT - 1) * (NT - 2);
  // fp64 Gram: the last tile column's u entries come through the same register (a per-lane address
  // select, so one load per tile); fp32 Gram: u is loaded beside it
  constexpr bool kOneLoad = std::is_same<GT, double>::value;
  GT graw[NTT];   // tile (L, I), L <= I, at L NT - L (L - 1) / 2 + (I - L)
  double uraw[NT];
#pragma unroll
  for (int L = 0; L < NT; ++L) {
#pragma unroll
    for (int I = L; I < NT; ++I) {
      GT g;
      if (I < NT - 1) {
        const int tb = 10 * L + 16 * (L * (NT - 2) - L * (L - 1) / 2) + (I == L ? 0 : 10 + 16 * (I - L - 1));
        g = Gs[4 * (tb + (I == L ? ldiag : loff))];
      } else {
        const GT* gp;
        const double* up;
        if (L < NT - 1) {
          gp = Gs + 4 * (base2 + L * 4 * w + ti * w + min(tj, max(w - 1, 0)));
          up = Us + 4 * (4 * L + ti);
        } else {
          const int cw = max(w, 1), dm = min(di, cw - 1);
          gp = Gs + 4 * (base2 + L * 4 * w + dm * w - dm * (dm - 1) / 2 + (min(dj, cw - 1) - dm));
          up = Us + 4 * min(4 * L + di, K - 1);
        }
        if constexpr (kOneLoad) {
          const bool take_u = L < NT - 1 ? tj == w : (dj == w && di < w);
          g = *(take_u ? reinterpret_cast<const GT*>(up) : gp);
        } else {
          g = *gp;
          uraw[L] = *up;
        }
      }
      graw[L * NT - L * (L - 1) / 2 + (I - L)] = g;
    }
  }
  // the augmented matrix's tile (L, I) from the loaded values: B = I + Gram, then the u column,
  // r'D^-1 r and identity padding in the last tile column
  auto tile_value = [&](int L, int I) -> double {
    GT g = graw[L * NT - L * (L - 1) / 2 + (I - L)];
    asm volatile("" : "+v"(g));        // formed here, at its row's step, not where it was loaded
    if (I < NT - 1) return I == L ? (double)g + done : (double)g;
    double u;
    if constexpr (kOneLoad) {
      u = (double)g;
    } else {
      u = uraw[L];
      asm volatile("" : "+v"(u));
    }
    if (L < NT - 1) return tj < w ? (double)g : (tj == w ? u : 0.0);
    return dj < w ? (double)g + done : (dj == w ? (di < w ? u : q1) : done);
  };
  double T[NTT];
  double inv_p[NT];  // this lane's element of -S_PP^-1 per finished block row P (negated once, not per MFMA)
  double pb = 1.0;  // prod_{p<k} D_p = pb 2^eb
  int eb = 0;
  double quad = 0.0;
  bool bad = false;
  // Left-looking block elimination: row J gets the updates of every finished row P < J, in the order
  // P = 0, 1, ... -- the same MFMAs, operands and accumulation order as the right-looking sweep, so
  // the results are bitwise those of it -- then its diagonal tile is factored.
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    const int jj = J * NT - J * (J - 1) / 2;
#pragma unroll
    for (int I = J; I < NT; ++I) T[jj + (I - J)] = tile_value(J, I);
#pragma unroll
    for (int P = 0; P < J; ++P) {
      const int pp = P * NT - P * (P - 1) / 2;
      const double x = __builtin_amdgcn_mfma_f64_4x4x4f64(inv_p[P], T[pp + (J - P)], 0.0, 0, 0, 0);
#pragma unroll
      for (int I = J; I < NT; ++I) {
        double& t = T[jj + (I - J)];
        t = __builtin_amdgcn_mfma_f64_4x4x4f64(x, T[pp + (I - P)], t, 0, 0, 0);
      }
    }
    // ---- diagonal tile -> LDS -> every lane of the sample
    double* diag = diag_all[wave][J & 1];
    diag[b * 16 + ti * 4 + tj] = T[jj];
    wave_sync();
    const double* dg = diag + b * 16;  // row-major 4 x 4 tile of this lane's sample
    const double2 r00 = *reinterpret_cast<const double2*>(dg + 0), r02 = *reinterpret_cast<const double2*>(dg + 2);
    const double2 r12 = *reinterpret_cast<const double2*>(dg + 6), r22 = *reinterpret_cast<const double2*>(dg + 10);
    const double m[16] = {r00.x, r00.y, r02.x, r02.y, 0, dg[5], r12.x, r12.y, 0, 0, r22.x, r22.y, 0, 0, 0, dg[15]};
    // 4 x 4 LDL^T of the (symmetric) tile from its upper triangle
    double a00 = m[0], a01 = m[1], a02 = m[2], a03 = m[3];
    double a11 = m[5], a12 = m[6], a13 = m[7];
    double a22 = m[10], a23 = m[11], a33 = m[15];
    const double D0 = a00, i0 = pivot_rcp<GT>(D0);
    const double l10 = a01 * i0, l20 = a02 * i0, l30 = a03 * i0;
    a11 = fma(-l10, a01, a11); a12 = fma(-l10, a02, a12); a13 = fma(-l10, a03, a13);
    a22 = fma(-l20, a02, a22); a23 = fma(-l20, a03, a23); a33 = fma(-l30, a03, a33);
    const double D1 = a11, i1 = pivot_rcp<GT>(D1);
    const double l21 = a12 * i1, l31 = a13 * i1;
    a22 = fma(-l21, a12, a22); a23 = fma(-l21, a13, a23); a33 = fma(-l31, a13, a33);
    const double D2 = a22, i2 = pivot_rcp<GT>(D2);
    const double l32 = a23 * i2;
    a33 = fma(-l32, a23, a33);
    const double D3 = a33, i3 = pivot_rcp<GT>(D3);
    const double Dp[4] = {D0, D1, D2, D3};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int p = 4 * J + t;
      if (J < NT - 1 || p < K) {  // every row of a whole tile row is a Gram row (4 (NT - 1) <= k)
        bad |= !(Dp[t] > 0.0) || !(Dp[t] < INFINITY);
        pb *= Dp[t];
      } else if (p == K) {
        quad = Dp[t];
      }
    }
    {
      int ex;
      pb = frexp(pb, &ex);
      eb += ex;
    }
    // this lane's element of S_JJ^-1: column ti (L^-T D^-1 L^-1 e_ti), row tj, so that the register
    // read as an MFMA A operand is S_JJ^-1 itself
    const double e0 = ti == 0 ? 1.0 : 0.0, e1 = ti == 1 ? 1.0 : 0.0, e2 = ti == 2 ? 1.0 : 0.0,
                 e3 = ti == 3 ? 1.0 : 0.0;
    const double y0 = e0, y1 = fma(-l10, y0, e1), y2 = fma(-l21, y1, fma(-l20, y0, e2)),
                 y3 = fma(-l32, y2, fma(-l31, y1, fma(-l30, y0, e3)));
    const double x3 = y3 * i3, x2 = fma(-l32, x3, y2 * i2), x1 = fma(-l31, x3, fma(-l21, x2, y1 * i1)),
                 x0 = fma(-l30, x3, fma(-l20, x2, fma(-l10, x1, y0 * i0)));
    inv_p[J] = -(tj == 0 ? x0 : (tj == 1 ? x1 : (tj == 2 ? x2 : x3)));
  }
  const double logdet_b = log(pb) + eb * kLn2;
  double ll = -0.5 * (quad + (logdet_d + logdet_b) + inf.n * kLog2Pi);  // log_mvnpdf_low_rank.m:30-32
  if (bad || !(fabs(ll) < INFINITY)) {
    ll = NAN;
    if (write) atomicOr(a.status, 1);
  }
  emit(ll);
}

}  // namespace

hipError_t launch_weights(const WeightsArgs& a, hipStream_t s) {
  // every sample of the GEMM's padded 128-sample tiles gets finite weights
  const dim3 grid((unsigned)(gemm_f64_rows(a.sc) / 64), kWeightQuarters);
  if (a.num_lines == 3)
    hipLaunchKernelGGL(weights_kernel<3>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(weights_kernel<0>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ldl_batch(const LdlArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kGemmMaxK) return hipErrorInvalidValue;
  // matrix-core LDL^T: 16 samples per block, NT = ceil((k + 1) / 4) tiles per side
  const dim3 grid((unsigned)((a.sc + 15) / 16)), blk(256);
  switch ((a.k + 1 + 3) / 4) {
#define NT_CASE(n)                                                              \
  case n:                                                                       \
    if (a.G32) hipLaunchKernelGGL((ldl_mfma_kernel<n, float>), grid, blk, 0, s, a);  \
    else hipLaunchKernelGGL((ldl_mfma_kernel<n, double>), grid, blk, 0, s, a);       \
    break;
    NT_CASE(1) NT_CASE(2) NT_CASE(3) NT_CASE(4) NT_CASE(5) NT_CASE(6) NT_CASE(7) NT_CASE(8) NT_CASE(9)
    NT_CASE(10) NT_CASE(11) NT_CASE(12) NT_CASE(13) NT_CASE(14) NT_CASE(15) NT_CASE(16) NT_CASE(17)
#undef NT_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace gpdla
