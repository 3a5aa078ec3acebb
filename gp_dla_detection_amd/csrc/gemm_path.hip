// Panel-GEMM path for any rank k <= kGemmMaxK (BASELINE configs[4]: k = 50): the north star's
// "MFMA for the n x k panel contraction" branch.  Per (spectrum, chunk of samples):
//   weights_kernel    Voigt absorption x pixel terms (process_qsos.m:186-197) ->
//                     Wg[slot][s] = a^2/d, Wu[slot][s] = a r/d, per-segment sum r^2/d, sum log d
//   rocBLAS dgemm x2  Gram[s] = PG^T Wg[:, s] (Khatri-Rao panel, k(k+1)/2 columns) and
//                     u[s] = M^T Wu[:, s]  (engine.hip)  -- log_mvnpdf_low_rank.m:13-23
//   ldl_batch_kernel  augmented LDL^T of [[I + Gram, u], [u', sum r^2/d]] per sample -> logdet and
//                     r'K^-1 r (log_mvnpdf_low_rank.m:24-32), one wave per sample.
// Slot layout, neutral padding rows and sample order are those of the fused path (kernels.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

// One wave per (segment g, quarter h) of the slot sweep (4 per block, blockIdx.y = h), lanes over
// 64 consecutive samples of the chunk; the wave walks its Ls/4 slots with the same register
// sliding window as the fused kernel (warmed up at its first slot).  Splitting each segment in
// four gives 16 waves per CU for a 16,384-sample chunk (4 with whole segments).  Writes are
// coalesced (sample-contiguous rows), slot scalars are wave-uniform loads; sum r^2/d and
// sum log d are left as kWeightParts partials per sample.
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
  const int64_t ldw = a.sc;
  for (int t = t0; t < t0 + Lq; ++t) {
    const int64_t slot = (int64_t)g * Ls + t;
    const double* sr = a.srow + slot * 8;
    const double lam = sr[0], y = sr[1], noise = sr[2], mu = sr[3], om2 = sr[4];
    const double w6 = raw(lam);
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
    if (((t - t0) & 3) == 3) {
      int ex;
      pm = frexp(pm, &ex);
      pe += ex;
    }
    if (active) {
      a.wg[slot * ldw + sl] = a2 * dinv;
      a.wu[slot * ldw + sl] = ab * rd;
    }
  }
  // slots past the 4 segments (capacity slack) are neutral rows of the panel: weight 0
  if (h == 0) {
    for (int64_t slot = 4 * (int64_t)Ls + g; slot < a.cap; slot += 4) {
      if (active) {
        a.wg[slot * ldw + sl] = 0.0;
        a.wu[slot * ldw + sl] = 0.0;
      }
    }
  }
  if (active) {
    a.q1p[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = q1;
    a.ldp[(int64_t)sl * kWeightParts + g * kWeightQuarters + h] = log(pm) + pe * kLn2;
  }
}

// the kWeightParts per-sample partials of sum r^2/d or sum log d, in slot order
__device__ inline double sum_parts(const double* p) {
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < kWeightParts; ++i) acc += p[i];
  return acc;
}

// Augmented LDL^T per sample, one wave per sample (4 per block), matrix packed lower-triangular
// in LDS: A(i, j), j <= i <= k, at i(i+1)/2 + j; row k is [u', sum r^2/d].  Right-looking: at
// pivot p every lane updates a share of the trailing triangle (index table tri: element t ->
// (row offset, column offset)); after the k pivots A(k, k) = r'D^-1 r - u'B^-1 u = r'K^-1 r.
constexpr int kTriMax = kGemmMaxK * (kGemmMaxK + 1) / 2;
constexpr int kPackedMax = (kGemmMaxK + 1) * (kGemmMaxK + 2) / 2;

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void ldl_batch_kernel(LdlArgs a) {
  __shared__ uint32_t tri[kTriMax];
  __shared__ double mats[4][kPackedMax];
  const int K = a.k;
  const int T0 = K * (K + 1) / 2;
  for (int t = threadIdx.x; t < T0; t += 256) {
    int ai = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    while ((ai + 1) * (ai + 2) / 2 <= t) ++ai;
    while (ai * (ai + 1) / 2 > t) --ai;
    tri[t] = ((uint32_t)ai << 16) | (uint32_t)(t - ai * (ai + 1) / 2);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sl = blockIdx.x * 4 + wave;
  if (sl >= a.sc) return;  // wave-uniform; no block barrier below
  const int64_t s = a.s0 + sl;
  const SpecInfo inf = a.info[a.q];
  auto emit = [&](double ll) {
    if (lane != 0) return;
    if (s == a.S) *a.ll_null = ll;
    else if (a.sample_ll) a.sample_ll[a.perm[s]] = ll;
  };
  if (inf.J == 0) {  // no usable pixel: NaN outputs (as the fused path)
    emit(NAN);
    return;
  }
  double* A = mats[wave];
  auto at = [&](int i, int j) -> double& { return A[i * (i + 1) / 2 + j]; };
  const int64_t E = T0;
  const double* Gs = a.G + (int64_t)sl * E;
  int start = 0;
  for (int r = 0; r < K; ++r) {  // Gram (r, c), r <= c, row-major upper -> A(c, r); B = I + Gram
    for (int c = r + lane; c < K; c += 64) at(c, r) = Gs[start + (c - r)] + (c == r ? 1.0 : 0.0);
    start += K - r;
  }
  for (int j = lane; j < K; j += 64) at(K, j) = a.U[(int64_t)sl * K + j];
  const double* q = a.q1p + (int64_t)sl * kWeightParts;
  const double* l4 = a.ldp + (int64_t)sl * kWeightParts;
  if (lane == 0) at(K, K) = sum_parts(q);
  const double logdet_d = sum_parts(l4);
  wave_sync();
  double logdet_b = 0.0;
  bool bad = false;
  for (int p = 0; p < K; ++p) {
    const double d = at(p, p);
    bad |= !(d > 0.0);
    logdet_b += log(d);
    const double invd = 1.0 / d;
    const int R = K - p, T = R * (R + 1) / 2;
    for (int t = lane; t < T; t += 64) {
      const uint32_t ab = tri[t];
      const int i = p + 1 + (int)(ab >> 16), j = p + 1 + (int)(ab & 0xffff);
      at(i, j) = fma(-at(i, p) * invd, at(j, p), at(i, j));
    }
    wave_sync();
  }
  const double quad = at(K, K);
  double ll = -0.5 * (quad + (logdet_d + logdet_b) + inf.n * kLog2Pi);  // log_mvnpdf_low_rank.m:30-32
  if (bad || !(fabs(ll) < INFINITY)) {
    ll = NAN;
    if (lane == 0) atomicOr(a.status, 1);
  }
  emit(ll);
}

// Register form of the same augmented LDL^T (k <= 63): one wave per sample, lane j holds column
// j of [[I + Gram, u], [u', sum r^2/d]] (rows 0..k) in VGPRs.  At pivot p every lane j > p
// updates its column with column p.  Column p is row p by symmetry, and row p is spread over the
// lanes (lane i holds A(p, i) = A(i, p) in col[p]): one ds_write_b64 per pivot publishes it to a
// 64-double LDS line that every lane then reads by broadcast (2 entries per ds_read_b128), so the
// update is ~1.5 instructions per entry with no cross-lane shuffles and no barrier (the wave's
// LDS operations complete in order).  KB bounds k + 1 at compile time (register arrays, unrolled
// pivots); the rank itself is a.k.
__device__ inline double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

template <int KB>
__global__ __launch_bounds__(256) void ldl_reg_kernel(LdlArgs a) {
  constexpr int kStage = (KB - 1) * KB / 2 + KB;  // packed Gram + u of the largest rank in the bucket
  __shared__ __attribute__((aligned(16))) double rowp_all[4][2][64];  // double-buffered by pivot parity
  __shared__ __attribute__((aligned(16))) double stage_all[4][kStage];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* stage = stage_all[wave];
  const int sl = blockIdx.x * 4 + wave;
  if (sl >= a.sc) return;  // wave-uniform
  const int K = a.k;
  const int64_t s = a.s0 + sl;
  const SpecInfo inf = a.info[a.q];
  auto emit = [&](double ll) {
    if (lane != 0) return;
    if (s == a.S) *a.ll_null = ll;
    else if (a.sample_ll) a.sample_ll[a.perm[s]] = ll;
  };
  if (inf.J == 0) {
    emit(NAN);
    return;
  }
  const int64_t E = (int64_t)K * (K + 1) / 2;
  const double* Gs = a.G + (int64_t)sl * E;
  const double* Us = a.U + (int64_t)sl * K;
  const double* q = a.q1p + (int64_t)sl * kWeightParts;
  const double* l4 = a.ldp + (int64_t)sl * kWeightParts;
  const int j = lane;
  // the sample's packed Gram and u, copied coalesced into this wave's LDS slice, then gathered
  // column-wise (the lower half of a column is strided in the packed layout)
  {  // all loads in flight before the first LDS store (one global-memory latency, not ~20)
    constexpr int kIt = (kStage + 63) / 64;
    double tmp[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = it * 64 + lane;
      tmp[it] = t < E ? Gs[t] : (t < E + K ? Us[t - E] : 0.0);
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = it * 64 + lane;
      if (t < E + K) stage[t] = tmp[it];
    }
  }
  __builtin_amdgcn_wave_barrier();
  double col[KB];
#pragma unroll
  for (int i = 0; i < KB; ++i) {
    double v = 0.0;
    if (i <= K && j <= K) {
      if (i < K && j < K) {
        const int r = i < j ? i : j, c = i < j ? j : i;  // Gram (r, c), row-major upper
        v = stage[r * K - r * (r - 1) / 2 + (c - r)] + (i == j ? 1.0 : 0.0);  // B = I + Gram
      } else if (i == K && j == K) {
        v = sum_parts(q);  // sum r^2 / d
      } else {
        v = stage[E + (i == K ? j : i)];  // u in row k / column k
      }
    }
    col[i] = v;
  }
  double pb = 1.0;  // prod D_p = pb 2^eb (frexp-renormalised, one log at the end)
  int eb = 0;
  bool bad = false;
#pragma unroll
  for (int p = 0; p < KB - 1; ++p) {
    if (p < K) {
      // two LDS lines alternate, so pivot p + 1's store cannot overwrite the line pivot p is
      // still reading; the one wave barrier orders this pivot's store before its loads
      double* rowp = rowp_all[wave][p & 1];
      rowp[j] = col[p];                 // row p = column p, lane i -> A(i, p)
      __builtin_amdgcn_wave_barrier();
      const double d = readlane_d(col[p], p);  // the pivot straight from lane p (no LDS round trip)
      bad |= !(d > 0.0);
      pb *= d;
      if ((p & 3) == 3) {
        int ex;
        pb = frexp(pb, &ex);
        eb += ex;
      }
      const double f = (j > p && j <= K) ? col[p] * rcp_nr(d) : 0.0;  // A(j, p) / D_p
      // rows past k hold zeros in every lane and stay zero: no per-row guard
#pragma unroll
      for (int i = p + 1; i < KB; ++i) col[i] = fma(-rowp[i], f, col[i]);  // A(i,j) -= A(i,p) A(j,p) / D_p
    }
  }
  double diag = 0.0;  // A(k, k) of lane k = r'D^-1 r - u'B^-1 u
#pragma unroll
  for (int i = 0; i < KB; ++i)
    if (i == K) diag = col[i];
  const double quad = readlane_d(diag, K);
  const double logdet_d = sum_parts(l4);
  const double logdet_b = log(pb) + eb * kLn2;
  double ll = -0.5 * (quad + (logdet_d + logdet_b) + inf.n * kLog2Pi);  // log_mvnpdf_low_rank.m:30-32
  if (bad || !(fabs(ll) < INFINITY)) {
    ll = NAN;
    if (lane == 0) atomicOr(a.status, 1);
  }
  emit(ll);
}

// 2-D block-cyclic form of the same augmented LDL^T for the larger ranks (k + 1 <= 8 NS, NS =
// ceil((KMAX + 1) / 8)): one wave per sample, lane (ra, cb) = (lane >> 3, lane & 7) holds
// A(ra + 8r, cb + 8c) for the register slots r >= c -- every lower-triangle entry exactly once,
// plus upper entries in the diagonal slots that are never read.  At pivot p the 8 lanes of
// column class p & 7 publish column p (rows > p; rows <= p as zeros) to a 64-double LDS line;
// every lane reads its row and column multipliers from that line (8 distinct addresses per read,
// consecutive doubles: conflict-free) and updates its live slots r >= c >= p / 8.  Slot blocks
// left of the pivot are skipped at compile time, so a lane issues ~Σ_p (NS - p/8)(NS - p/8 + 1)/2
// FMAs (666 at k = 50) where the lane-per-column form issues Σ_p (KB - 1 - p) (1,325), and all 64
// lanes hold live entries until the last column block.
template <int KMAX>
__global__ __launch_bounds__(256) void ldl_cyc_kernel(LdlArgs a) {
  constexpr int NS = (KMAX + 1 + 7) / 8;
  constexpr int N8 = 8 * NS;
  constexpr int kStage = KMAX * (KMAX + 1) / 2 + KMAX;  // packed Gram + u of the largest rank
  __shared__ __attribute__((aligned(16))) double colp_all[4][2][N8];  // double-buffered by pivot parity
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#if !GPDLA_LDL_GATHER
  __shared__ __attribute__((aligned(16))) double stage_all[4][kStage];
  double* stage = stage_all[wave];
#else
  (void)kStage;
#endif
  const int sl = blockIdx.x * 4 + wave;
  if (sl >= a.sc) return;  // wave-uniform
  const int K = a.k;
  const int64_t s = a.s0 + sl;
  const SpecInfo inf = a.info[a.q];
  auto emit = [&](double ll) {
    if (lane != 0) return;
    if (s == a.S) *a.ll_null = ll;
    else if (a.sample_ll) a.sample_ll[a.perm[s]] = ll;
  };
  if (inf.J == 0) {
    emit(NAN);
    return;
  }
  const int64_t E = (int64_t)K * (K + 1) / 2;
  const double* Gs = a.G + (int64_t)sl * E;
  const double* Us = a.U + (int64_t)sl * K;
  const double* q = a.q1p + (int64_t)sl * kWeightParts;
  const double* l4 = a.ldp + (int64_t)sl * kWeightParts;
#if GPDLA_LDL_GATHER
  auto entry = [&](int64_t t) { return t < E ? Gs[t] : Us[t - E]; };
#else
  {  // coalesced copy of the packed Gram and u into this wave's LDS slice (all loads in flight first)
    constexpr int kIt = (kStage + 63) / 64;
    double tmp[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = it * 64 + lane;
      tmp[it] = t < E ? Gs[t] : (t < E + K ? Us[t - E] : 0.0);
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int t = it * 64 + lane;
      if (t < E + K) stage[t] = tmp[it];
    }
  }
  __builtin_amdgcn_wave_barrier();
  auto entry = [&](int64_t t) { return stage[t]; };
#endif
  const int ra = lane >> 3, cb = lane & 7;
  double A[NS][NS];
#pragma unroll
  for (int r = 0; r < NS; ++r) {
#pragma unroll
    for (int c = 0; c <= r; ++c) {
      const int i = ra + 8 * r, j = cb + 8 * c;
      double v = 0.0;
      if (i <= K && j <= K && i >= j) {
        if (i < K) v = entry(j * K - j * (j - 1) / 2 + (i - j)) + (i == j ? 1.0 : 0.0);  // B = I + Gram
        else if (j < K) v = entry(E + j);                                                  // row k: u'
        else v = sum_parts(q);                                                             // sum r^2 / d
      }
      A[r][c] = v;
    }
  }
  double pb = 1.0;  // prod D_p = pb 2^eb (frexp-renormalised, one log at the end)
  int eb = 0;
  bool bad = false;
  // column blocks unrolled (register slots compile-time per block), the 8 pivots of a block not
#pragma unroll
  for (int c0 = 0; c0 < NS; ++c0) {
#pragma unroll 1
    for (int pp = 0; pp < 8; ++pp) {
      const int p = 8 * c0 + pp;
      if (p >= K) break;
      double* colp = colp_all[wave][p & 1];
      if (cb == pp) {  // column p: rows ra + 8r, r >= c0; rows <= p published as zeros
#pragma unroll
        for (int r = c0; r < NS; ++r) colp[ra + 8 * r] = (r > c0 || ra + 8 * r > p) ? A[r][c0] : 0.0;
      }
      __builtin_amdgcn_wave_barrier();
      const double d = readlane_d(A[c0][c0], (pp << 3) | pp);  // A(p, p)
      bad |= !(d > 0.0);
      pb *= d;
      if ((p & 3) == 3) {
        int ex;
        pb = frexp(pb, &ex);
        eb += ex;
      }
      const double invd = rcp_nr(d);
      double R[NS], F[NS];
#pragma unroll
      for (int r = c0; r < NS; ++r) {
        R[r] = colp[ra + 8 * r];          // A(i, p), zero for i <= p
        F[r] = colp[cb + 8 * r] * invd;   // A(j, p) / D_p, zero for j <= p
      }
#pragma unroll
      for (int r = c0; r < NS; ++r) {
#pragma unroll
        for (int c = c0; c <= r; ++c) A[r][c] = fma(-R[r], F[c], A[r][c]);  // A(i,j) -= A(i,p) A(j,p) / D_p
      }
    }
  }
  double diag = 0.0;  // A(k, k) = r'D^-1 r - u'B^-1 u, at lane (k & 7, k & 7), slot (k / 8, k / 8)
#pragma unroll
  for (int r = 0; r < NS; ++r)
    if (r == (K >> 3)) diag = A[r][r];
  const double quad = readlane_d(diag, ((K & 7) << 3) | (K & 7));
  const double logdet_d = sum_parts(l4);
  const double logdet_b = log(pb) + eb * kLn2;
  double ll = -0.5 * (quad + (logdet_d + logdet_b) + inf.n * kLog2Pi);  // log_mvnpdf_low_rank.m:30-32
  if (bad || !(fabs(ll) < INFINITY)) {
    ll = NAN;
    if (lane == 0) atomicOr(a.status, 1);
  }
  emit(ll);
}

}  // namespace

hipError_t launch_weights(const WeightsArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)((a.sc + 63) / 64), kWeightQuarters);
  if (a.num_lines == 3)
    hipLaunchKernelGGL(weights_kernel<3>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(weights_kernel<0>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ldl_batch(const LdlArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kGemmMaxK) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((a.sc + 3) / 4)), blk(256);
#if GPDLA_LDL_CYCLIC
  // 2-D block-cyclic register path for k >= 32 (configs[4]: k = 50)
  if (a.k >= 32 && a.k <= 63) {
    if (a.k <= 39) hipLaunchKernelGGL(ldl_cyc_kernel<39>, grid, blk, 0, s, a);
    else if (a.k <= 47) hipLaunchKernelGGL(ldl_cyc_kernel<47>, grid, blk, 0, s, a);
    else if (a.k <= 51) hipLaunchKernelGGL(ldl_cyc_kernel<51>, grid, blk, 0, s, a);
    else if (a.k <= 55) hipLaunchKernelGGL(ldl_cyc_kernel<55>, grid, blk, 0, s, a);
    else hipLaunchKernelGGL(ldl_cyc_kernel<63>, grid, blk, 0, s, a);
    return hipGetLastError();
  }
#endif
#if GPDLA_LDL_REGISTERS
  // register path: column j of the augmented (k+1) x (k+1) matrix in lane j (k <= 63)
  if (a.k <= 15) hipLaunchKernelGGL(ldl_reg_kernel<16>, grid, blk, 0, s, a);
  else if (a.k <= 31) hipLaunchKernelGGL(ldl_reg_kernel<32>, grid, blk, 0, s, a);
  else if (a.k <= 47) hipLaunchKernelGGL(ldl_reg_kernel<48>, grid, blk, 0, s, a);
  else if (a.k <= 51) hipLaunchKernelGGL(ldl_reg_kernel<52>, grid, blk, 0, s, a);   // configs[4]: k = 50
  else if (a.k <= 63) hipLaunchKernelGGL(ldl_reg_kernel<64>, grid, blk, 0, s, a);
  else
#endif
    hipLaunchKernelGGL(ldl_batch_kernel, grid, blk, 0, s, a);
  return hipGetLastError();
}

}  // namespace gpdla
