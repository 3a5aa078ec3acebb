// GP null-model training objective on gfx950: spectrum_loss.m (negative log likelihood of one
// centred rest-frame spectrum and its gradient wrt M, log omega, log c_0, log tau_0, log beta)
// summed over the training set as objective.m does.
//
// The per-spectrum work is the same Woodbury core as the hot path (B = I + M'D^-1 M, its
// Cholesky, K^-1 y = D^-1 y - D^-1 M B^-1 M'D^-1 y), plus the gradient terms; the identities
//   K^-1 M = D^-1 M B^-1                       (spectrum_loss.m:55, since C M = I - B^-1)
//   diag K^-1 = d^-1 - d^-2 diag(M B^-1 M')    (spectrum_loss.m:59)
// let one block per spectrum produce every term with k x k work per pixel and no n x n object.
// The dM sum over spectra is never formed per spectrum: with u_i = M_i B^-1 the spectrum's row is
//   dM_i = -(t_i g' - w_i M_i B^-1)      (t = K^-1 y, w = d^-1, g = M'K^-1 y)
// so sum_s dM_i = M_i X_i - h_i with X_i = sum_s w_s,i B_s^-1 and h_i = sum_s t_s,i g_s: one
// pixel x spectrum x (B^-1 entries, g) GEMM on the f64 matrix cores (objective_accum_kernel) and a
// k^2-per-pixel finish (objective_dM_kernel), in place of k P partials written and re-read per
// spectrum (973 MB per evaluation at k = 20, 5,000 spectra).  The remaining per-spectrum partials
// (d log omega, the scalars) are summed in 64 spectrum chunks, then the chunks in order.  Every sum
// has a fixed order: results are deterministic (no atomics).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../../include/gpdla.h"
#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

constexpr int kObjMaxK = 64;
constexpr int kObjMaxPixels = 4096;
constexpr int kObjThreads = 256;
constexpr int kObjScalars = 8;  // per spectrum: nlog_p, dlog_c_0, dlog_tau_0, dlog_beta, n, bad, -, -

struct ObjArgs {
  int32_t P;                 // pixels per spectrum row (the rest grid)
  int32_t k;
  int64_t ld;                // row stride of y / lya_1pz / noise
  const double* y;           // [Q][ld] centred flux, NaN = missing (objective.m:43)
  const double* lya_1pz;     // [Q][ld]
  const double* noise;       // [Q][ld]
  const double* M;           // [P x k] column-major (x(1:P*k), objective.m:22-23)
  const double* MT;          // [4 ceil(P / 4)][KP] the same M pixel-major, zero-padded (objective_mt_kernel)
  const double* omega2;      // [P] spectrum_loss's omega2 argument, or exp(2 log omega) (objective.m:25-32)
  double c_0, tau_0, beta;
  int32_t ldw;               // row stride of part_w / part_t (P rounded up to 32, zero tail)
  int32_t nep, nxp;          // part_bg row length; offset of g in it (see obj_nxp)
  double* part_w;            // [Q][ldw] D^-1 (0 = excluded pixel)
  double* part_t;            // [Q][ldw] K^-1 y (0 = excluded pixel)
  double* part_bg;           // [Q][nep] B^-1's upper triangle (packed rows), then g = M'K^-1 y at nxp
  const double* part_gram;   // [Q][nep] objective_gram_kernel: B - I (packed like part_bg), then v = M'D^-1 y
  double* part_dlo;          // [Q][P]
  double* part_s;            // [Q][kObjScalars]
  double* part_px;           // [Q][4][P] pass 1's pixel terms for pass 6: an, da0, da1, da2 (:62-73)
};

// The 4x4 tiles of pass 6's matrix-core U = M B^-1 (k > 32) for a compile-time rank bound KB
template <int KB>
struct ObjTiles {
  static constexpr int NTr = (KB + 3) / 4;
  static constexpr int NTc = (KB + 4) / 4;
  static constexpr int KP = 4 * NTc;                              // MT row length (doubles)
};

__host__ __device__ constexpr int obj_kb(int k) {
  return k <= 8 ? 8 : k <= 16 ? 16 : k <= 20 ? 20 : k <= 24 ? 24 : k <= 32 ? 32 : 64;
}
// part_bg row: B^-1's k (k + 1) / 2 upper entries, padded to a multiple of 64 (the GEMM's entry tile,
// so no tile mixes the D^-1- and the K^-1 y-weighted segments), then g in a 64-entry tile
__host__ __device__ constexpr int obj_nxp(int k) { return (k * (k + 1) / 2 + 63) / 64 * 64; }
__host__ __device__ constexpr int obj_nep(int k) { return obj_nxp(k) + 64; }
__host__ __device__ constexpr int obj_ldw(int64_t P) { return (int)((P + 31) / 32 * 32); }
// packed index of B^-1[r][c], r <= c
__device__ inline int obj_packed(int r, int c, int k) { return r * k - r * (r - 1) / 2 + (c - r); }
__host__ __device__ constexpr int obj_kp(int kb) { return 4 * ((kb + 4) / 4); }

// omega^2 = exp(2 log omega) per pixel (objective.m:32), once per evaluation rather than per spectrum
__global__ __launch_bounds__(256) void objective_omega2_kernel(const double* __restrict__ log_omega, int32_t P,
                                                               double* __restrict__ om2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < P) om2[i] = exp(2 * log_omega[i]);
}

// MT[p][r] = M[r][p] for p < P, r < k; zero elsewhere (the padding rows / columns the tiles read)
__global__ __launch_bounds__(256) void objective_mt_kernel(const double* __restrict__ M, int32_t P, int32_t k,
                                                           int32_t KP, int64_t rows, double* __restrict__ MT) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * KP) return;
  const int64_t p = e / KP;
  const int r = (int)(e - p * KP);
  MT[e] = (p < P && r < k) ? M[(int64_t)r * P + p] : 0.0;
}

__device__ inline double block_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// pixel scalars of spectrum_loss.m:23-31
struct PixelTerms {
  double om2, sf, tau, absorb, an, d;
};

__device__ inline PixelTerms pixel_terms(const ObjArgs& a, int i, double lya, double nv) {
  PixelTerms p;
  p.om2 = a.omega2[i];                                            // objective.m:32 (objective_omega2_kernel)
  p.tau = a.tau_0 * pow(lya, a.beta);                             // spectrum_loss.m:23
  p.absorb = exp(-p.tau);                                         // :24
  p.sf = 1 - p.absorb + a.c_0;                                    // :27
  p.an = p.om2 * (p.sf * p.sf);                                   // :28
  p.d = nv + p.an;                                                // :30
  return p;
}

// pass 1, one block per spectrum: D^-1 and D^-1 y per pixel (to the GEMM operand rows part_w /
// part_t), sum log d and n (to part_s[4], [6]), and the gradient's pixel terms for pass 6
__global__ __launch_bounds__(kObjThreads) void objective_pixel_kernel(ObjArgs a) {
  __shared__ double red[8];
  const int P = a.P;
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.x;
  const double* y = a.y + q * a.ld;
  const double* lya = a.lya_1pz + q * a.ld;
  const double* nv = a.noise + q * a.ld;
  double* wout = a.part_w + q * (int64_t)a.ldw;
  double* tout = a.part_t + q * (int64_t)a.ldw;
  double logd = 0.0, cnt = 0.0;
  for (int i = tid; i < P; i += kObjThreads) {
    const double yi = y[i];
    const bool valid = !(yi != yi);                               // objective.m:43 ~isnan
    double wi = 0.0, ti = 0.0;
    if (valid) {
      const double lyi = lya[i];
      const PixelTerms p = pixel_terms(a, i, lyi, nv[i]);
      wi = 1.0 / p.d;                                             // :32
      ti = wi * yi;                                               // :33
      logd += log(p.d);                                           // :44
      cnt += 1.0;
      // the gradient's pixel terms (:62-73) for pass 6, which would otherwise pay for the pow / exp /
      // log again
      double* px = a.part_px + q * 4 * (int64_t)P + i;
      const double da1 = p.om2 * p.sf * p.tau * p.absorb;         // :69
      px[0] = p.an;                                                // :62
      px[P] = a.c_0 * p.om2 * p.sf;                               // :65
      px[2 * P] = da1;
      px[3 * P] = da1 * log(lyi) * a.beta;                        // :73
    }
    wout[i] = wi;
    tout[i] = ti;
  }
  logd = block_sum(logd, red);
  cnt = block_sum(cnt, red);
  if (tid == 0) {
    a.part_s[q * kObjScalars + 4] = cnt;
    a.part_s[q * kObjScalars + 6] = logd;
  }
}

// pass 2 for every spectrum at once: [B - I | v][s][e] = sum_i A[s][i] KR[i][e] with KR[i] = the
// Khatri-Rao row (M_ir M_ic, r <= c, packed) then M_i at nxp (objective_kr_kernel), A = D^-1 for the
// B entries and D^-1 y for v (spectrum_loss.m:41-42, :46).  Block = 4 waves on a 32-spectrum x
// 64-entry tile, taking every 4th super-step of 16 pixels, added in wave order.  v_mfma_f64_4x4x4_4b
// with the K index permuted inside a super-step: step q's K index kk is pixel pix0 + 4 kk + q (A and B
// alike), so a lane's A operands for 4 steps are 32 contiguous bytes of an operand row; instruction
// (g, eg) is spectra s0 + 8 i + g x entries e0 + 4 (4 b + j) + eg
struct ObjGramArgs {
  int32_t ldw, nep, nxp, nss;   // nss = ldw / 16 super-steps
  int32_t et0, n_et;            // the entry tiles launched: et0 .. et0 + n_et - 1
  const double* W;
  const double* T;
  const double* KR;             // [ldw][nep]
  double* out;                  // [rows][nep]
};

__global__ __launch_bounds__(256) void objective_gram_kernel(ObjGramArgs a) {
  __shared__ double sred[32 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kk = lane >> 4, i4 = lane & 3, j16 = lane & 15;
  const int st = blockIdx.x / a.n_et, et = a.et0 + (blockIdx.x - st * a.n_et);
  const int64_t s0 = 32 * (int64_t)st;
  const int e0 = 64 * et;
  const double* __restrict__ A = e0 >= a.nxp ? a.T : a.W;
  double acc[8][4];
#pragma unroll
  for (int g = 0; g < 8; ++g)
#pragma unroll
    for (int eg = 0; eg < 4; ++eg) acc[g][eg] = 0.0;
  for (int ss = wave; ss < a.nss; ss += 4) {
    const int pix0 = 16 * ss;
    double av[8][4];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const double2* ap = reinterpret_cast<const double2*>(A + (s0 + 8 * i4 + g) * a.ldw + pix0 + 4 * kk);
      const double2 v0 = ap[0], v1 = ap[1];
      av[g][0] = v0.x;
      av[g][1] = v0.y;
      av[g][2] = v1.x;
      av[g][3] = v1.y;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double2* bp = reinterpret_cast<const double2*>(a.KR + (int64_t)(pix0 + 4 * kk + q) * a.nep + e0 + 4 * j16);
      const double2 b0 = bp[0], b1 = bp[1];
      const double bv[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int eg = 0; eg < 4; ++eg) acc[g][eg] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[g][q], bv[eg], acc[g][eg], 0, 0, 0);
    }
  }
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv)
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int eg = 0; eg < 4; ++eg) {
          double& d = sred[(4 * g + eg) * 64 + lane];
          d = (wv ? d : 0.0) + acc[g][eg];
        }
    __syncthreads();
  }
  double* out = a.out + s0 * a.nep + e0;
  for (int idx = threadIdx.x; idx < 32 * 64; idx += 256) {
    const int sp = idx >> 6, e = idx & 63;
    out[(int64_t)sp * a.nep + e] = sred[(4 * (sp & 7) + (e & 3)) * 64 + 16 * (sp >> 3) + (e >> 2)];
  }
}

// KR[i][e]: M_ir M_ic for packed e = (r, c), r <= c; M_ir at nxp + r; zero elsewhere (pixel rows past P,
// the padding entries)
__global__ __launch_bounds__(256) void objective_kr_kernel(const double* __restrict__ M, int32_t P, int32_t k,
                                                           int32_t nxp, int32_t nep, int64_t rows,
                                                           double* __restrict__ KR) {
  const int64_t el = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (el >= rows * nep) return;
  const int64_t i = el / nep;
  const int e = (int)(el - i * nep);
  double v = 0.0;
  if (i < P) {
    if (e >= nxp) {
      if (e - nxp < k) v = M[(int64_t)(e - nxp) * P + i];
    } else if (e < k * (k + 1) / 2) {
      int r = 0, start = 0;
      while (e >= start + (k - r)) {
        start += k - r;
        ++r;
      }
      const int c = r + (e - start);
      v = M[(int64_t)r * P + i] * M[(int64_t)c * P + i];
    }
  }
  KR[el] = v;
}

// passes 3-6, one block per spectrum.  KB: compile-time bound on k (register arrays, unrolled loops);
// the rank itself is a.k <= KB
template <int KB>
__global__ __launch_bounds__(kObjThreads) __attribute__((amdgpu_waves_per_eu(KB <= 24 ? 3 : 1)))
void objective_spectrum_kernel(ObjArgs a) {
  extern __shared__ double sm[];
  const int P = a.P, k = a.k;
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.x;
  double* w = sm;              // [P] d^-1 (0 = excluded pixel)
  double* t = w + P;           // [P] D^-1 y, then K^-1 y
  double* B = t + P;           // 2 x [k][k + 1]: [B | v], then [B^-1 | C y] (pass 3's two buffers)
  double* s = B + 2 * k * k + 2 * k;   // [k] B^-1 M' D^-1 y (= C y)
  double* red = s + 2 * k;     // [8] block reductions (after s and a spare [k])
  // KB <= 32: B^-1 and C y zero-padded to KB (passes 4 and 6 run unguarded, fully unrolled loops)
  double* Bp = red + 8;        // [KB][KB]
  double* sp = Bp + KB * KB;   // [KB]
  __shared__ int s_bad;
  const double* y = a.y + q * a.ld;
  if (tid == 0) s_bad = 0;

  // pass 1's w, D^-1 y, sum log d, n (objective_pixel_kernel); [B - I | v] (objective_gram_kernel)
  {
    const double* win = a.part_w + q * (int64_t)a.ldw;
    const double* tin = a.part_t + q * (int64_t)a.ldw;
    for (int i = tid; i < P; i += kObjThreads) {
      w[i] = win[i];
      t[i] = tin[i];
    }
    const double* gr = a.part_gram + q * (int64_t)a.nep;
    for (int e = tid; e < k * k; e += kObjThreads) {
      const int r = e / k, c = e - r * k;
      B[r * (k + 1) + c] = gr[r <= c ? obj_packed(r, c, k) : obj_packed(c, r, k)] + (r == c ? 1.0 : 0.0);
    }
    for (int r = tid; r < k; r += kObjThreads) B[r * (k + 1) + k] = gr[a.nxp + r];
  }
  const double cnt = a.part_s[q * kObjScalars + 4], logd = a.part_s[q * kObjScalars + 6];
  using TL = ObjTiles<KB>;
  const int lane = tid & 63, wave = tid >> 6;
  __syncthreads();

  // pass 3: Gauss-Jordan on [B | v] by the whole block (B is symmetric positive definite with
  // eigenvalues >= 1: no pivoting): B^-1 in place, s = B^-1 v = C y in the augmented column (:46-48),
  // log det B = the sum of the pivots' logs (= 2 sum log diag of spectrum_loss.m:43's Cholesky factor,
  // :44); a non-positive pivot flags the spectrum as chol would.  Each pivot reads one buffer and writes
  // the other (one barrier per pivot); a thread's entries (and their row / column) are fixed across
  // pivots, so the divisions are done once
  const int ld = k + 1;
  const double* Bi;
  {
    constexpr int NE = (KB * (KB + 1) + kObjThreads - 1) / kObjThreads;
    const int ne = k * ld;
    int ei[NE], ej[NE];
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * kObjThreads;
      ei[n] = e / ld;
      ej[n] = e - ei[n] * ld;
    }
    double* cur = B;
    double* nxt = B + ne;
    double ldb = 0.0;
    for (int p = 0; p < k; ++p) {
      const double piv = cur[p * ld + p];
      if (tid == 0) {
        if (!(piv > 0.0)) s_bad = 1;
        ldb += log(piv);
      }
      const double inv = 1.0 / piv;
#pragma unroll
      for (int n = 0; n < NE; ++n) {
        const int e = tid + n * kObjThreads;
        if (e < ne) {
          const int i = ei[n], j = ej[n];
          double v;
          if (i == p)
            v = j == p ? inv : cur[e] * inv;
          else if (j == p)
            v = -cur[e] * inv;
          else
            v = fma(-cur[i * ld + p] * inv, cur[p * ld + j], cur[e]);
          nxt[e] = v;
        }
      }
      __syncthreads();
      double* sw = cur;
      cur = nxt;
      nxt = sw;
    }
    if (tid == 0) red[6] = ldb;
    for (int r = tid; r < k; r += kObjThreads) s[r] = cur[r * ld + k];
    if constexpr (KB <= 32) {
      for (int e = tid; e < KB * KB; e += kObjThreads) {
        const int r = e / KB, c = e - r * KB;
        Bp[e] = (r < k && c < k) ? cur[r * ld + c] : 0.0;
      }
      for (int r = tid; r < KB; r += kObjThreads) sp[r] = r < k ? cur[r * ld + k] : 0.0;
    }
    Bi = cur;
  }
  __syncthreads();

  // pass 4: K^-1 y = D^-1 y - D^-1 M (C y) (:48), in place over D^-1 y in part_t (the operand of g's and
  // the dM GEMMs; excluded pixels stay 0); y' K^-1 y
  double* tout = a.part_t + q * (int64_t)a.ldw;
  double yky = 0.0;
  for (int i = tid; i < P; i += kObjThreads) {
    const double wi = w[i];
    if (wi != 0.0) {
      // the row's loads issued together; rows past k repeat row k - 1 (finite) against the zero padding
      double Mi[KB];
#pragma unroll
      for (int r = 0; r < KB; ++r) Mi[r] = a.M[(int64_t)(r < k ? r : k - 1) * P + i];
      double ms = 0.0;
      if constexpr (KB <= 32) {
#pragma unroll
        for (int r = 0; r < KB; ++r) ms = fma(Mi[r] * wi, sp[r], ms);
      } else {
#pragma unroll
        for (int r = 0; r < KB; ++r)
          if (r < k) ms = fma(Mi[r] * wi, s[r], ms);
      }
      const double ti = t[i] - ms;
      t[i] = ti;
      tout[i] = ti;
      yky = fma(y[i], ti, yky);
    }
  }
  yky = block_sum(yky, red);  // (its barriers also publish t)

  // the dM GEMM's operand: this spectrum's B^-1 (upper triangle; g = M'K^-1 y (:55) lands at nxp from
  // objective_gram_kernel's second launch on K^-1 y)
  {
    double* bg = a.part_bg + q * (int64_t)a.nep;
    for (int e = tid; e < k * k; e += kObjThreads) {
      const int r = e / k, c = e - r * k;
      if (r <= c) bg[obj_packed(r, c, k)] = Bi[r * ld + c];
    }
  }

  // pass 6: diag K^-1 = d^-1 - d^-2 diag(M B^-1 M') (:59), d log omega (:62) and the scalar gradient
  // sums (:65-74) per pixel; w and K^-1 y to the GEMM's operand rows.  (The dM row -(t_i g' - w_i M_i B^-1)
  // of :54-55 is summed over spectra by objective_accum_kernel / objective_dM_kernel instead.)  For k > 32
  // u = M_i B^-1 comes from the matrix cores; up to 32, diag(M B^-1 M') on the VALU over B^-1's upper
  // triangle
  double sc0 = 0.0, stau = 0.0, sbeta = 0.0;
  double* dlo = a.part_dlo + q * (int64_t)P;
  if constexpr (KB > 32) {
    // U = M B^-1 with 16 pixels x 4 columns per accumulator: block b of v_mfma_f64_4x4x4_4b takes
    // pixels p16 + 4 b .. + 3 (A[i][kk] = B^-1[4 rc + kk][4 ct + i] at lane 16 kk + 4 b + i, the same for
    // the four blocks; B[kk][j] = M[p16 + 4 b + j][4 rc + kk] at lane 16 kk + 4 b + j), so D[i][j] =
    // U[p16 + 4 b + j][4 ct + i] sits at lane 16 i + 4 b + j
    constexpr int NCT = (KB + 3) / 4;
    const double* px = a.part_px + q * 4 * (int64_t)P;
    const int n16p = (P + 15) / 16;
    const int pj = lane & 15, ci = lane >> 4;
    for (int pt = wave; pt < n16p; pt += 4) {
      const int p16 = 16 * pt;
      const int pp = p16 + pj;
      const int pb = pp < P ? pp : P - 1;
      const double* mrow = a.MT + (int64_t)pb * TL::KP;
      const double wi = pp < P ? w[pp] : 0.0, ti = pp < P ? t[pp] : 0.0;
      double qd = 0.0;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const int c = 4 * ct + ci;
        double acc = 0.0;
#pragma unroll
        for (int rc = 0; rc < TL::NTr; ++rc) {
          const int ar = 4 * rc + (lane >> 4), ac = 4 * ct + (lane & 3);
          const double av = (ar < k && ac < k) ? Bi[ar * ld + ac] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_4x4x4f64(av, mrow[4 * rc + (lane >> 4)], acc, 0, 0, 0);
        }
        if (pp < P && c < k) qd = fma(acc, mrow[c], qd);
      }
      qd += __shfl_xor(qd, 16);
      qd += __shfl_xor(qd, 32);
      if (ci == 0 && pp < P) {
        if (wi == 0.0) {
          dlo[pp] = 0.0;
        } else {
          const double dk = wi - wi * wi * qd;
          dlo[pp] = -(px[pp] * (ti * ti - dk));
          const double da0 = px[P + pp];
          sc0 += -(ti * da0) * ti + dk * da0;
          const double da1 = px[2 * P + pp];
          stau += -(ti * da1) * ti + dk * da1;
          const double da2 = px[3 * P + pp];
          sbeta += -(ti * da2) * ti + dk * da2;
        }
      }
    }

  } else {
    for (int i = tid; i < P; i += kObjThreads) {
      const double wi = w[i];
      const double ti = t[i];
      if (wi == 0.0) {
        dlo[i] = 0.0;
        continue;
      }
      double Mi[KB];
#pragma unroll
      for (int r = 0; r < KB; ++r) Mi[r] = a.M[(int64_t)(r < k ? r : k - 1) * P + i];
      // M_i B^-1 M_i' over the upper triangle: sum_r M_r (B_rr M_r + 2 sum_{c > r} B_rc M_c), over the
      // zero-padded copy (compile-time LDS offsets, no per-entry guards)
      double qd = 0.0;
#pragma unroll
      for (int r = 0; r < KB; ++r) {
        double off = 0.0;
#pragma unroll
        for (int c = r + 1; c < KB; ++c) off = fma(Mi[c], Bp[r * KB + c], off);
        qd = fma(Mi[r], fma(Mi[r], Bp[r * KB + r], 2.0 * off), qd);
      }
      const double dk = wi - wi * wi * qd;                          // diag K^-1 (:59)
      const double* px = a.part_px + q * 4 * (int64_t)P + i;        // pass 1's terms
      dlo[i] = -(px[0] * (ti * ti - dk));                           // :62
      const double da0 = px[P];                                     // :65
      sc0 += -(ti * da0) * ti + dk * da0;                           // :66
      const double da1 = px[2 * P];                                 // :69
      stau += -(ti * da1) * ti + dk * da1;                          // :70
      const double da2 = px[3 * P];                                 // :73
      sbeta += -(ti * da2) * ti + dk * da2;                         // :74
    }
  }
  sc0 = block_sum(sc0, red);
  stau = block_sum(stau, red);
  sbeta = block_sum(sbeta, red);
  if (tid == 0) {
    double* o = a.part_s + q * kObjScalars;
    o[0] = 0.5 * (yky + (logd + red[6]) + cnt * kLog2Pi);        // :52
    o[1] = sc0;
    o[2] = stau;
    o[3] = sbeta;
    o[4] = cnt;
    o[5] = s_bad ? 1.0 : 0.0;
    o[6] = 0.0;   // (objective_pixel_kernel's sum log d)
    o[7] = 0.0;
  }
}

// sum the per-spectrum partials in spectrum order into the running totals (objective.m:46-52).  One
// thread per element walks the spectra in order; kSumDepth partials are loaded before the adds that
// use them, so a thread keeps that many loads in flight instead of one (the adds, and so the result,
// stay in spectrum order)
#ifndef GPDLA_OBJ_SUM_DEPTH
#define GPDLA_OBJ_SUM_DEPTH 64                   // (over all 5,000 spectra: 16: 206 us per sum, 32: 177, 64: 149)
#endif
constexpr int kSumDepth = GPDLA_OBJ_SUM_DEPTH;

constexpr int kSumThreads = 64;   // one wave per block: the few thousand elements spread over every CU

__global__ __launch_bounds__(kSumThreads) void objective_sum_kernel(int64_t nq, int64_t per,
                                                                    const double* __restrict__ part,
                                                                    double* __restrict__ total) {
  const int64_t e = (int64_t)blockIdx.x * kSumThreads + threadIdx.x;
  if (e >= per) return;
  double acc = total[e];
  int64_t q = 0;
  for (; q + kSumDepth <= nq; q += kSumDepth) {
    double v[kSumDepth];
#pragma unroll
    for (int j = 0; j < kSumDepth; ++j) v[j] = part[(q + j) * per + e];
#pragma unroll
    for (int j = 0; j < kSumDepth; ++j) acc += v[j];
  }
  for (; q < nq; ++q) acc += part[q * per + e];
  total[e] = acc;
}

// the same in kSumChunks spectrum chunks: out[c][e] = sum over chunk c (in spectrum order); the chunks
// are then added in order by objective_sum_kernel.  A per-element walk over all spectra is one dependent
// chain per thread (d log omega: 1,217 threads x 5,000 spectra); the chunks put 64 x more in flight
constexpr int kSumChunks = 64;

__global__ __launch_bounds__(kSumThreads) void objective_chunk_sum_kernel(int64_t nq, int64_t per,
                                                                          const double* __restrict__ part,
                                                                          double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kSumThreads + threadIdx.x;
  if (e >= per) return;
  const int64_t c = blockIdx.y;
  const int64_t q0 = nq * c / kSumChunks, q1 = nq * (c + 1) / kSumChunks;
  constexpr int kD = 16;
  double acc = 0.0;
  int64_t q = q0;
  for (; q + kD <= q1; q += kD) {
    double v[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j) v[j] = part[(q + j) * per + e];
#pragma unroll
    for (int j = 0; j < kD; ++j) acc += v[j];
  }
  for (; q < q1; ++q) acc += part[q * per + e];
  out[c * per + e] = acc;
}

// [X | h] partials: part[c][i][e] = sum_{s in chunk c} A[s][i] BG[s][e], A = part_w for the B^-1 entries
// (e < nxp), part_t for g's (e >= nxp).  8 spectrum chunks, chunk c on XCD c (blockIdx % 8: the
// dispatcher's XCD): a chunk's operand rows (3.9 MB at k = 20, 5,000 spectra) stay in one L2.
// Block = 4 waves on one 32-pixel x 64-entry tile, taking every 4th K step of 4 spectra; their sums are
// added in wave order.  v_mfma_f64_4x4x4_4b (A[i][kk] at lane 16 kk + 4 b + i, B[kk][j] at
// 16 kk + 4 b + j, D[i][j] at 16 i + 4 b + j): instruction (g, eg) is pixels p0 + 8 i + g x entries
// e0 + 4 (4 b + j) + eg, so a lane's 8 A operands are 64 contiguous bytes of its operand row and its 4
// B operands 32.
struct ObjAccArgs {
  int32_t ldw, nep, nxp;
  int64_t nq;
  const double* W;
  const double* T;
  const double* BG;
  double* part;   // [8][ldw][nep]
};

__global__ __launch_bounds__(256) void objective_accum_kernel(ObjAccArgs a) {
  __shared__ double sred[32 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kk = lane >> 4, i4 = lane & 3, j16 = lane & 15;
  const int chunk = blockIdx.x & 7, tile = blockIdx.x >> 3;
  const int n_et = a.nep / 64;
  const int pt = tile / n_et, et = tile - pt * n_et;
  const int p0 = 32 * pt, e0 = 64 * et;
  const double* __restrict__ A = e0 >= a.nxp ? a.T : a.W;
  const int64_t s0 = a.nq * chunk / 8, s1 = a.nq * (chunk + 1) / 8;
  const int64_t nks = (s1 - s0 + 3) / 4;
  double acc[8][4];
#pragma unroll
  for (int g = 0; g < 8; ++g)
#pragma unroll
    for (int eg = 0; eg < 4; ++eg) acc[g][eg] = 0.0;
  auto load = [&](int64_t ks, double (&av)[8], double (&bv)[4]) {
    const int64_t s = s0 + 4 * ks + kk;
    if (ks < nks && s < s1) {
      const double2* ap = reinterpret_cast<const double2*>(A + s * a.ldw + p0 + 8 * i4);
      const double2* bp = reinterpret_cast<const double2*>(a.BG + s * a.nep + e0 + 4 * j16);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const double2 v = ap[h];
        av[2 * h] = v.x;
        av[2 * h + 1] = v.y;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double2 v = bp[h];
        bv[2 * h] = v.x;
        bv[2 * h + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int h = 0; h < 8; ++h) av[h] = 0.0;
#pragma unroll
      for (int h = 0; h < 4; ++h) bv[h] = 0.0;
    }
  };
  auto mma = [&](const double (&av)[8], const double (&bv)[4]) {
#pragma unroll
    for (int g = 0; g < 8; ++g)
#pragma unroll
      for (int eg = 0; eg < 4; ++eg) acc[g][eg] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[g], bv[eg], acc[g][eg], 0, 0, 0);
  };
  double A0[8], B0[4], A1[8], B1[4];
  load(wave, A0, B0);
  for (int64_t ks = wave; ks < nks; ks += 8) {
    load(ks + 4, A1, B1);
    mma(A0, B0);
    if (ks + 4 < nks) {
      load(ks + 8, A0, B0);
      mma(A1, B1);
    }
  }
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv)
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int eg = 0; eg < 4; ++eg) {
          double& d = sred[(4 * g + eg) * 64 + lane];
          d = (wv ? d : 0.0) + acc[g][eg];
        }
    __syncthreads();
  }
  // pixel p0 + px (px = 8 i + g), entry e0 + e (e = 4 (4 b + j) + eg): lane 16 i + 4 b + j of (g, eg)
  double* out = a.part + ((int64_t)chunk * a.ldw + p0) * a.nep + e0;
  for (int idx = threadIdx.x; idx < 32 * 64; idx += 256) {
    const int px = idx >> 6, e = idx & 63;
    out[(int64_t)px * a.nep + e] = sred[(4 * (px & 7) + (e & 3)) * 64 + 16 * (px >> 3) + (e >> 2)];
  }
}

// dM_i += M_i X_i - h_i (the chunks' partials added in order), one block per pixel
constexpr int kDMThreads = 128;
constexpr int kObjMaxNep = obj_nxp(kObjMaxK) + 64;

__global__ __launch_bounds__(kDMThreads) void objective_dM_kernel(int32_t P, int32_t k, int32_t ldw, int32_t nep,
                                                                  int32_t nxp, const double* __restrict__ part,
                                                                  const double* __restrict__ M,
                                                                  double* __restrict__ total) {
  __shared__ double xs[kObjMaxNep];
  const int i = blockIdx.x;
  for (int e = threadIdx.x; e < nep; e += kDMThreads) {
    double v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = part[((int64_t)c * ldw + i) * nep + e];
    double x = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) x += v[c];
    xs[e] = x;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += kDMThreads) {
    double u = 0.0;
    for (int r = 0; r < k; ++r)
      u = fma(M[(int64_t)r * P + i], xs[r <= c ? obj_packed(r, c, k) : obj_packed(c, r, k)], u);
    // -(h - M X): -(t g' - w M B^-1) summed over the spectra (spectrum_loss.m:54-55, objective.m:47)
    total[(int64_t)c * P + i] += -(xs[nxp + c] - u);
  }
}

}  // namespace

}  // namespace gpdla

using namespace gpdla;

struct gpdla_objective {
  int device = 0;
  int64_t Q = 0, P = 0;
  int32_t k = 0;
  int64_t batch = 0;
  hipStream_t stream = nullptr;
  double* y = nullptr;
  double* lya = nullptr;
  double* noise = nullptr;
  bool owns_data = true;
  double* x = nullptr;        // [P k + P + 3]
  double* part_w = nullptr;   // [batch][ldw]
  double* part_t = nullptr;   // [batch][ldw]
  double* part_bg = nullptr;  // [rows][nep] (g's tile is written for whole 32-spectrum tiles)
  double* part_gram = nullptr;  // [rows][nep] objective_gram_kernel's [B - I | v]
  double* kr = nullptr;       // [ldw][nep] the Khatri-Rao panel of M
  int64_t rows = 0;           // batch rounded up to the Gram's 32-spectrum tiles
  double* part_acc = nullptr; // [8][ldw][nep] objective_accum_kernel's chunk partials
  double* part_chunk = nullptr;  // [kSumChunks][P + kObjScalars] chunk sums
  double* part_dlo = nullptr;
  double* part_s = nullptr;
  double* part_px = nullptr;  // [batch][4][P]
  double* tot = nullptr;      // [k P + P + kObjScalars]
  double* mt = nullptr;       // [4 ceil(P / 4)][obj_kp(obj_kb(k))] pixel-major M
  double* om2 = nullptr;      // [P] omega^2 of the evaluation's log omega
};

namespace {

int obj_fail(gpdla_objective* o, int rc) {
  gpdla_objective_destroy(o);
  return rc;
}

size_t obj_shared_bytes(int64_t P, int k) {
  const int kb = obj_kb(k);
  return (size_t)(2 * P + 2 * k * k + 4 * k + 8 + (kb <= 32 ? kb * kb + kb : 0)) * sizeof(double);
}

// one pass over all spectra with the M / log omega / (c_0, tau_0, beta) already in place
int obj_run(gpdla_objective* o, const double* dM_src, const double* lo_src, const double* om2_src,
            double c_0, double tau_0, double beta, double* host_tot) {
  const int64_t P = o->P;
  const int k = o->k;
  const int64_t per_dM = (int64_t)k * P;
  HIP_TRY(hipMemsetAsync(o->tot, 0, (per_dM + P + kObjScalars) * sizeof(double), o->stream));
  const size_t shm = obj_shared_bytes(P, k);
  const int KP = obj_kp(obj_kb(k));
  const int64_t mt_rows = 4 * ((P + 3) / 4);
  hipLaunchKernelGGL(objective_mt_kernel, dim3((unsigned)((mt_rows * KP + 255) / 256)), dim3(256), 0, o->stream,
                     dM_src, (int32_t)P, (int32_t)k, (int32_t)KP, mt_rows, o->mt);
  const int ldw = obj_ldw(P), nep = obj_nep(k), nxp = obj_nxp(k);
  hipLaunchKernelGGL(objective_kr_kernel, dim3((unsigned)(((int64_t)ldw * nep + 255) / 256)), dim3(256), 0, o->stream,
                     dM_src, (int32_t)P, (int32_t)k, (int32_t)nxp, (int32_t)nep, (int64_t)ldw, o->kr);
  if (!om2_src)
    hipLaunchKernelGGL(objective_omega2_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, o->stream, lo_src,
                       (int32_t)P, o->om2);
  for (int64_t q0 = 0; q0 < o->Q; q0 += o->batch) {
    const int64_t nq = std::min(o->batch, o->Q - q0);
    ObjArgs a{};
    a.P = (int32_t)P;
    a.k = k;
    a.ld = P;
    a.y = o->y + q0 * P;
    a.lya_1pz = o->lya + q0 * P;
    a.noise = o->noise + q0 * P;
    a.M = dM_src;
    a.MT = o->mt;
    a.omega2 = om2_src ? om2_src : o->om2;
    a.c_0 = c_0;
    a.tau_0 = tau_0;
    a.beta = beta;
    a.ldw = obj_ldw(P);
    a.nep = obj_nep(k);
    a.nxp = obj_nxp(k);
    a.part_w = o->part_w;
    a.part_t = o->part_t;
    a.part_bg = o->part_bg;
    a.part_gram = o->part_gram;
    a.part_dlo = o->part_dlo;
    a.part_s = o->part_s;
    a.part_px = o->part_px;
    const dim3 grid((unsigned)nq), blk(kObjThreads);
    hipLaunchKernelGGL(objective_pixel_kernel, grid, blk, 0, o->stream, a);
    ObjGramArgs gm{};
    gm.ldw = ldw;
    gm.nep = nep;
    gm.nxp = nxp;
    gm.nss = ldw / 16;
    gm.W = o->part_w;
    gm.T = o->part_t;
    gm.KR = o->kr;
    gm.out = o->part_gram;
    gm.et0 = 0;
    gm.n_et = nep / 64;
    hipLaunchKernelGGL(objective_gram_kernel, dim3((unsigned)((nq + 31) / 32 * gm.n_et)), dim3(256), 0, o->stream, gm);
    // dynamic LDS above 64 KiB (long rest grids with high rank) must be opted into per kernel
    auto launch = [&](auto kern) -> int {
      if (shm > 65536)
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
      hipLaunchKernelGGL(kern, grid, blk, shm, o->stream, a);
      HIP_TRY(hipGetLastError());
      return GPDLA_OK;
    };
    int rc = k <= 8 ? launch(objective_spectrum_kernel<8>)
             : k <= 16 ? launch(objective_spectrum_kernel<16>)
             : k <= 20 ? launch(objective_spectrum_kernel<20>)
             : k <= 24 ? launch(objective_spectrum_kernel<24>)
             : k <= 32 ? launch(objective_spectrum_kernel<32>)
                       : launch(objective_spectrum_kernel<64>);
    if (rc) return rc;
    // g = M'K^-1 y for every spectrum (spectrum_loss.m:55): the Gram GEMM's v tile on K^-1 y, into g's
    // tile of part_bg
    gm.out = o->part_bg;
    gm.et0 = nep / 64 - 1;
    gm.n_et = 1;
    hipLaunchKernelGGL(objective_gram_kernel, dim3((unsigned)((nq + 31) / 32)), dim3(256), 0, o->stream, gm);
    // dM: the pixel x spectrum GEMM's chunk partials, then M_i X_i - h_i per pixel
    ObjAccArgs g{};
    g.ldw = a.ldw;
    g.nep = a.nep;
    g.nxp = a.nxp;
    g.nq = nq;
    g.W = o->part_w;
    g.T = o->part_t;
    g.BG = o->part_bg;
    g.part = o->part_acc;
    const int64_t n_tiles = (int64_t)(a.ldw / 32) * (a.nep / 64);
    hipLaunchKernelGGL(objective_accum_kernel, dim3((unsigned)(8 * n_tiles)), dim3(256), 0, o->stream, g);
    hipLaunchKernelGGL(objective_dM_kernel, dim3((unsigned)P), dim3(kDMThreads), 0, o->stream, (int32_t)P, (int32_t)k,
                       a.ldw, a.nep, a.nxp, (const double*)o->part_acc, dM_src, o->tot);
    // d log omega and the scalars: spectrum chunks, then the chunks in order
    double* dlo_chunks = o->part_chunk;
    double* s_chunks = o->part_chunk + kSumChunks * P;
    hipLaunchKernelGGL(objective_chunk_sum_kernel, dim3((unsigned)((P + kSumThreads - 1) / kSumThreads), kSumChunks),
                       dim3(kSumThreads), 0, o->stream, nq, P, (const double*)o->part_dlo, dlo_chunks);
    hipLaunchKernelGGL(objective_chunk_sum_kernel, dim3(1, kSumChunks), dim3(kSumThreads), 0, o->stream, nq,
                       (int64_t)kObjScalars, (const double*)o->part_s, s_chunks);
    hipLaunchKernelGGL(objective_sum_kernel, dim3((unsigned)((P + kSumThreads - 1) / kSumThreads)), dim3(kSumThreads),
                       0, o->stream, (int64_t)kSumChunks, P, (const double*)dlo_chunks, o->tot + per_dM);
    hipLaunchKernelGGL(objective_sum_kernel, dim3(1), dim3(kSumThreads), 0, o->stream, (int64_t)kSumChunks,
                       (int64_t)kObjScalars, (const double*)s_chunks, o->tot + per_dM + P);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpyAsync(host_tot, o->tot, (per_dM + P + kObjScalars) * sizeof(double), hipMemcpyDeviceToHost,
                         o->stream));
  HIP_TRY(hipStreamSynchronize(o->stream));
  return GPDLA_OK;
}

}  // namespace

extern "C" {

void gpdla_objective_destroy(gpdla_objective* o) {
  if (!o) return;
  (void)hipSetDevice(o->device);
  if (o->owns_data) {
    (void)hipFree(o->y);
    (void)hipFree(o->lya);
    (void)hipFree(o->noise);
  }
  (void)hipFree(o->x);
  (void)hipFree(o->part_w);
  (void)hipFree(o->part_t);
  (void)hipFree(o->part_bg);
  (void)hipFree(o->part_gram);
  (void)hipFree(o->kr);
  (void)hipFree(o->part_acc);
  (void)hipFree(o->part_chunk);
  (void)hipFree(o->part_dlo);
  (void)hipFree(o->part_s);
  (void)hipFree(o->part_px);
  (void)hipFree(o->tot);
  (void)hipFree(o->mt);
  (void)hipFree(o->om2);
  if (o->stream) (void)hipStreamDestroy(o->stream);
  delete o;
}

int gpdla_objective_create(int32_t device, int64_t num_quasars, int64_t num_pixels, int32_t k,
                           const double* centered_rest_fluxes, const double* lya_1pzs,
                           const double* rest_noise_variances, int32_t memory, gpdla_objective** out) {
  if (!out) return set_error(GPDLA_EINVAL, "null output handle");
  *out = nullptr;
  if (num_quasars < 0 || num_pixels < 1 || num_pixels > kObjMaxPixels || k < 1 || k > kObjMaxK)
    return set_error(GPDLA_EINVAL, "need 1 <= num_pixels <= %d, 1 <= k <= %d, num_quasars >= 0", kObjMaxPixels,
                     kObjMaxK);
  if (memory != GPDLA_MEM_HOST && memory != GPDLA_MEM_DEVICE) return set_error(GPDLA_EINVAL, "bad memory kind");
  if (num_quasars > 0 && (!centered_rest_fluxes || !lya_1pzs || !rest_noise_variances))
    return set_error(GPDLA_EINVAL, "null data array");
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  auto* o = new gpdla_objective();
  o->device = device;
  o->Q = num_quasars;
  o->P = num_pixels;
  o->k = k;
  // spectra per launch: bounded by the partial-gradient buffers (<= 4 GiB; a DR9-sized training set in one)
  const int64_t per = (int64_t)(k + 1) * num_pixels + kObjScalars;
  const int64_t ldw = obj_ldw(num_pixels), nep = obj_nep(k);
  const int64_t per_q = 2 * ldw + 2 * nep + 5 * num_pixels + kObjScalars;   // w, t, Gram, [B^-1 | g], d log omega, px
  o->batch = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(num_quasars, 1), (1LL << 29) / per_q));
  // GPDLA_OBJECTIVE_BATCH caps the spectra per launch further (smaller workspaces; the tests use it to
  // run the multi-launch path on a small set)
  if (const char* cap = std::getenv("GPDLA_OBJECTIVE_BATCH")) {
    const long long v = std::atoll(cap);
    if (v > 0) o->batch = std::min<int64_t>(o->batch, v);
  }
  o->rows = (o->batch + 31) / 32 * 32;
  if (hipStreamCreateWithFlags(&o->stream, hipStreamNonBlocking) != hipSuccess)
    return obj_fail(o, set_error(GPDLA_EDEVICE, "hipStreamCreate failed"));
  const size_t data = (size_t)std::max<int64_t>(num_quasars, 1) * num_pixels * sizeof(double);
  if (memory == GPDLA_MEM_DEVICE) {
    o->owns_data = false;
    o->y = const_cast<double*>(centered_rest_fluxes);
    o->lya = const_cast<double*>(lya_1pzs);
    o->noise = const_cast<double*>(rest_noise_variances);
  } else {
    if (hipMalloc(&o->y, data) != hipSuccess || hipMalloc(&o->lya, data) != hipSuccess ||
        hipMalloc(&o->noise, data) != hipSuccess)
      return obj_fail(o, set_error(GPDLA_ENOMEM, "objective data allocation failed"));
    const size_t bytes = (size_t)num_quasars * num_pixels * sizeof(double);
    if (bytes && (hipMemcpy(o->y, centered_rest_fluxes, bytes, hipMemcpyHostToDevice) != hipSuccess ||
                  hipMemcpy(o->lya, lya_1pzs, bytes, hipMemcpyHostToDevice) != hipSuccess ||
                  hipMemcpy(o->noise, rest_noise_variances, bytes, hipMemcpyHostToDevice) != hipSuccess))
      return obj_fail(o, set_error(GPDLA_EDEVICE, "objective data upload failed"));
  }
  if (hipMalloc(&o->x, (size_t)((k + 1) * num_pixels + 3) * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_w, (size_t)o->rows * ldw * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_t, (size_t)o->rows * ldw * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_gram, (size_t)o->rows * nep * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->kr, (size_t)ldw * nep * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_bg, (size_t)o->rows * nep * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_acc, (size_t)8 * ldw * nep * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_chunk, (size_t)kSumChunks * (num_pixels + kObjScalars) * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_dlo, (size_t)o->batch * num_pixels * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_s, (size_t)o->batch * kObjScalars * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_px, (size_t)o->batch * 4 * num_pixels * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->tot, (size_t)per * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->mt, (size_t)(4 * ((num_pixels + 3) / 4)) * obj_kp(obj_kb(k)) * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->om2, (size_t)num_pixels * sizeof(double)) != hipSuccess)
    return obj_fail(o, set_error(GPDLA_ENOMEM, "objective workspace allocation failed"));
  // the operand rows' padding (pixels past P, entries past B^-1's triangle and g) is never written: zero
  if (hipMemset(o->part_w, 0, (size_t)o->rows * ldw * sizeof(double)) != hipSuccess ||
      hipMemset(o->part_t, 0, (size_t)o->rows * ldw * sizeof(double)) != hipSuccess ||
      hipMemset(o->part_bg, 0, (size_t)o->rows * nep * sizeof(double)) != hipSuccess)
    return obj_fail(o, set_error(GPDLA_EDEVICE, "objective workspace initialisation failed"));
  *out = o;
  return GPDLA_OK;
}

int gpdla_objective_eval(gpdla_objective* o, const double* x, double* f, double* g) {
  if (!o || !x || !f) return set_error(GPDLA_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(o->device));
  const int64_t P = o->P;
  const int k = o->k;
  const int64_t nx = (int64_t)(k + 1) * P + 3;
  HIP_TRY(hipMemcpyAsync(o->x, x, nx * sizeof(double), hipMemcpyHostToDevice, o->stream));
  // objective.m:28-35
  const double c_0 = std::exp(x[nx - 3]), tau_0 = std::exp(x[nx - 2]), beta = std::exp(x[nx - 1]);
  std::vector<double> tot((size_t)(k + 1) * P + kObjScalars);
  int rc = obj_run(o, o->x, o->x + (int64_t)k * P, nullptr, c_0, tau_0, beta, tot.data());
  if (rc) return rc;
  const double* s = tot.data() + (int64_t)(k + 1) * P;
  *f = s[0];                                                      // objective.m:50 (no prior term)
  if (g) {
    for (int64_t i = 0; i < (int64_t)(k + 1) * P; ++i) g[i] = tot[i];
    // priors on tau_0 and beta enter the gradient only (objective.m:59-71)
    constexpr double tau_0_mu = 0.0023, tau_0_sigma = 0.0007, beta_mu = 3.65, beta_sigma = 0.21;
    g[nx - 3] = s[1];
    g[nx - 2] = s[2] + tau_0 * (tau_0 - tau_0_mu) / (tau_0_sigma * tau_0_sigma);
    g[nx - 1] = s[3] + beta * (beta - beta_mu) / (beta_sigma * beta_sigma);
  }
  if (s[5] > 0) return set_error(GPDLA_ENUMERIC, "non-positive Cholesky pivot in spectrum_loss");
  return GPDLA_OK;
}

int gpdla_spectrum_loss_f64(const double* y, const double* lya_1pz, const double* noise_variance,
                            const double* M, const double* omega2, int64_t n, int32_t k, double c_0,
                            double tau_0, double beta, double* nlog_p, double* dM, double* dlog_omega,
                            double* dlog_c_0, double* dlog_tau_0, double* dlog_beta) {
  if (!y || !lya_1pz || !noise_variance || !M || !omega2 || !nlog_p)
    return set_error(GPDLA_EINVAL, "null argument");
  gpdla_objective* o = nullptr;
  int rc = gpdla_objective_create(0, 1, n, k, y, lya_1pz, noise_variance, GPDLA_MEM_HOST, &o);
  if (rc) return rc;
  double* dbuf = nullptr;
  std::vector<double> tot((size_t)(k + 1) * n + kObjScalars);
  auto run = [&]() -> int {
    HIP_TRY(hipMalloc(&dbuf, (size_t)(k + 1) * n * sizeof(double)));
    HIP_TRY(hipMemcpy(dbuf, M, (size_t)k * n * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dbuf + (int64_t)k * n, omega2, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
    return obj_run(o, dbuf, nullptr, dbuf + (int64_t)k * n, c_0, tau_0, beta, tot.data());
  };
  rc = run();
  if (dbuf) (void)hipFree(dbuf);
  gpdla_objective_destroy(o);
  if (rc) return rc;
  const double* s = tot.data() + (int64_t)(k + 1) * n;
  *nlog_p = s[0];
  if (dM)
    for (int64_t i = 0; i < (int64_t)k * n; ++i) dM[i] = tot[i];
  if (dlog_omega)
    for (int64_t i = 0; i < n; ++i) dlog_omega[i] = tot[(int64_t)k * n + i];
  if (dlog_c_0) *dlog_c_0 = s[1];
  if (dlog_tau_0) *dlog_tau_0 = s[2];
  if (dlog_beta) *dlog_beta = s[3];
  if (s[5] > 0) return set_error(GPDLA_ENUMERIC, "non-positive Cholesky pivot in spectrum_loss");
  return GPDLA_OK;
}

}  // extern "C"
