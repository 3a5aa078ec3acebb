// fp64 Gram / u contraction of the panel-GEMM path (path panel_gemm: any rank 1..kGemmMaxK at the
// reference's own fp64 precision; BASELINE configs[4] shape k = 50), on the f64 matrix cores.
// Replaces, per spectrum and sample chunk (log_mvnpdf_low_rank.m:13-23 for every sample at once):
//   Gram[s][e] = sum_t Wg[t][s] P[t][e]    (P: the Khatri-Rao panel rows M_r M_c, tile-major Gram order)
//   u[s][i]    = sum_t Wu[t][s] M[t][i]
// with Wg = a^2/d, Wu = a r/d from weights_kernel (gemm_path.hip).  K dimension = the spectrum's
// pixel slots; M dimension = samples; N dimension = Gram entries (or the k u entries).
//
// Instruction: v_mfma_f64_4x4x4_4b (72 TF/s on the box against 49 for v_mfma_f64_16x16x4,
// tools/probe_f64b.hip).  Its four 4x4x4 blocks take the SAME A (4 samples x 4 slots) and four
// different B (4 slots x 4 entries each), so one instruction is a 4-sample x 16-entry piece of the
// tile, and a wave's 32 samples x 128 entries are 8 x 8 such pieces: 64 MFMAs per K step of 4 slots
// on 8 A and 8 B registers (0.125 LDS bytes per flop).  Operand maps (probed, tools/probe_layout.hip):
// A[i][k] at lane 16k + 4b + i, B[k][j] at 16k + 4b + j, D[i][j] at 16i + 4b + j.
//
// Block: 4 waves = 128 samples x 128 entries.  B (the panel, shared by the 4 waves) is staged
// through a double-buffered LDS tile, 16 slots per stage, with the entries permuted so a lane reads
// its 8 B operands of a K step as 4 ds_read_b128; A (the weights, private to a wave) comes from
// global memory, one K step ahead, in the tile layout weights_kernel writes: per 32-sample tile,
// [slot][32], sample 4g + i at position 8i + g, so a lane's 8 A operands are 64 contiguous bytes.
// Blocks map to (sample tile, entry tile) in XCD-contiguous runs, entry tile fastest: a sample tile's
// weights are fetched into one XCD's L2 and reused by all its entry tiles.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

constexpr int kFS = kGemmF64TileS;   // samples per block (4 waves x 32)
constexpr int kFE = 128;             // entries per block
constexpr int kFKC = 16;             // slots per LDS stage (4 K steps)
constexpr int kFRow = kFE + 2;       // LDS row stride (doubles): rows of a K step on different banks

__global__ __launch_bounds__(256, 2) void gemm_f64_kernel(GemmF64Args a) {
  __shared__ __attribute__((aligned(16))) double Bs[2][kFKC][kFRow];
  const int n_et = (a.nent + kFE - 1) / kFE;
  const int n_st = (a.sc + kFS - 1) / kFS;
  // XCD-contiguous runs: the dispatcher deals block b to XCD b % 8
  const int per = gridDim.x / 8;
  const int lin = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (lin >= n_st * n_et) return;
  const int st = lin / n_et, et = lin - st * n_et;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kk = lane >> 4, i4 = lane & 3, j16 = lane & 15;
  const int e_base = et * kFE;
  const int64_t cap = a.cap, cap16 = a.cap16;
  const int nchunk = (int)(cap16 / kFKC);

  // A: this wave's 32-sample weight tile; lane (kk, i4) reads slot t0 + kk, positions 8 i4 .. 8 i4 + 7
  const double* Wt = a.W + ((int64_t)(st * 4 + wave) * cap16) * 32 + kk * 32 + i4 * 8;
  auto load_a = [&](int64_t t0, double (&r)[8]) {
    const double2* p = reinterpret_cast<const double2*>(Wt + t0 * 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double2 v = p[q];
      r[2 * q] = v.x;
      r[2 * q + 1] = v.y;
    }
  };
  // B staging: thread -> (slot tid / 16, entries 8 (tid % 16) .. + 7) of the stage
  const int bs_slot = tid >> 4, bs_e = (tid & 15) * 8;
  auto load_b = [&](int c, double (&r)[8]) {
    const int64_t t = (int64_t)c * kFKC + bs_slot;
    const int e = e_base + bs_e;
    const double* src = a.P + t * a.ldp + e;
    if (t < cap && e + 8 <= a.nent) {
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = src[q];
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = (t < cap && e + q < a.nent) ? src[q] : 0.0;
    }
  };
  // entry e_local lives at column 8 (e_local & 15) + (e_local >> 4): a lane's 8 entries j16 + 16 eg
  // are 8 consecutive doubles
  auto store_b = [&](int buf, const double (&r)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int el = bs_e + q;
      Bs[buf][bs_slot][8 * (el & 15) + (el >> 4)] = r[q];
    }
  };

  double acc[8][8];
#pragma unroll
  for (int g = 0; g < 8; ++g)
#pragma unroll
    for (int eg = 0; eg < 8; ++eg) acc[g][eg] = 0.0;

  double bst[8];
  load_b(0, bst);
  store_b(0, bst);
  double A0[8], A1[8];
  load_a(0, A0);
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunk;
    if (more) load_b(c + 1, bst);                  // next stage, in flight during this one's MFMAs
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      double (&Ac)[8] = (ks & 1) ? A1 : A0;
      double (&An)[8] = (ks & 1) ? A0 : A1;
      const int64_t tn = (int64_t)c * kFKC + 4 * (ks + 1);
      if (tn < cap16) load_a(tn, An);              // next K step's weights
      const double2* bp = reinterpret_cast<const double2*>(&Bs[buf][4 * ks + kk][8 * j16]);
      double Bv[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double2 v = bp[q];
        Bv[2 * q] = v.x;
        Bv[2 * q + 1] = v.y;
      }
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int eg = 0; eg < 8; ++eg) acc[g][eg] = __builtin_amdgcn_mfma_f64_4x4x4f64(Ac[g], Bv[eg], acc[g][eg], 0, 0, 0);
    }
    if (more) store_b(buf ^ 1, bst);
    __syncthreads();
  }
  // D: lane 16 i + 4 b + j holds sample 4 g + (lane >> 4), entry 16 eg + (lane & 15); in the
  // quad_index layout a wave's store of (g, eg) is 64 consecutive doubles (every sample of the
  // padded tile is stored; those past sc are never read)
  const int s_wave = st * kFS + wave * 32;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    double* cg = a.C + quad_index(s_wave + 4 * g, 0, a.nent) + kk;
#pragma unroll
    for (int eg = 0; eg < 8; ++eg) {
      const int e = e_base + 16 * eg + j16;
      if (e < a.nent) cg[4 * e] = acc[g][eg];
    }
  }
}

}  // namespace

hipError_t launch_gemm_f64(const GemmF64Args& a, hipStream_t s) {
  if (a.nent < 1 || a.sc < 1 || a.cap16 % kFKC != 0 || a.cap16 < a.cap) return hipErrorInvalidValue;
  const int64_t n_et = (a.nent + kFE - 1) / kFE, n_st = (a.sc + kFS - 1) / kFS;
  const int64_t nb = (n_et * n_st + 7) / 8 * 8;     // a multiple of 8 for the XCD runs
  if (nb > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gemm_f64_kernel, dim3((unsigned)nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace gpdla
