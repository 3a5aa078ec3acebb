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
// Block: 4 waves = 128 samples x 128 Gram entries (or 64 u entries); K in stages of 16 slots.  Both operands reach LDS by
// LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, no VGPRs, no VALU), double-buffered:
// the next stage's pieces fly while this one's MFMAs run, and the stage ends with a vmcnt(0) wait and
// one barrier.
//   * B, the panel (shared by the 4 waves): each slot's 128 entries are one contiguous 1 KiB row of
//     the panel (rows 16-B aligned: gemm_ldp pads the row length to even) -> one piece per slot, LDS
//     rows padded by 64 B so the 4 slots of a K step sit on different banks.  MFMA column (eg, lane
//     j16) is entry 8 j16 + eg of the tile, so a lane's 8 B operands are 64 contiguous bytes.
//   * A, the weights (private to a wave): the tile layout weights_kernel writes (per 32-sample tile,
//     [slot][32], sample 4g + i at position 8i + g), so a wave's 16 slots are 4 KiB contiguous = 4
//     pieces, and a lane's 8 A operands of a K step are again 64 contiguous bytes.
// Per K step a lane reads 4 + 4 ds_read_b128 and issues 64 MFMAs; the address arithmetic is
// per-stage scalar work.  Rows past the spectrum's slots read the next rows (finite panel values; a
// zeroed tail past the last spectrum, engine.hip) against exactly-zero weights.
// One launch computes both products (GemmF64Args::seg): a sample tile's entry tiles are the Gram's
// followed by u's, which read Wu and the M panel instead (uniform per block).  Blocks map to (sample
// tile, entry tile) in XCD-contiguous runs, entry tile fastest: a sample tile's weights are fetched
// into one XCD's L2 and reused by all its entry tiles.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

constexpr int kFS = kGemmF64TileS;   // samples per block (4 waves x 32)
constexpr int kFKC = 16;             // slots per stage (4 K steps)
constexpr int kBRow = 128 + 8;       // LDS B row stride (doubles): one 1 KiB piece + 64 B
constexpr int kBStage = kFKC * kBRow;
constexpr int kAStage = kGemmF64Waves * kFKC * 32;
constexpr int kStage = kBStage + kAStage;
// entry tile widths: 16 kEG entries, kEG = 8 for the Gram (128 entries, one whole piece), 4 for u
// (64: k = 50 fills 78 % of it, against 39 % of a 128-entry tile)
constexpr int kEG0 = 8, kEG1 = 4;
__host__ __device__ constexpr int f64_tiles(int nent, int eg) { return (nent + 16 * eg - 1) / (16 * eg); }

template <int kEG>
__device__ __forceinline__ void gemm_f64_tile(const GemmF64Seg& g_, int64_t cap16, int st, int et, double* lds) {
  constexpr int kFE = 16 * kEG;
  const double* __restrict__ gW = g_.W;
  const int64_t ldp = g_.ldp;
  const int nent = g_.nent;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kk = lane >> 4, i4 = lane & 3, j16 = lane & 15;
  const int e_base = et * kFE;
  const int nchunk = (int)(cap16 / kFKC);
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const uint32_t voff = (uint32_t)lane * 16;
  const double* Pt = g_.P + e_base;                                        // + slot * ldp
  const double* Wt = gW + (int64_t)(st * kGemmF64Waves + wave) * cap16 * 32;
  constexpr int kBRowsPerWave = kFKC / kGemmF64Waves;

  // a stage: 16 panel rows (one 1 KiB piece each from the tile's first entry; a 64-entry tile uses
  // the first half) and the wave's 16 x 32 weights (4 pieces)
  auto stage = [&](int c, int buf) {
    const uint32_t sb = lds_base + (uint32_t)(buf * kStage * 8);
#pragma unroll
    for (int r = 0; r < kBRowsPerWave; ++r) {
      const int row = wave * kBRowsPerWave + r;
      dma_piece(Pt + ((int64_t)c * kFKC + row) * ldp, voff, sb + (uint32_t)(row * kBRow * 8));
    }
    const double* wsrc = Wt + (int64_t)c * kFKC * 32;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      dma_piece(wsrc + p * 128, voff, sb + (uint32_t)((kBStage + wave * kFKC * 32 + p * 128) * 8));
  };

  double acc[8][kEG];
#pragma unroll
  for (int g = 0; g < 8; ++g)
#pragma unroll
    for (int eg = 0; eg < kEG; ++eg) acc[g][eg] = 0.0;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunk) stage(c + 1, buf ^ 1);
    const double* Bb = lds + buf * kStage;
    const double* Ab = Bb + kBStage + wave * kFKC * 32;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const double2* ap = reinterpret_cast<const double2*>(Ab + (4 * ks + kk) * 32 + 8 * i4);
      const double2* bp = reinterpret_cast<const double2*>(Bb + (4 * ks + kk) * kBRow + kEG * j16);
      double Av[8], Bv[kEG];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double2 va = ap[q];
        Av[2 * q] = va.x;
        Av[2 * q + 1] = va.y;
      }
#pragma unroll
      for (int q = 0; q < kEG / 2; ++q) {
        const double2 vb = bp[q];
        Bv[2 * q] = vb.x;
        Bv[2 * q + 1] = vb.y;
      }
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int eg = 0; eg < kEG; ++eg) acc[g][eg] = __builtin_amdgcn_mfma_f64_4x4x4f64(Av[g], Bv[eg], acc[g][eg], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of the next stage
    __syncthreads();                                     // ... and everyone's; this buffer is free
  }
  // D: lane 16 i + 4 b + j holds sample 4 g + (lane >> 4) and MFMA column (eg, j16), i.e. entry
  // e_base + kEG j16 + eg, stored in the quad_index layout (every sample of the padded tile; those
  // past sc are never read)
  const int s_wave = st * kFS + wave * 32;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    double* cg = g_.C + quad_index(s_wave + 4 * g, 0, nent) + kk;
#pragma unroll
    for (int eg = 0; eg < kEG; ++eg) {
      const int e = e_base + kEG * j16 + eg;
      if (e < nent) cg[4 * e] = acc[g][eg];
    }
  }
}

__global__ __launch_bounds__(64 * kGemmF64Waves, 8 / kGemmF64Waves) void gemm_f64_kernel(GemmF64Args a) {
  __shared__ __attribute__((aligned(16))) double lds[2 * kStage];
  const int n_et0 = f64_tiles(a.seg[0].nent, kEG0);
  const int n_et = n_et0 + (a.nseg > 1 ? f64_tiles(a.seg[1].nent, kEG1) : 0);
  const int n_st = (a.sc + kFS - 1) / kFS;
  // XCD-contiguous runs: the dispatcher deals block b to XCD b % 8
  const int per = gridDim.x / 8;
  const int lin = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (lin >= n_st * n_et) return;
  const int st = lin / n_et, et = lin - st * n_et;
  if (et < n_et0)
    gemm_f64_tile<kEG0>(a.seg[0], a.cap16, st, et, lds);
  else
    gemm_f64_tile<kEG1>(a.seg[1], a.cap16, st, et - n_et0, lds);
}

}  // namespace

hipError_t launch_gemm_f64(const GemmF64Args& a, hipStream_t s) {
  if (a.nseg < 1 || a.nseg > 2 || a.sc < 1 || a.cap16 % kFKC != 0 || a.cap16 < a.cap) return hipErrorInvalidValue;
  int64_t n_et = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.seg[i].nent < 1) return hipErrorInvalidValue;
    n_et += f64_tiles(a.seg[i].nent, i == 0 ? kEG0 : kEG1);
  }
  const int64_t n_st = (a.sc + kFS - 1) / kFS;
  const int64_t nb = (n_et * n_st + 7) / 8 * 8;     // a multiple of 8 for the XCD runs
  if (nb > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gemm_f64_kernel, dim3((unsigned)nb), dim3(64 * kGemmF64Waves), 0, s, a);
  return hipGetLastError();
}

}  // namespace gpdla
