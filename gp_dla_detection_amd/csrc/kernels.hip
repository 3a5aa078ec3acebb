// HIP kernels for gfx950 (MI355X): spectrum preparation, the fused
// Voigt x low-rank-Gaussian likelihood sweep, and the per-spectrum log-mean-exp.
//
// Reference path (sbird/gp_dla_detection): process_qsos.m:96-212, voigt.c:253-304,
// log_mvnpdf_low_rank.m:5-33.  See DESIGN.md for the data layout and roofline.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "internal.h"

namespace gpdla {

namespace {

// ---------------------------------------------------------------------------------------------
// prep: process_qsos.m:96-177 for one spectrum per block.  Builds the slot panel (interpolated
// model, Khatri-Rao rows, slot scalars), the padded wavelength grid and the spectrum info.
// ---------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a) {
  using Lay = Layout<K>;
  __shared__ int s_i4[4];
  __shared__ double s_d4[4];
  // pass 3 scratch: each wave's interpolated M row of its current slot, and the Gram pair (r, c) of
  // every Khatri-Rao entry (fused layout)
  constexpr int kMaxKK = K > 0 ? K : kGemmMaxK;
  constexpr int kNPairs = K > 0 ? Lay::kNGram : kGemmMaxK * (kGemmMaxK + 1) / 2;
  __shared__ double s_M[4][kMaxKK];
  __shared__ uint16_t s_rc[kNPairs];
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t pb = a.offsets[q];
  const int Lpix = (int)(a.offsets[q + 1] - pb);
  const double z = a.z_qsos[q];
  const double* wl = a.wavelengths + pb;
  const uint8_t* mk = a.mask + pb;

  const int chunk = (Lpix + 255) / 256;
  const int i0 = min(tid * chunk, Lpix), i1 = min(i0 + chunk, Lpix);
  int c_in = 0, c_un = 0;
  double mn_in = INFINITY, mx_in = -INFINITY, mn_un = INFINITY, mx_un = -INFINITY;
  double mn_e = INFINITY, mx_e = -INFINITY;  // binary exponents of the used pixels' noise variances
  for (int i = i0; i < i1; ++i) {
    const double lam = wl[i];
    const double rest = lam / (1 + z);                                  // :102
    const bool inr = (rest >= a.min_lambda) && (rest <= a.max_lambda);  // :104-105
    const bool un = inr && (mk[i] == 0);                                // :111
    c_in += inr;
    c_un += un;
    if (inr) { mn_in = fmin(mn_in, lam); mx_in = fmax(mx_in, lam); }
    if (un) {
      mn_un = fmin(mn_un, lam); mx_un = fmax(mx_un, lam);
      const double nv = a.noise[pb + i];
      if (nv > 0.0 && nv < INFINITY) { const double e = (double)ilogb(nv); mn_e = fmin(mn_e, e); mx_e = fmax(mx_e, e); }
    }
  }
  int m = 0, n = 0;
  int pos_in = block_excl_scan(c_in, s_i4, &m);
  int pos_un = block_excl_scan(c_un, s_i4, &n);
  mn_in = block_reduce_min(mn_in, s_d4);
  mx_in = block_reduce_max(mx_in, s_d4);
  mn_un = block_reduce_min(mn_un, s_d4);
  mx_un = block_reduce_max(mx_un, s_d4);
  mn_e = block_reduce_min(mn_e, s_d4);
  mx_e = block_reduce_max(mx_e, s_d4);
  // Units.  The panel weights kernels keep prod d in a running product renormalised once per 16
  // pixels (the fused sweep renormalises per 4, or per pixel when 4 d's leave the range), so a
  // spectrum whose d = omega^2 a^2 + sigma^2 sit far from 1 (e.g. flux in cgs units, sigma^2 ~ 1e-34)
  // would leave the double range.  Such a spectrum is evaluated in other units: flux, mu and M times
  // 2^(E/2), sigma^2 and omega^2 times 2^E (E even).  d lies in [min sigma^2, max omega^2 + max sigma^2];
  // E centres the binary exponents of that interval (sigma^2 from pass 1, the model's omega^2 bound
  // from the engine) on 0.  Power-of-two scaling is exact: every Gram/u entry, r'D^-1 r and pivot is
  // the same double, and log det D = log det D' - n E ln 2 (SpecInfo::de_shift).  Spectra with all
  // exponents within +-60 are not scaled at all (E = 0), i.e. bitwise the unscaled evaluation.
  int E = 0;
  if (mn_e <= mx_e) {
    const double hi_e = fmax(mx_e, (double)a.om2_hi_e);
    if (mn_e < -60.0 || hi_e > 60.0) E = -2 * (int)rint(0.25 * (mn_e + hi_e));
  }
  const double fy = ldexp(1.0, E / 2), fv = ldexp(1.0, E);

  const int J = (n > 0 && m > 0) ? (a.absorption_mode ? m : n) : 0;
  const int L = (J + 3) / 4;
  const int64_t sb = a.slot_base[q], lb = a.lam_base[q];
  const int64_t cap = a.slot_cap[q];
  double* lam_pad = a.lam_pad + lb;
  int32_t* smap = a.slot_pixel + sb;

  // pass 2: scatter in-range wavelengths and the slot -> pixel map
  for (int i = i0; i < i1; ++i) {
    const double lam = wl[i];
    const double rest = lam / (1 + z);
    const bool inr = (rest >= a.min_lambda) && (rest <= a.max_lambda);
    const bool un = inr && (mk[i] == 0);
    if (inr) {
      lam_pad[3 + pos_in] = lam;                                        // :109,173
      if (a.absorption_mode) smap[pos_in] = un ? i : -1;
      ++pos_in;
    }
    if (un) {
      if (!a.absorption_mode) smap[pos_un] = i;
      ++pos_un;
    }
  }
  // padded ends: [logspace(lo - w s, lo - s, w)'; lambda_m; logspace(hi + s, hi + w s, w)'] (:169-177)
  if (m > 0 && tid < 2 * kWidth) {
    const double sp = a.pixel_spacing;
    const double ws = kWidth * sp;
    if (tid < kWidth) {
      const double lo = log10(mn_in);
      const double d1 = lo - ws, d2 = lo - sp;
      const double v = (tid == kWidth - 1) ? d2 : d1 + tid * ((d2 - d1) / (kWidth - 1));
      lam_pad[tid] = pow(10.0, v);
    } else {
      const int t = tid - kWidth;
      const double hi = log10(mx_in);
      const double d1 = hi + sp, d2 = hi + ws;
      const double v = (t == kWidth - 1) ? d2 : d1 + t * ((d2 - d1) / (kWidth - 1));
      lam_pad[3 + m + t] = pow(10.0, v);
    }
  }
  // replicate the last padded wavelength over the capacity tail (keeps every window finite)
  {
    const double last = m > 0 ? pow(10.0, log10(mx_in) + kWidth * a.pixel_spacing) : 1.0;
    const int64_t first = m > 0 ? (int64_t)m + 2 * kWidth : 0;
    for (int64_t i = first + tid; i < cap + 8; i += 256) lam_pad[i] = last;
  }
  if (tid == 0 && blockIdx.y == 0) {
    SpecInfo inf;
    inf.J = J;
    inf.L = L;
    inf.n = n;
    inf.m = m;
    inf.zmin = n > 0 ? fmax(mn_un / a.lya - 1, (a.lyman_limit * (1 + z)) / a.lya - 1 + a.min_z_cut) : NAN;
    inf.zmax = n > 0 ? (mx_un / a.lya - 1) - a.max_z_cut : NAN;
    inf.slot_base = sb;
    inf.lam_base = lb;
    inf.flags = (J == 0);
    inf.scale_e = E;
    inf.de_shift = -(double)n * E;
    a.info[q] = inf;
  }
  __syncthreads();

  // pass 3: panel rows, one wave per slot, lanes over entries.  gridDim.y blocks share a spectrum's
  // slots (passes 1-2 above are repeated by each of them and write identical values)
  const int lane = tid & 63, wave = tid >> 6;
  const double* rest_g = a.rest;
  const int G = a.num_rest;
  // entry -> (r, c): fused layout e = row-major upper-triangle pair; panel-GEMM layout e =
  // gram_tile_index(r, c, k) (internal.h)
  if constexpr (K > 0) {
    for (int e = tid; e < Lay::kNGram; e += 256) {
      int r, c;
      gram_pair<K>(e, r, c);
      s_rc[e] = (uint16_t)(r | (c << 8));
    }
  } else {
    for (int r = 0; r < a.k; ++r)
      for (int c = r + tid; c < a.k; c += 256) s_rc[gram_tile_index(r, c, a.k)] = (uint16_t)(r | (c << 8));
  }
  __syncthreads();
  // interpolation index (interp_index: the largest gi in [0, G - 2] with rest_g[gi] <= x, else 0) by
  // two rounds of a 64-way search over the lanes -- two dependent loads instead of log2 G
  const int s1 = (G - 1 + 63) / 64;
  auto search = [&](double x) {
    if (s1 > 64) return interp_index(rest_g, G, x);  // grids over 4,097 points: binary search
    const int i1 = lane * s1;
    const bool p1 = i1 < G - 1 && rest_g[i1] <= x;
    int lo = max(0, (int)__builtin_popcountll(__ballot(p1)) - 1) * s1;
    const int i2 = lo + lane;
    const bool p2 = lane < s1 && i2 < G - 1 && rest_g[i2] <= x;
    const int c2 = (int)__builtin_popcountll(__ballot(p2));
    return c2 > 0 ? lo + c2 - 1 : lo;
  };
  // Slot j holds segment gg = j / Ls, step t = j % Ls, i.e. pixel-order position gg L + t; the
  // steps t >= L that round each segment up to whole chunks are neutral rows (like masked pixels).
  const int Ls = L > 0 ? ((L + kChunkSteps - 1) / kChunkSteps) * kChunkSteps : kChunkSteps;
  auto slot_pixel = [&](int64_t j, int& pos) {
    const int gg = (int)(j / Ls), t = (int)(j - (int64_t)gg * Ls);
    pos = (gg < 4 && t < L) ? gg * L + t : -1;
    return (pos >= 0 && pos < J) ? smap[pos] : -1;
  };
  const int KK = K > 0 ? K : a.k;  // K == 0: panel-GEMM layout at runtime rank a.k

  // pass 3a: slot scalars, one thread per slot (the interpolation of mu, log omega and the pow / exp
  // of process_qsos.m:139-147 at full SIMD width; they were one lane's work per slot-wave)
  for (int64_t j = tid + 256 * (int64_t)blockIdx.y; j < cap; j += 256 * (int64_t)gridDim.y) {
    int pos;
    const int pix = slot_pixel(j, pos);
    double sc[6] = {lam_pad[(pos >= 0 ? pos : j) + 2 * kWidth],  // lam (any finite value if neutral),
                    0.0, 1.0, 0.0, 0.0, 0.0};                     // y, noise, mu, om2, valid (neutral)
    if (pix >= 0) {
      const double lam = wl[pix];
      const double rest = lam / (1 + z);
      const int gi = interp_index(rest_g, G, rest);
      const double mu = interp_eval(rest_g, a.mu, G, gi, rest);             // :139
      const double lom = interp_eval(rest_g, a.log_omega, G, gi, rest);     // :142
      const double lya_z = (lam - a.lya) / a.lya;                           // :118-120
      double om2 = exp(2 * lom);                                            // :143
      const double sf = 1 - exp(-a.tau_0 * pow(1 + lya_z, a.beta)) + a.c_0;  // :145
      om2 = om2 * (sf * sf);                                                // :147
      sc[1] = a.flux[pb + pix] * fy;   // unit scaling (pass 1): exact, 1.0 unless E != 0
      sc[2] = a.noise[pb + pix] * fv;
      sc[3] = mu * fy;
      sc[4] = om2 * fv;
      sc[5] = 1.0;
    }
    if constexpr (K > 0) {
      double* row = a.panel + (sb + j) * Lay::kRow;
      row[Lay::kLam] = sc[0];
      row[Lay::kY] = sc[1];
      row[Lay::kNoise] = sc[2];
      row[Lay::kMu] = sc[3];
      row[Lay::kOmega2] = sc[4];
      row[Lay::kValid] = sc[5];
      // the remaining spare words
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int t2 = Lay::kTiles; t2 < Lay::kJS; ++t2)
          if (!(jj < 3 && t2 < Lay::kTiles + 2)) row[jj * Lay::kJS + t2] = 0.0;
    } else {
      double* sr = a.srow + (sb + j) * 8;
#pragma unroll
      for (int w = 0; w < 6; ++w) sr[w] = sc[w];
      // the int8 path's per-slot quantisation scales (gemm_i8.hip weights_i8_kernel), hoisted out
      // of the per-sample loop: u~ scale 2^31 / beta and Gram scale (omega^2 + sigma^2) 2^32
      sr[6] = kI8ScaleU / u_bound(sc[1], sc[3], sc[2]);
      sr[7] = (sc[4] + sc[2]) * kI8ScaleG;
    }
  }

  // pass 3b: Khatri-Rao rows, one wave per slot
  for (int64_t j = wave + 4 * (int64_t)blockIdx.y; j < cap; j += 4 * (int64_t)gridDim.y) {
    int pos;
    const int pix = slot_pixel(j, pos);
    double* sM = s_M[wave];
    if (pix >= 0) {
      const double lam = wl[pix];
      const double rest = lam / (1 + z);
      const int gi = search(rest);
      const bool at_end = rest >= rest_g[G - 1];
      const double* M0 = a.M_rowmajor + (int64_t)gi * KK;
      const double* M1 = a.M_rowmajor + (int64_t)(at_end ? gi : gi + 1) * KK;
      const double x0 = rest_g[gi], x1 = rest_g[at_end ? gi : gi + 1];
      // M row at this pixel, process_qsos.m:140 (griddedInterpolant 'linear', per column), once per
      // column into this wave's LDS row
      for (int col = lane; col < KK; col += 64) {
        double v;
        if (at_end) {
          v = a.M_rowmajor[(int64_t)(G - 1) * KK + col];
        } else {
          const double slope = (M1[col] - M0[col]) / (x1 - x0);
          v = slope * (rest - x0) + M0[col];
        }
        sM[col] = v * fy;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the wave's LDS row before its reads
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto Mi = [&](int col) { return sM[col]; };
    if constexpr (K > 0) {
      double* row = a.panel + (sb + j) * Lay::kRow;
      for (int e = lane; e < 4 * Lay::kTiles; e += 64) {
        double v = 0.0;
        if (pix >= 0) {
          if (e < Lay::kNGram) {
            const int rc = s_rc[e];
            v = Mi(rc & 255) * Mi(rc >> 8);
          } else if (e >= 4 * Lay::kGT && e - 4 * Lay::kGT < K) {
            v = Mi(e - 4 * Lay::kGT);
          }
        }
        row[(e & 3) * Lay::kJS + (e >> 2)] = v;
      }
    } else {
      // panel-GEMM layout: Khatri-Rao row (entry (r, c) at gram_tile_index(r, c), internal.h) and M
      // row (the 8 slot scalars come from pass 3a); all zero for masked and padding slots
      const int64_t E = (int64_t)KK * (KK + 1) / 2;
      double* pg = a.panel ? a.panel + (sb + j) * gemm_ldp(KK) : nullptr;
      double* pm = a.panel_m + (sb + j) * gemm_ldm(KK);
      if (a.panel)  // (the int8 panel paths form these from the M rows in convert_gemm_i8_kernel)
        for (int64_t e = lane; e < E; e += 64) {
          const int rc = s_rc[e];
          pg[e] = pix >= 0 ? Mi(rc & 255) * Mi(rc >> 8) : 0.0;
        }
      for (int c = lane; c < KK; c += 64) pm[c] = pix >= 0 ? Mi(c) : 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads of this slot's row done before
    __builtin_amdgcn_wave_barrier();                         // the next slot overwrites it
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------------------------------------
// likelihood: for one spectrum and 64 samples (4 waves x 16), sweep all slots:
//   per lane (sample s = lane & 15, segment g = lane >> 4): Voigt raw profile at the leading
//   padded wavelength, 7-tap convolution from a register window, DLA-modulated pixel terms
//   a^2/d and a r/d (process_qsos.m:189-197), then v_mfma_f64_4x4x4_4b over the Khatri-Rao
//   tiles (Gram + u).  Panel rows are staged chunk by chunk into a double-buffered LDS ring by
//   global_load_lds (the next chunk's DMA overlaps this chunk's compute).  The epilogue moves each
//   sample's entries to its quad of lanes by DPP rotations and runs the augmented LDL^T there.
// ---------------------------------------------------------------------------------------------
// Stage chunk c (4 steps x 4 segments = 16 rows) into an LDS ring buffer.  Wave w copies the 4
// rows of segment w, which are contiguous in the panel (rows w Ls + 4c .. +3), to LDS rows
// 4 tt + w, each as kPieces 1 KiB global_load_lds_dwordx4 pieces (the last piece over-reads up to
// kRowL - kRow doubles into the next row; the panel has that much slack at its end).  The row base
// is wave-uniform (SGPRs, saddr form), the per-lane byte offsets are fixed VGPRs, so a piece
// costs no VALU.  Issued from inline asm so hipcc does not make the other buffer's ds_reads wait
// on it; the consumer waits with an explicit s_waitcnt vmcnt(0) + barrier at the end of the chunk.
// Hazards inside the string: s_nop 4 for a fresh SGPR base read by a global_* op, s_nop 0 between
// the M0 write and the LDS-DMA that reads it.
template <int K>
__device__ inline void stage_chunk(const double* __restrict__ panel, int Ls, int c, uint32_t buf,
                                   int wave_s, const uint32_t (&voff)[Layout<K>::kPieces]) {
  using Lay = Layout<K>;
#pragma unroll
  for (int tt = 0; tt < kChunkSteps; ++tt) {
    const double* src = panel + ((int64_t)wave_s * Ls + c * kChunkSteps + tt) * Lay::kRow;
    const uint32_t dst = buf + (uint32_t)((tt * 4 + wave_s) * Lay::kRowS * 8);
#pragma unroll
    for (int h = 0; h < Lay::kPieces; ++h) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(dst + h * 1024), "v"(voff[h]), "s"(src) : "memory", "m0");
#pragma clang diagnostic pop
    }
  }
}

template <int K, int NL>
__global__ __launch_bounds__(256, (K <= 20 ? 2 : 1)) void likelihood_kernel(LikelihoodArgs a) {
  using Lay = Layout<K>;
  constexpr int kTiles = Lay::kTiles;
  constexpr int kGT = Lay::kGT;
  constexpr int kRowS = Lay::kRowS;
  constexpr int kJS = Lay::kJS;
  constexpr int kBuf = 4 * kChunkSteps * kRowS;
  static_assert(kWavesPerBlock == 4, "stage_chunk: one wave per segment");
  constexpr int kWingLds = 4 * ((3 * kWingStride + 3) / 4);
  constexpr int kExpLds = 128;
  constexpr int kCoreLds = NL == 3 ? 3 * kCoreTable + kWingLds + kExpLds : 1;
  __shared__ __attribute__((aligned(16))) double lds[2 * kBuf + kCoreLds];
  double* core_lds = lds + 2 * kBuf;
  double* wing_lds = core_lds + 3 * kCoreTable;
  double* exp_lds = wing_lds + kWingLds;

  // XCD-aware block order: the dispatcher deals consecutive blocks round-robin over the 8 XCDs,
  // so block b runs on XCD b % 8.  Virtual index v gives each XCD one contiguous eighth of the
  // (spectrum, sample-block) space: the blocks sharing a spectrum's panel share one XCD's L2.
  const int64_t blocks_x = (a.S + 1 + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const int64_t per_xcd = gridDim.x / 8;  // grid is padded to a multiple of 8
  const int64_t v = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (v >= blocks_x * a.q_count) return;
  const int q = (int)(v / blocks_x);
  const int64_t bx = v - (int64_t)q * blocks_x;
  const SpecInfo inf = a.info[q];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t s_base = bx * kSamplesPerBlock + wave * kSamplesPerWave;
  if (inf.J == 0) {  // unusable spectrum (no unmasked in-range pixel): NaN outputs
    const int64_t su = s_base + (lane >> 2);
    if ((lane & 3) == 0 && su < a.S && a.sample_ll) a.sample_ll[q * a.ld + su] = NAN;
    if ((lane & 3) == 0 && su == a.S) a.ll_null[q] = NAN;
    return;
  }
  const int L = inf.L;
  const int nchunks = (L + kChunkSteps - 1) / kChunkSteps;
  const int Ls = nchunks * kChunkSteps;  // segment stride in the panel; rows L..Ls-1 are neutral
  const double* panel = a.panel + inf.slot_base * Lay::kRow;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  uint32_t voff[Lay::kPieces];
#pragma unroll
  for (int h = 0; h < Lay::kPieces; ++h) voff[h] = (uint32_t)(lane * 16 + h * 1024);

  // prologue: first chunk's DMA, then the core tables (plain loads) while it flies
  stage_chunk<K>(panel, Ls, 0, lds_base, wave_s, voff);
  if constexpr (NL == 3) {
    for (int i = threadIdx.x; i < 3 * kCoreTable; i += 256) core_lds[i] = a.lines.buf[i];
    if (threadIdx.x < 128) exp_lds[threadIdx.x] = a.lines.buf[kLineBufExp128 + threadIdx.x];
    if (threadIdx.x < 3 * kWingStride) wing_lds[threadIdx.x] = a.lines.buf[kLineBufWing + threadIdx.x];
  }

  // ---- per-lane sample constants (MFMA A-operand layout: sample = lane & 15, segment = lane >> 4)
  const int g = lane >> 4;
  const int64_t s = s_base + (lane & 15);
  // The null model (s == S) and the idle lanes past it (s > S, outputs discarded) run with N = 0:
  // every raw profile is then exp(0) = 1 exactly and the 7 taps sum to exactly 1.0 in the order
  // below, i.e. absorption 1 (process_qsos.m:150-152) with no select in the sweep.
  const double off = (s < a.S) ? a.offsets[s] : 0.5;
  const double N = (s < a.S) ? a.nhi[s] : 0.0;
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
  // exp without its clamp (exp_tab128_nc): only a core-zone lane (|x| < kCoreX) can reach v = N tot
  // below -2^31 ln2/128 (tau up to ~6e9 at a line centre); its fix-up clamps tot at -1100 / N.  Outside
  // the core |tot| <= sum_j f_j(kCoreX) (the wings decrease with |x|), so a wave whose N_HI keep
  // N sum_j f_j(kCoreX) <= 1e7 needs no clamp at all; any other wave (N_HI beyond ~1e27) clamps every
  // lane (wave-uniform branch).
  const double core_lim = -1100.0 / N;  // -inf for N = 0
  bool wave_clamp = false;
  if constexpr (NL == 3) {
    double fmax9 = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) fmax9 += fabs(wing_poly(wing_lds + j * kWingStride, 1.0 / (kCoreX * kCoreX)));
    wave_clamp = __builtin_amdgcn_ballot_w64(!(N * fmax9 <= 1e7)) != 0;
  }

  auto raw = [&](double lam, const double* wing) {
    if constexpr (NL == 3) return raw_profile3<kExpLds>(lam, afac, N, core_lds, wing, exp_lds);
    else return raw_profile(lam, zfac, N, a.num_lines, a.lines);
  };
  // sliding window over a ring of 10 registers: at the start of a chunk of phase P the window (raw
  // profiles at the 6 padded positions ahead of the chunk's first pixel) is win[(4 P + i) % 10],
  // i = 0..5, and the chunk's 4 new raw profiles go to win[(4 P + 6 + tt) % 10] (dead values).  The
  // chunk loop is unrolled by 5 (4 * 5 = 0 mod 10), so every index is a compile-time register and
  // the window never moves (one step at a time, each chunk ended in 6 register copies).
  double win[10];
#pragma unroll
  for (int i = 0; i < 6; ++i) win[i] = raw(lw[i], wing_lds);

  double acc[kTiles];
#pragma unroll
  for (int t = 0; t < kTiles; ++t) acc[t] = 0.0;
  double q1 = 0.0;  // sum r^2 / d
  double pm = 1.0;  // prod d = pm * 2^pe
  int pe = 0;

  auto chunk = [&](const int c, auto phase) __attribute__((always_inline)) {
    constexpr int B = (4 * decltype(phase)::value) % 10;
    double* cur = lds + (c & 1) * kBuf;
    if (c + 1 < nchunks)
      stage_chunk<K>(panel, Ls, c + 1, lds_base + (uint32_t)(((c + 1) & 1) * kBuf * 8), wave_s, voff);
    // raw profiles of the chunk's 4 steps first: branch-free outer damping wings (one basic block,
    // so the 4 chains interleave), a rare fix-up for lanes with |x| < kOuterX (the nearest line's
    // inner wing or core, nearest_line), then the 4 table exps
    double rwv[kChunkSteps];
    if constexpr (NL == 3) {
      double tot[kChunkSteps], lamc[kChunkSteps];
      uint32_t cm = 0;
#pragma unroll
      for (int tt = 0; tt < kChunkSteps; ++tt) {
        lamc[tt] = cur[(tt * 4 + g) * kRowS + Lay::kLam];
        tot[tt] = 0.0;
      }
      // T_j = 1/x_j^2 of the 3 lines and 4 steps from ONE reciprocal (batch_rcp4 of the 4 steps'
      // x_0^2 x_1^2 x_2^2; 3 fewer v_rcp_f64 per chunk than one per step).  x_j^2 + 2^-60 equals x_j^2
      // for |x_j| >= 2^-30 and keeps each factor in [2^-60, ~2^37], so the 12-factor product stays a
      // normal double; a lane on a line centre gets a huge but finite T_j that the core fix-up discards.
      double Tj[3][kChunkSteps];
      {
        double a0[kChunkSteps], a1[kChunkSteps], a2[kChunkSteps], p01[kChunkSteps], qq[kChunkSteps], iq[kChunkSteps];
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) {
          const double x0 = fma(lamc[tt], afac[0], -kC2), x1 = fma(lamc[tt], afac[1], -kC2),
                       x2 = fma(lamc[tt], afac[2], -kC2);
          cm |= (((fabs(x0) < kOuterX) | (fabs(x1) < kOuterX) | (fabs(x2) < kOuterX)) ? 1u : 0u) << tt;
          a0[tt] = fma(x0, x0, 0x1p-60); a1[tt] = fma(x1, x1, 0x1p-60); a2[tt] = fma(x2, x2, 0x1p-60);
          p01[tt] = a0[tt] * a1[tt];
          qq[tt] = p01[tt] * a2[tt];
        }
        batch_rcp4(qq, iq);
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) {
          const double r01 = iq[tt] * a2[tt];
          Tj[0][tt] = a1[tt] * r01;
          Tj[1][tt] = a0[tt] * r01;
          Tj[2][tt] = p01[tt] * iq[tt];
        }
      }
      // line-outer order (same per-step summation order): one line's 9 coefficients live at a
      // time, re-read from LDS per line (opaque zero offset) rather than hoisted
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        int zoff;
        asm volatile("s_mov_b32 %0, 0" : "=s"(zoff));
        const double* wl = wing_lds + zoff + j * kWingStride;
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) {
          tot[tt] -= outer_poly(wl, Tj[j][tt]);
        }
      }
      if (cm) {
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) {
          if (cm & (1u << tt)) {
            double ax, T;
            const double* wl;
            int j;
            nearest_line(lamc[tt], afac, Tj[0][tt], Tj[1][tt], Tj[2][tt], wing_lds, ax, T, wl, j);
            if (ax >= kCoreX) {
              // inner wing: the line's outer value swapped for its wing polynomial (both finite and
              // of the same size here, so the swap costs no precision)
              tot[tt] += outer_poly(wl, T) - wing_poly(wl, T);
            } else {
              // core: this line's outer value is meaningless (T_j up to 2^1000), so the sum is
              // rebuilt from the other two lines' outer wings and this line's core polynomial
              const double cf = core_eval(core_lds + j * kCoreTable, ax);
              double t = 0.0;
#pragma unroll
              for (int jj = 0; jj < 3; ++jj) t -= jj == j ? cf : outer_poly(wing_lds + jj * kWingStride, Tj[jj][tt]);
              tot[tt] = fmax(t, core_lim);
            }
          }
        }
      }
      if (wave_clamp) {
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) rwv[tt] = exp_tab128_nc(fmax(N * tot[tt], -1100.0), exp_lds);
      } else {
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) rwv[tt] = exp_tab128_nc(N * tot[tt], exp_lds);
      }
    }
    // the chunk's per-pixel weights first -- 4 independent 7-tap + weight chains the scheduler can
    // interleave (one step at a time they were serial dependent chains of ~16 DP ops in front of each
    // step's MFMAs) -- then the 4 steps' MFMAs
    // The 4 steps' 1/d share one reciprocal too (batch_rcp4_guarded: d = omega^2 a^2 + sigma^2 is
    // not bounded a priori, so a wave whose product leaves [2^-1000, 2^1000] takes 4 reciprocals).
    double wgs[kChunkSteps], wus[kChunkSteps];
    double abs_[kChunkSteps], rs[kChunkSteps], a2s[kChunkSteps], ds[kChunkSteps];
#pragma unroll
    for (int tt = 0; tt < kChunkSteps; ++tt) {
      const double* row = cur + (tt * 4 + g) * kRowS;
      double lam, y, noise, mu, om2;
      if constexpr ((kTiles & 1) == 0) {
        const double2 s0 = *reinterpret_cast<const double2*>(row + Lay::kLam);
        const double2 s1 = *reinterpret_cast<const double2*>(row + Lay::kNoise);
        lam = s0.x; y = s0.y; noise = s1.x; mu = s1.y; om2 = row[Lay::kOmega2];
      } else {
        lam = row[Lay::kLam]; y = row[Lay::kY]; noise = row[Lay::kNoise];
        mu = row[Lay::kMu]; om2 = row[Lay::kOmega2];
      }
      double w6;
      if constexpr (NL == 3) {
        w6 = rwv[tt];
        (void)lam;
      } else {
        w6 = raw(lam, wing_lds);
      }
      // instrumental broadening, voigt.c:297-299 (zero-initialised accumulator, taps in order)
      double ab = win[(B + tt) % 10] * kInstrumentProfile[0];
#pragma unroll
      for (int i = 1; i < 6; ++i) ab = fma(win[(B + tt + i) % 10], kInstrumentProfile[i], ab);
      ab = fma(w6, kInstrumentProfile[6], ab);
      win[(B + tt + 6) % 10] = w6;
      // process_qsos.m:191-197 and log_mvnpdf_low_rank.m:11-15.  Masked / padding rows carry
      // y = mu = om2 = 0, noise = 1 and an all-zero Khatri-Rao row, so they add exactly nothing
      // (r = 0, d = 1, zero B operands) without a per-pixel select.
      const double r = fma(-mu, ab, y);
      const double a2 = ab * ab;
      const double d = fma(om2, a2, noise);
      abs_[tt] = ab; rs[tt] = r; a2s[tt] = a2; ds[tt] = d;
    }
    {
      double dinv[kChunkSteps], P;
      const bool p_ok = batch_rcp4_guarded(ds, dinv, P);
#pragma unroll
      for (int tt = 0; tt < kChunkSteps; ++tt) {
        const double rd = rs[tt] * dinv[tt];
        wgs[tt] = a2s[tt] * dinv[tt];
        wus[tt] = abs_[tt] * rd;
        q1 = fma(rs[tt], rd, q1);
      }
      // prod d: the chunk's product P of the 4 d's when it is in range (pm stays in [2^-1001, 2^1000]
      // until the per-chunk frexp below), otherwise one factor at a time, renormalised after each
      if (p_ok) {
        pm *= P;
      } else {
#pragma unroll
        for (int tt = 0; tt < kChunkSteps; ++tt) {
          int ex;
          pm = frexp(pm * ds[tt], &ex);
          pe += ex;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tt = 0; tt < kChunkSteps; ++tt) {
      const double wg = wgs[tt], wu = wus[tt];
      // B operands: tile t, entry 4t + (lane & 3) of this lane's segment row
      const double* brow = cur + (tt * 4 + g) * kRowS + (lane & 3) * kJS;
#pragma unroll
      for (int tp = 0; tp < kTiles; tp += 2) {
        if (tp + 1 < kTiles) {
          const double2 b = *reinterpret_cast<const double2*>(brow + tp);
          acc[tp] = __builtin_amdgcn_mfma_f64_4x4x4f64(tp < kGT ? wg : wu, b.x, acc[tp], 0, 0, 0);
          acc[tp + 1] = __builtin_amdgcn_mfma_f64_4x4x4f64(tp + 1 < kGT ? wg : wu, b.y, acc[tp + 1], 0, 0, 0);
        } else {
          acc[tp] = __builtin_amdgcn_mfma_f64_4x4x4f64(tp < kGT ? wg : wu, brow[tp], acc[tp], 0, 0, 0);
        }
      }
    }
    // One software pipeline over the chunk's 4 x kTiles MFMAs with the B-operand reads kD ahead
    // (ds_read_b128 = 2 tiles; the default schedule kept 3 in flight and each MFMA pair waited on
    // its read).  kD = 4 / 6 / 8 against the default: -0.2 / -0.3 / -0.0% kernel time (profiles/r5c).
    {
      constexpr int kReads = kChunkSteps * ((kTiles + 1) / 2), kD = 6;
      __builtin_amdgcn_sched_group_barrier(0x100, kD, 0);
#pragma unroll
      for (int i = 0; i < kReads - kD; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * kD, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    {  // keep the running product in range
      int ex;
      pm = frexp(pm, &ex);
      pe += ex;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA for chunk c+1 landed
    __syncthreads();                                   // ... and everyone's; buffer c free again
  };
  using std::integral_constant;
  for (int c = 0; c < nchunks; c += 5) {
    chunk(c, integral_constant<int, 0>{});
    if (c + 1 >= nchunks) break;
    chunk(c + 1, integral_constant<int, 1>{});
    if (c + 2 >= nchunks) break;
    chunk(c + 2, integral_constant<int, 2>{});
    if (c + 3 >= nchunks) break;
    chunk(c + 3, integral_constant<int, 3>{});
    if (c + 4 >= nchunks) break;
    chunk(c + 4, integral_constant<int, 4>{});
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

  // ---- epilogue: the augmented LDL^T per sample in registers, a quad of lanes each, its matrix
  //      moved out of the accumulators by quad rotations (fill_from_acc, device_common.h).
  //      D lane map of 4x4x4_4b: sample 4*((lane>>2)&3) + (lane>>4), entry 4t + (lane&3), so quad
  //      Q = lane >> 2 already holds all entries of sample 4 (Q & 3) + (Q >> 2); its scalars come
  //      from lane (that sample) of the segment-combined sums above.
  const int jq = lane & 3, Q = lane >> 2;
  const int sig = 4 * (Q & 3) + (Q >> 2);
  const double qs = __shfl(q1, sig), dm = __shfl(pm, sig);
  const int de = __shfl(pe, sig);
  constexpr int NJJ = (K + 3) / 4;
  double A[NJJ][4 * NJJ], U[NJJ];
  fill_from_acc<K, 0>(A, U, acc, jq);
  bool bad;
  const double ll = ldl_factor<K>(A, U, qs, dm, (double)de + inf.de_shift, jq, inf.n, bad);
  const int64_t s2 = s_base + sig;
  if (jq == 0 && s2 <= a.S) {
    if (bad) atomicOr(a.status, 1);
    if (s2 == a.S) a.ll_null[q] = ll;
    else if (a.sample_ll) a.sample_ll[q * a.ld + a.perm[s2]] = ll;
  }
}

// ---------------------------------------------------------------------------------------------
// log-mean-exp over samples, process_qsos.m:202-209
// ---------------------------------------------------------------------------------------------
// log-mean-exp per spectrum (process_qsos.m:202-209): one 1,024-thread block per spectrum, each
// thread with kReduceUnroll independent loads in flight per pass (a 256-thread block with one load
// per iteration was load-latency bound: 0.29 ms for 64 spectra x 10^5 samples, profiles/r9z)
constexpr int kReduceThreads = 1024, kReduceUnroll = 4;

template <bool kMax>
__device__ inline double block_reduce_1024(double v, double* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_xor(v, off);
    v = kMax ? fmax(v, o) : v + o;
  }
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double r = lds[0];
#pragma unroll
  for (int w = 1; w < kReduceThreads / 64; ++w) r = kMax ? fmax(r, lds[w]) : r + lds[w];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kReduceThreads) void reduce_kernel(ReduceArgs a) {
  __shared__ double s_w[kReduceThreads / 64];
  const int q = blockIdx.x;
  const double* ll = a.sample_ll + q * a.ld;
  const int64_t S = a.S;
  constexpr int kStride = kReduceThreads * kReduceUnroll;
  double mx = -INFINITY;
  bool nan = false;
  int64_t s = threadIdx.x;
  for (; s + (kReduceUnroll - 1) * kReduceThreads < S; s += kStride) {
    double v[kReduceUnroll];
#pragma unroll
    for (int u = 0; u < kReduceUnroll; ++u) v[u] = ll[s + u * kReduceThreads];
#pragma unroll
    for (int u = 0; u < kReduceUnroll; ++u) {
      nan |= (v[u] != v[u]);
      mx = fmax(mx, v[u]);
    }
  }
  for (int64_t t = s; t < S; t += kReduceThreads) {
    const double v = ll[t];
    nan |= (v != v);
    mx = fmax(mx, v);
  }
  mx = block_reduce_1024<true>(mx, s_w);
  double sum = 0.0;
  s = threadIdx.x;
  for (; s + (kReduceUnroll - 1) * kReduceThreads < S; s += kStride) {
    double v[kReduceUnroll];
#pragma unroll
    for (int u = 0; u < kReduceUnroll; ++u) v[u] = ll[s + u * kReduceThreads];
#pragma unroll
    for (int u = 0; u < kReduceUnroll; ++u) sum += exp(v[u] - mx);
  }
  for (int64_t t = s; t < S; t += kReduceThreads) sum += exp(ll[t] - mx);
  sum = block_reduce_1024<false>(sum, s_w);
  const double anynan = block_reduce_1024<true>(nan ? 1.0 : 0.0, s_w);
  if (threadIdx.x == 0) {
    const SpecInfo inf = a.info[q];
    double r = mx + log(sum / (double)a.S);
    if (anynan > 0 || inf.J == 0) r = NAN;
    a.ll_dla[q] = r;
    if (a.zmin) a.zmin[q] = inf.zmin;
    if (a.zmax) a.zmax[q] = inf.zmax;
    if (a.num_pixels) a.num_pixels[q] = inf.n;
  }
}

// ---------------------------------------------------------------------------------------------
// standalone voigt (MEX replacement): one block per (z, N); raw profile staged in LDS
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void voigt_batch_kernel(const double* __restrict__ lambdas,
                                                          int64_t n_padded,
                                                          const double* __restrict__ zs,
                                                          const double* __restrict__ Ns,
                                                          int32_t num_lines, LineArgs lines,
                                                          double* __restrict__ out) {
  __shared__ double raw[256 + 2 * kWidth];
  const int64_t sidx = blockIdx.x;
  const double zfac = 1.0 / (1 + zs[sidx]);
  const double N = Ns[sidx];
  const int64_t n_out = n_padded - 2 * kWidth;
  double* o = out + sidx * n_out;
  for (int64_t base = 0; base < n_out; base += 256) {
    __syncthreads();
    for (int i = threadIdx.x; i < 256 + 2 * kWidth; i += 256) {
      const int64_t p = base + i;
      raw[i] = (p < n_padded) ? raw_profile(lambdas[p], zfac, N, num_lines, lines) : 0.0;
    }
    __syncthreads();
    const int64_t i = base + threadIdx.x;
    if (i < n_out) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k <= 2 * kWidth; ++k) acc += raw[threadIdx.x + k] * kInstrumentProfile[k];
      o[i] = acc;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// standalone log_mvnpdf_low_rank (the MEX drop-in; the engine fuses this into its sweeps): one
// block of 1,024 threads.
//   * Gram and u: the pixels go through LDS in chunks of 64 rows of M, staged column by column
//     (coalesced reads of the column-major n x k M) as M and D^-1 M, the next chunk's values
//     already in registers while this one is summed.  Thread t owns Gram / u entries t % 256,
//     t % 256 + 256, ... and sums them over the chunk's pixels p = t / 256 (mod 4); the four
//     partial sums of an entry are added at the end (log_mvnpdf_low_rank.m:13-23).
//   * The augmented (k+1) x (k+1) matrix [[I + Gram, u], [u', r'D^-1 r]] is factored R'R in LDS,
//     right-looking, every step's trailing update spread over the block: its last column is
//     t = R^-T u and its last pivot before the square root is r'D^-1 r - t't, so log det B =
//     2 sum_p log R_pp and the quadratic form come out of the same elimination
//     (log_mvnpdf_low_rank.m:24-32).
// ---------------------------------------------------------------------------------------------
constexpr int kMvnMaxK = 64;
constexpr int kMvnChunk = 64;
constexpr int kMvnThreads = 1024;
constexpr int kMvnPhases = kMvnThreads / 256;
constexpr int kMvnSlots = (kMvnMaxK * (kMvnMaxK + 1) / 2 + kMvnMaxK + 255) / 256;  // entries per thread
constexpr int kMvnMPer = (kMvnChunk * kMvnMaxK + kMvnThreads - 1) / kMvnThreads;   // M values per thread
__global__ __launch_bounds__(kMvnThreads) void mvn_single_kernel(const double* __restrict__ y,
                                                                 const double* __restrict__ mu,
                                                                 const double* __restrict__ M,
                                                                 const double* __restrict__ d, int64_t n,
                                                                 int32_t k, double* out, int32_t* status) {
  constexpr int kMs = kMvnChunk * (kMvnMaxK + 1), kMw = kMvnChunk * (kMvnMaxK + 2);
  __shared__ double sm[kMs + kMw];                   // chunk rows of M and of D^-1 M; column k of
  __shared__ double A[kMvnMaxK + 1][kMvnMaxK + 2];   // the latter r/d, column k+1 1/d
  __shared__ double s_d4[16];
  double (*Ms)[kMvnMaxK + 1] = reinterpret_cast<double (*)[kMvnMaxK + 1]>(sm);
  double (*Mw)[kMvnMaxK + 2] = reinterpret_cast<double (*)[kMvnMaxK + 2]>(sm + kMs);
  const int tid = threadIdx.x, et = tid & 255, phase = tid >> 8;
  const int nent = k * (k + 1) / 2, ntot = nent + k;
  int er[kMvnSlots], ec[kMvnSlots];                 // entry et + 256 j -> (row, column); column k = u
#pragma unroll
  for (int j = 0; j < kMvnSlots; ++j) {
    const int e = et + 256 * j;
    if (e < nent) {
      int r = 0, start = 0;
      while (e >= start + (k - r)) { start += k - r; ++r; }
      er[j] = r; ec[j] = r + (e - start);
    } else {
      er[j] = e - nent; ec[j] = k;
    }
  }
  double acc[kMvnSlots];
#pragma unroll
  for (int j = 0; j < kMvnSlots; ++j) acc[j] = 0.0;
  double q1 = 0.0, ld = 0.0;
  // registers holding a chunk in flight: M values idx = tid + 1024 i (column idx / 64, row idx % 64)
  // and, for the first 64 threads, the pixel's y - mu and d
  double mreg[kMvnMPer], rreg = 0.0, dreg = 1.0;
  auto fetch = [&](int64_t p0) {
    const int np = (int)min<int64_t>(kMvnChunk, n - p0);
#pragma unroll
    for (int i = 0; i < kMvnMPer; ++i) {
      const int idx = tid + kMvnThreads * i, c = idx / kMvnChunk, pr = idx % kMvnChunk;
      mreg[i] = (c < k && pr < np) ? M[(p0 + pr) + (int64_t)c * n] : 0.0;
    }
    if (tid < kMvnChunk && tid < np) {
      rreg = y[p0 + tid] - mu[p0 + tid];
      dreg = d[p0 + tid];
    }
  };
  if (n > 0) fetch(0);
  for (int64_t p0 = 0; p0 < n; p0 += kMvnChunk) {
    const int np = (int)min<int64_t>(kMvnChunk, n - p0);
    __syncthreads();                                   // the previous chunk's sums are done
    if (tid < kMvnChunk) {
      double wi = 0.0, rwi = 0.0;
      if (tid < np) {
        wi = 1.0 / dreg;
        rwi = rreg * wi;
        q1 += rreg * rwi;
        ld += log(dreg);
      }
      Mw[tid][kMvnMaxK + 1] = wi;
      Mw[tid][k] = rwi;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kMvnMPer; ++i) {
      const int idx = tid + kMvnThreads * i, c = idx / kMvnChunk, pr = idx % kMvnChunk;
      if (c < k) {
        Ms[pr][c] = mreg[i];
        Mw[pr][c] = mreg[i] * Mw[pr][kMvnMaxK + 1];
      }
    }
    __syncthreads();
    if (p0 + kMvnChunk < n) fetch(p0 + kMvnChunk);     // next chunk's loads fly during the sums
#pragma unroll
    for (int j = 0; j < kMvnSlots; ++j) {
      if (et + 256 * j < ntot) {
        const int r = er[j], c = ec[j];
        double a = acc[j];
        for (int pr = phase; pr < np; pr += kMvnPhases) a = fma(Ms[pr][r], Mw[pr][c], a);
        acc[j] = a;
      }
    }
  }
  // q1 and sum log d live in threads 0..63 (wave 0); the 4 phases' partial entry sums meet in LDS
  if (tid < 64) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      q1 += __shfl_xor(q1, off);
      ld += __shfl_xor(ld, off);
    }
  }
  __syncthreads();
  double* red = sm;                                    // [2][kMvnSlots * 256]
  constexpr int kRed = kMvnSlots * 256;
  for (int half = kMvnPhases / 2; half >= 1; half >>= 1) {
    if (phase >= half && phase < 2 * half) {
#pragma unroll
      for (int j = 0; j < kMvnSlots; ++j) red[(phase - half) * kRed + et + 256 * j] = acc[j];
    }
    __syncthreads();
    if (phase < half) {
#pragma unroll
      for (int j = 0; j < kMvnSlots; ++j) acc[j] += red[phase * kRed + et + 256 * j];
    }
    __syncthreads();
  }
  if (phase == 0) {
#pragma unroll
    for (int j = 0; j < kMvnSlots; ++j)
      if (et + 256 * j < ntot) A[er[j]][ec[j]] = acc[j] + (er[j] == ec[j] ? 1.0 : 0.0);
  }
  if (tid == 0) A[k][k] = q1;
  __syncthreads();
  // augmented upper Cholesky, right-looking: row p scaled by 1/R_pp, then the trailing upper
  // triangle (rows and columns p+1 .. k) updated by the whole block
  bool bad = false;
  double logdet = 0.0;
  for (int p = 0; p < k; ++p) {
    const double v = A[p][p];
    bad |= !(v > 0.0);
    const double rpp = sqrt(v);
    logdet += log(rpp);
    const int m = k - p;                               // columns p+1 .. k
    __syncthreads();                                   // everyone has read A[p][p]
    if (tid < m) A[p][p + 1 + tid] /= rpp;
    __syncthreads();
    for (int idx = tid; idx < m * m; idx += kMvnThreads) {
      const int r = p + 1 + idx / m, c = p + 1 + idx % m;
      if (r <= c) A[r][c] = fma(-A[p][r], A[p][c], A[r][c]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    const double quad = A[k][k];                       // r'D^-1 r - t't
    double res = -0.5 * (quad + (ld + 2 * logdet) + n * kLog2Pi);
    int st = 0;
    if (bad || !(fabs(res) < INFINITY)) {
      res = NAN;
      st = 1;
    }
    *out = res;
    *status = st;
  }
}

template <int K>
hipError_t launch_prep_k(const PrepArgs& a, hipStream_t s) {
  // the panel-GEMM layout (K == 0) writes k(k+1)/2 doubles per slot for few spectra per batch:
  // spread each spectrum's slots over 16 blocks (the fused layout: one block per spectrum; 4 or 8
  // gained < 7% of prep's 1.08 ms, profiles/r2w)
  hipLaunchKernelGGL(prep_kernel<K>, dim3(a.q_count, K == 0 ? 16 : 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int K>
hipError_t launch_likelihood_k(const LikelihoodArgs& a, hipStream_t s) {
  const int64_t blocks_x = (a.S + 1 + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const int64_t nb = (blocks_x * a.q_count + 7) / 8 * 8;  // 1-D, padded for the XCD remap
  if (nb > INT32_MAX) return hipErrorInvalidValue;
  if (a.num_lines == 3)
    hipLaunchKernelGGL((likelihood_kernel<K, 3>), dim3((unsigned)nb), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((likelihood_kernel<K, 0>), dim3((unsigned)nb), dim3(256), 0, s, a);
  return hipGetLastError();
}



}  // namespace

#define GPDLA_FOR_EACH_RANK(X) X(4) X(8) X(10) X(12) X(16) X(20) X(24)

bool rank_supported(int K) {
#define X(k) if (K == k) return true;
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return false;
}

// smallest compiled rank >= k (0: none).  The engine runs a rank k between the compiled ones on it
// with M padded by zero columns: those add Gram rows/columns that are exactly 0, diagonal 1 (B = I +
// M' D^-1 M) and u entries 0, so their LDL^T pivots are exactly 1 (log 1 = 0) and every update they
// make subtracts an exact 0 -- the log-likelihood is the rank-k one, bit for bit.
int fused_rank(int k) {
  if (k < 1) return 0;
#define X(kk) if (k <= kk) return kk;
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return 0;
}

int scratch_doubles(int K) {
#define X(k) if (K == k) return Layout<k>::kES;
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return 0;
}

int panel_row_doubles(int K) {
#define X(k) if (K == k) return Layout<k>::kRow;
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return 0;
}
int panel_lds_row_doubles(int K) {
#define X(k) if (K == k) return Layout<k>::kRowL;
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return 0;
}

hipError_t launch_prep(int K, const PrepArgs& a, hipStream_t s) {
  if (K == 0) return launch_prep_k<0>(a, s);  // panel-GEMM layout, rank a.k
#define X(k) if (K == k) return launch_prep_k<k>(a, s);
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_likelihood(int K, const LikelihoodArgs& a, hipStream_t s) {
#define X(k) if (K == k) return launch_likelihood_k<k>(a, s);
  GPDLA_FOR_EACH_RANK(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_reduce(const ReduceArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(reduce_kernel, dim3(a.q_count), dim3(kReduceThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_voigt_batch(const double* lambdas, int64_t n_padded, const double* z,
                              const double* N, int64_t count, int32_t num_lines,
                              const LineArgs& lines, double* out, hipStream_t s) {
  hipLaunchKernelGGL(voigt_batch_kernel, dim3((unsigned)count), dim3(256), 0, s, lambdas,
                     n_padded, z, N, num_lines, lines, out);
  return hipGetLastError();
}

hipError_t launch_mvn_single(const double* y, const double* mu, const double* M_colmajor,
                             const double* d, int64_t n, int32_t k, double* out, int32_t* status,
                             hipStream_t s) {
  if (k > kMvnMaxK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mvn_single_kernel, dim3(1), dim3(kMvnThreads), 0, s, y, mu, M_colmajor, d, n, k,
                     out, status);
  return hipGetLastError();
}

}  // namespace gpdla
