// Internal declarations shared by the kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "line_profile.h"
#include "lyman_series.h"
#include "tuning.h"

// HIP call -> C-ABI status (GPDLA_ENOMEM / GPDLA_EDEVICE with a message), in functions returning int
#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return ::gpdla::set_error(e_ == hipErrorOutOfMemory ? GPDLA_ENOMEM : GPDLA_EDEVICE,   \
                                "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                                __FILE__, __LINE__);                                        \
  } while (0)

namespace gpdla {

// C-ABI error reporting shared by the translation units (engine.hip): sets gpdla_last_error()
int set_error(int code, const char* fmt, ...);
// GPDLA_OK if `device` is a usable HIP device, else GPDLA_EDEVICE / GPDLA_EINVAL (no CPU fallback)
int check_device(int32_t device);

// Launch times of the calling thread's last one-shot call (ingest, sampler): HIP events around each
// kernel on the null stream, read back by gpdla_last_call_kernel_ms (engine.hip).  Usage: reset()
// at the call's start, before() / after() around each launch, then finish() once the call's last
// synchronous copy has returned.
struct LaunchTimes {
  static constexpr int kMax = 8;
  hipEvent_t ev[2 * kMax] = {};
  double ms[kMax] = {};
  int n = 0, done = 0;
  void reset() { n = done = 0; }
  void before() {
    if (n < kMax && (ev[2 * n] || hipEventCreate(&ev[2 * n]) == hipSuccess)) (void)hipEventRecord(ev[2 * n], 0);
  }
  void after() {
    if (n < kMax && (ev[2 * n + 1] || hipEventCreate(&ev[2 * n + 1]) == hipSuccess)) {
      (void)hipEventRecord(ev[2 * n + 1], 0);
      ++n;
    }
  }
  void finish() {
    for (int i = 0; i < n; ++i) {
      float t = 0.0f;
      ms[i] = hipEventSynchronize(ev[2 * i + 1]) == hipSuccess && hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]) ==
                  hipSuccess ? (double)t : -1.0;
    }
    done = n;
  }
};
LaunchTimes& launch_times();

// ---------------------------------------------------------------------------------------------
// Device data layout (HBM)
//
// A spectrum is turned into J "slots" (pixels the likelihood sweeps).  In reference mode slot j is
// the j-th unmasked in-range pixel and its absorption is the j-th value of the m-point profile
// (process_qsos.m:180,189); in unmasked mode J = m and masked slots carry weight 0.
//
// The sweep is split into 4 contiguous segments of L = ceil(J/4) slots (segment g = slots
// [gL, gL+L)); lanes g = 0..3 of a wave walk their segment in step, so the 7-tap instrument
// convolution is a register sliding window and the 4 segments form the K=4 dimension of a
// v_mfma_f64_4x4x4_4b.
//
// Panel row (one per slot, kRow doubles, 16-byte aligned): the Khatri-Rao row
//     e < NGRAM      : M_r * M_c  for Gram pair e = (r, c), r <= c (row-major upper triangle)
//     NGRAM..4GT-1   : 0 (tile padding)
//     4GT + i, i < K : M_i                       (the u = M' D^-1 diag(a) r contraction)
// stored permuted as row[(e & 3) * JS + (e >> 2)], so a lane with j = e & 3 reads consecutive
// tiles with one ds_read_b128.  Spare words per j hold the slot scalars.
// ---------------------------------------------------------------------------------------------
template <int K>
struct Layout {
  static constexpr int kNGram = K * (K + 1) / 2;
  static constexpr int kGT = (kNGram + 3) / 4;  // Gram tiles (4 entries each)
  static constexpr int kUT = (K + 3) / 4;       // u tiles
  static constexpr int kTiles = kGT + kUT;
  static constexpr int kJS = ((kTiles + 2) + 1) & ~1;  // per-j stride (doubles), even
  static constexpr int kRow = 4 * kJS;                 // doubles per slot row (HBM panel stride)
  static constexpr int kRowL = (kRow + 127) & ~127;    // DMA span per row: whole 1 KiB pieces
  static constexpr int kPieces = kRowL / 128;          // global_load_lds_dwordx4 per staged row
  // LDS row stride: the span plus 16 B, so the 4 segment rows a ds_read_b128 lane group touches
  // start in different bank quads (with the bare span, rows g and g+1 hit the same banks: every
  // B-operand read was a 2-way conflict, SQ_LDS_BANK_CONFLICT = 36% of LDS cycles, profiles/r1f)
  static constexpr int kRowS = kRowL + 2;
  static constexpr int kES = 4 * kTiles + 8;           // epilogue doubles per sample (Gram, u, scalars)
  // slot scalars in the spare words
  static constexpr int kLam = 0 * kJS + kTiles;        // padded wavelength at slot + 6
  static constexpr int kY = 0 * kJS + kTiles + 1;
  static constexpr int kNoise = 1 * kJS + kTiles;
  static constexpr int kMu = 1 * kJS + kTiles + 1;
  static constexpr int kOmega2 = 2 * kJS + kTiles;
  static constexpr int kValid = 2 * kJS + kTiles + 1;
};

struct SpecInfo {
  int32_t J;          // slots (0 => unusable spectrum)
  int32_t L;          // segment length ceil(J/4)
  int32_t n;          // unmasked in-range pixels (the n in n*log(2 pi))
  int32_t m;          // in-range pixels including masked
  double zmin, zmax;  // process_qsos.m:160-161
  int64_t slot_base;  // first panel row of this spectrum
  int64_t lam_base;   // first element of this spectrum's padded-wavelength array
  int32_t flags;
  int32_t scale_e;    // prep's unit scaling: noise, omega^2 x 2^scale_e; flux, mu, M x 2^(scale_e / 2)
  double de_shift;    // -n scale_e: log det D = log det D' + de_shift ln 2 (exact power-of-two scaling)
};

constexpr int kChunkSteps = 4;       // pixel steps staged per LDS chunk
constexpr int kSamplesPerWave = 16;
constexpr int kWavesPerBlock = 4;
constexpr int kSamplesPerBlock = kSamplesPerWave * kWavesPerBlock;

struct PrepArgs {
  int32_t q_count;
  const int64_t* offsets;        // device, [q_count + 1], relative to the pixel arrays below
  const double* wavelengths;
  const double* flux;
  const double* noise;
  const uint8_t* mask;
  const double* z_qsos;          // device, [q_count]
  const int64_t* slot_base;      // device, [q_count]
  const int64_t* lam_base;       // device, [q_count]
  const int64_t* slot_cap;       // device, [q_count]
  // model (device, rest grid row-major [G][K])
  int32_t num_rest;
  const double* rest;
  const double* mu;
  const double* M_rowmajor;
  const double* log_omega;
  double c_0, tau_0, beta;
  // params
  double min_lambda, max_lambda, lya, lyman_limit, min_z_cut, max_z_cut, pixel_spacing;
  int32_t absorption_mode;
  int32_t k;                     // rank (read by the panel-GEMM layout, prep_kernel<0>)
  int32_t om2_hi_e;              // binary exponent of the model's largest omega^2 (1 + c_0)^2 (units)
  // outputs
  SpecInfo* info;
  double* panel;                 // fused layout: [slots][kRow]; GEMM layout: [slots][k(k+1)/2] (nullptr:
                                 // the int8 panel paths form the Khatri-Rao entries from panel_m themselves)
  double* panel_m;               // GEMM layout only: [slots][k] M rows
  double* srow;                  // GEMM layout only: [slots][8] lam, y, noise, mu, om2, valid
  double* lam_pad;
  int32_t* slot_pixel;           // scratch map slot -> pixel (size = total slot capacity)
};

// Line-profile data.  Device buffer layout (doubles):
//   [kMaxLines][kCoreTable] core tables | [kMaxLines][kWingStride] wing polynomials |
//   fac[kMaxLines] | 2^(j/64)[64]
// fac_j = c / (lambda_j 1e8) / (sigma sqrt 2), so x_j = lambda * fac_j / (1 + z) - c / (sigma sqrt 2)
// (voigt.c:278-279,287 divided by sigma sqrt 2).
constexpr size_t kLineBufWing = (size_t)kMaxLines * kCoreTable;
constexpr size_t kLineBufFac = kLineBufWing + (size_t)kMaxLines * kWingStride;
constexpr size_t kLineBufExp2 = kLineBufFac + kMaxLines;  // 2^(j/64), j = 0..63 (exp_tab64)
constexpr size_t kLineBufExp128 = kLineBufExp2 + 64;      // 2^(j/128), j = 0..127 (exp_tab128_nc)
constexpr size_t kLineBufDoubles = kLineBufExp128 + 128;

struct LineArgs {
  const double* buf;   // device line buffer (layout above)
};

// ---- panel-GEMM path (any rank 1..kGemmMaxK; gemm_path.hip + gemm_f64.hip or gemm_i8.hip)
constexpr int kGemmMaxK = 64;
constexpr int kWeightQuarters = 4;                 // weights_kernel: waves per segment
// weights kernels: raw profiles per fix-up branch (raw_profile3_batch).  configs[4] A/B: 2 beats 1 and
// 4 (4 needs more registers than 4 waves per SIMD allow; profiles/r4k)
constexpr int kWB = 2;
constexpr int kWeightParts = 4 * kWeightQuarters;  // per-sample partial sums (segment x quarter)

struct WeightsArgs {
  const SpecInfo* info;
  int32_t q;                     // spectrum within the batch
  const double* srow;            // this spectrum's slot scalars [cap][8]
  const double* lam_pad;         // this spectrum's padded wavelengths
  int64_t cap;                   // this spectrum's slot capacity (GEMM inner dimension)
  const double* offsets;         // [S] ascending offsets
  const double* nhi;             // [S]
  int64_t S, s0;                 // chunk = sorted samples s0 .. s0 + sc - 1 (index S = null model)
  int32_t sc;
  int32_t num_lines;
  LineArgs lines;
  double* wg;                    // a^2 / d, weight tiles of gemm_f64 (GemmF64Args)
  double* wu;                    // a r / d, likewise
  double* q1p;                   // [sc][kWeightParts] partial sum r^2 / d
  double* ldp;                   // [sc][kWeightParts] partial sum log d
};

struct LdlArgs {
  const SpecInfo* info;
  int32_t q;
  int32_t k;
  const double* G;               // Gram, quad_index(s, e, k(k+1)/2), entries in gram_tile_index order
  const float* G32;              // the same in fp32 (panel_gemm_i8_24), or nullptr: then G is read
  const double* U;               // u, quad_index(s, i, k)
  const double* q1p;
  const double* ldp;
  int64_t S, s0;
  int32_t sc;
  const int32_t* perm;
  double* sample_ll;             // this spectrum's row, or nullptr
  double* ll_null;               // this spectrum's entry
  int32_t* status;
};

hipError_t launch_weights(const WeightsArgs& a, hipStream_t s);
hipError_t launch_ldl_batch(const LdlArgs& a, hipStream_t s);

// Gram / u hand-off between the panel GEMMs (gemm_f64.hip, gemm_i8.hip) and ldl_mfma_kernel:
// samples in groups of 4, entry e of sample s at (s >> 2) 4 n + 4 e + (s & 3) (n = entries per
// sample).  A GEMM lane's 4 consecutive samples of one entry are one 16-B (fp32) or 32-B store, and
// the LDL^T wave (4 samples x the 16 positions of a tile) reads 64 consecutive values.  Buffers
// cover whole GEMM sample tiles (gemm_f64_rows), so the GEMMs store without a sample bound.
__host__ __device__ inline int64_t quad_index(int64_t s, int64_t e, int64_t n) {
  return (s >> 2) * 4 * n + 4 * e + (s & 3);
}

// fp64 Gram / u GEMM of the panel path (gemm_f64.hip).  The weights are stored per 32-sample tile
// as [tile][slot (cap16)][32], sample 4 g + i of the tile at position 8 i + g (weights_kernel), for
// whole 128-sample blocks (sc rounded up to kGemmF64TileS)
constexpr int kGemmF64Waves = GPDLA_F64_WAVES;     // waves per block, 32 samples each
constexpr int kGemmF64TileS = 32 * kGemmF64Waves;
__host__ __device__ inline int64_t gemm_f64_cap16(int64_t cap) { return (cap + 15) / 16 * 16; }
// row strides (doubles) of the panel-GEMM layout's Khatri-Rao rows (k(k+1)/2 entries) and M rows
// (k): rounded up to even so every row starts 16-B aligned for gemm_f64's LDS-DMA pieces
__host__ __device__ inline int64_t gemm_ldp(int k) { return ((int64_t)k * (k + 1) / 2 + 1) / 2 * 2; }
__host__ __device__ inline int64_t gemm_ldm(int k) { return ((int64_t)k + 1) / 2 * 2; }
// doubles read past the last panel / M row by gemm_f64 (the pad rows up to cap16 and a 128-entry
// piece starting in the last row); the engine keeps them zeroed
__host__ __device__ inline int64_t gemm_panel_slack(int64_t ld) { return 16 * ld + 128; }
__host__ __device__ inline int64_t gemm_f64_rows(int64_t sc) { return (sc + kGemmF64TileS - 1) / kGemmF64TileS * kGemmF64TileS; }
struct GemmF64Seg {              // one product C = W' P of a launch
  const double* W;               // weight tiles (layout above)
  const double* P;               // [slot][ldp] this spectrum's panel rows
  int64_t ldp;                   // doubles per panel row
  int32_t nent;                  // output entries per sample (k(k+1)/2 Gram, or k u)
  double* C;                     // quad_index(s, e, nent), for every sample of the padded tiles
};
struct GemmF64Args {
  GemmF64Seg seg[2];             // Gram and u, one launch (the u entry tiles after the Gram ones)
  int32_t nseg;
  int64_t cap, cap16;            // slots, and slots padded to 16 (the weights' tile rows)
  int32_t sc;                    // samples of the chunk
};
hipError_t launch_gemm_f64(const GemmF64Args& a, hipStream_t s);

struct LikelihoodArgs {
  int32_t q_count;
  const SpecInfo* info;
  const double* panel;
  const double* lam_pad;
  const double* offsets;         // [S] offset samples (ascending; see engine.hip)
  const double* nhi;             // [S]
  const int32_t* perm;           // [S] sorted sample index -> output sample index
  int64_t S;
  int32_t num_lines;
  LineArgs lines;
  double* sample_ll;             // [q_count][ld] or nullptr
  int64_t ld;
  double* ll_null;               // [q_count]
  int32_t* status;
};

// ---- int8 Ozaki-sliced fused path (kernels_i8.hip; ranks with i8_supported(K))
//
// The Gram/u contraction sum_slot w(sample, slot) P(slot, entry) runs on v_mfma_i32_16x16x64_i8
// exactly in integers: per slot the weights are w~ = a^2/d (omega^2+sigma^2) in [0, 1] (Gram) and
// a r/d / beta in [-1, 1] (u, beta a static per-slot bound), quantised as X_A = rint(w~ 2^30); the
// panel entries P~ = M_r M_c / (omega^2+sigma^2) and M_i beta as X_B = rint(P~ / s_e 2^30) with a
// per-entry power-of-two scale s_e.  X_A + 2^31 is split into 4 bytes (XOR 0x80 -> signed digits,
// offset 0x808080 per slot), X_B into 4 balanced signed base-256 digits; the 13 digit pairs of
// level i + j <= 4 accumulate exactly in int32 per level, and the epilogue forms
//   sum_slot X_A X_B = sum_l 2^(8(6-l)) C_l + 0x808080 * colsum_e
// in fp64.  See DESIGN.md section 4 for the error budget.
template <int K>
struct I8Layout {
  static constexpr int kNGram = K * (K + 1) / 2;
  static constexpr int kGT = (kNGram + 15) / 16;     // Gram tiles (16 entries each)
  static constexpr int kUT = (K + 15) / 16;          // u tiles
  static constexpr int kTiles = kGT + kUT;
  static constexpr int kEnt = 16 * kTiles;           // entries incl. padding (<= 256)
  static constexpr int kUBase = 16 * kGT;            // entry of u_0
  static constexpr int kChunkSlots = 64;             // 4 segments x 16 steps (MFMA K = 64)
  static constexpr int kPlaneBytes = kEnt * 64;      // one digit plane of a chunk
  static constexpr int kChunkBytes = 4 * kPlaneBytes;
  static constexpr int kScal = 8;                    // doubles per slot record
  static constexpr int kScalBytes = kChunkSlots * kScal * 8;
};
constexpr int kI8MaxSlots = 30000;  // int32 level sums stay exact up to 4 * 32767 * 2^14 < 2^31

struct ConvertI8Args {
  int32_t q_count;
  const SpecInfo* info;
  const double* panel;           // fused f64 layout (prep_kernel<K>)
  const double* lam_pad;
  const int64_t* chunk_base;     // device, [q_count]: first i8 chunk of each spectrum
  uint8_t* panel_i8;             // [chunks][4 planes][kEnt][64 B] (16 B granules swizzled)
  double* scal;                  // [chunks][64][8]: lam(+6), y, noise, mu, om2, gscale, uscale, 0
  double* ent;                   // [q_count][2][kEnt]: s_e, colsum_e
};

struct LikelihoodI8Args {
  int32_t q_count;
  const SpecInfo* info;
  const uint8_t* panel_i8;
  const double* scal;
  const double* ent;
  const int64_t* chunk_base;
  const double* lam_pad;
  const double* offsets;
  const double* nhi;
  const int32_t* perm;
  int64_t S;
  LineArgs lines;
  double* scratch;               // [grid blocks][64][Layout<K>::kES]
  double* sample_ll;
  int64_t ld;
  double* ll_null;
  int32_t* status;
};

// ---- int8 Ozaki contraction on the panel-GEMM path (gemm_i8.hip; any rank 1..kGemmMaxK)
// K index of slot (segment g, step t): g Ls16 + t with Ls16 = 16 ceil(L / 16); a spectrum's K
// extent 4 Ls16 is a multiple of 64 and at most kstride = i8_gemm_kstride(slot_cap).
// Entries: Gram 0..E-1 padded to Ep = 64 ceil(E / 64), then u 0..k-1 padded to 64 ceil(k / 64).
__host__ __device__ inline int64_t i8_gemm_kstride(int64_t slot_cap) {
  return 64 * ((slot_cap - 16 + 63 + 63) / 64);  // >= lpix + 63 >= 4 Ls16 (slot_cap = 4 ceil(lpix/4) + 16)
}
// Order of the k(k+1)/2 Gram entries (r <= c < k) in the panel-GEMM path's Khatri-Rao rows and
// Gram arrays: tile-major over the 4 x 4 tiles the LDL^T factors (gemm_path.hip ldl_mfma_kernel), so
// the 16 lanes reading one tile of a sample read 128 contiguous bytes.  With NT = ceil((k+1)/4) tiles
// per side, the first 4 (NT - 1) columns form whole tile columns: tiles (L, I), L <= I <= NT - 2,
// row-block major, 10 entries (upper triangle, i <= j) on the diagonal and 16 (i-major) off it.  The
// w = k - 4 (NT - 1) <= 3 Gram columns of the last tile column follow: 4 w entries per tile (L, NT-1),
// L < NT - 1, then the w (w + 1) / 2 of the corner tile.
__host__ __device__ inline int gram_tile_index(int r, int c, int k) {
  const int NT = (k + 4) / 4, Kf = 4 * (NT - 1), w = k - Kf;
  const int L = r >> 2, I = c >> 2, i = r & 3, j = c & 3;
  if (c < Kf) {
    const int row = 10 * L + 16 * (L * (NT - 2) - L * (L - 1) / 2);
    return row + (I == L ? i * 4 - i * (i - 1) / 2 + (j - i) : 10 + 16 * (I - L - 1) + 4 * i + j);
  }
  const int base2 = 10 * (NT - 1) + 8 * (NT - 1) * (NT - 2);
  return base2 + L * 4 * w + (L == NT - 1 ? i * w - i * (i - 1) / 2 + (j - i) : i * w + j);
}

// The 24-bit path's error is absolute, ~2^-24 of the Gram's scale: relative to max(|ll|, 1) it grows
// where |ll| is small, which short spectra make likely (n = 3: 5.05e-7 against the fp64 panel,
// profiles/round5/r10b).  Spectra of at most kI8NarrowKs 64-slot K steps (<= 128 pixels) therefore
// take the 32-bit digits (4 planes, ~1e-9) on that path; they cost next to nothing.  Decided on the
// slot capacity (host and device agree without a sync): ks_bound = ceil(ceil(lpix / 4) / 16).
constexpr int kI8NarrowKs = 2;
__host__ __device__ inline int i8_ks_bound(int64_t slot_cap) { return (int)(((slot_cap - 16) / 4 + 15) / 16); }
__host__ __device__ inline int i8_spectrum_nd(int nd, int64_t slot_cap) {
  return (nd == 3 && i8_ks_bound(slot_cap) <= kI8NarrowKs) ? 4 : nd;
}

__host__ __device__ inline int i8_gemm_entries(int k) {
  return 64 * ((k * (k + 1) / 2 + 63) / 64) + 64 * ((k + 63) / 64);
}

struct ConvertGemmI8Args {
  int32_t k;
  const SpecInfo* info;
  const double* panel_m;         // [slots][k] M rows (the Khatri-Rao entries are formed from them)
  const double* srow;            // [slots][8]
  const int64_t* slot_base;      // device [q]
  const int64_t* slot_cap;       // device [q]
  const int64_t* bbase;          // device [q]: byte offset of the spectrum's B digit planes
  int32_t nd;                    // Gram digit planes written: 4 (levels <= 3) or 3 (levels <= 2); u: 4
  uint8_t* bdig;                 // [planes 4][entries][kstride] per spectrum
  double* ent;                   // [q][2][entries]: s_e / scaleA, c * colsum_e
};

struct WeightsI8Args {
  const SpecInfo* info;
  int32_t q;
  const double* srow;            // this spectrum's slot scalars
  const double* lam_pad;         // this spectrum's padded wavelengths
  int64_t kstride;
  const double* offsets;
  const double* nhi;
  int64_t S, s0;
  int32_t sc;
  int64_t rows;                  // sample rows allocated per digit plane (>= sc, multiple of 128)
  LineArgs lines;
  int32_t nd;                    // Gram digit planes written (4 or 3); u: 4
  uint8_t* adig;                 // [type 2 (Gram, u)][plane 4][rows][kstride]
  double* q1p;
  double* ldp;
};

struct GemmI8Args {
  const SpecInfo* info;
  int32_t q;
  int32_t k;
  int64_t kstride;
  int64_t rows;
  int32_t sc;
  int32_t nd;                    // Gram digit planes per operand: 4 (10 pairs, levels <= 3) or 3 (6 pairs); u: 4
  int32_t e_tile0, ny;           // set by launch_gemm_i8: first 64-entry tile and tile count of a launch
  int32_t ks_bound;              // bound on the spectrum's 64-slot K steps, ceil(ceil(lpix / 4) / 16)
  int32_t u_tile;                // set by launch_gemm_i8: the u entry tile fused into the Gram launch, or -1
  const uint8_t* adig;
  const uint8_t* bdig;           // this spectrum's B planes
  const double* ent;             // this spectrum's [2][entries]
  double* G;                     // quad_index(s, e, E), every sample of the rows
  float* G32;                    // if set, the Gram goes here in fp32 instead (24-bit path)
  double* U;                     // quad_index(s, i, k)
};

hipError_t launch_convert_gemm_i8(const ConvertGemmI8Args& a, int32_t q_count, hipStream_t s);
hipError_t launch_weights_i8(const WeightsI8Args& a, hipStream_t s);
hipError_t launch_diag_raw_profile(const double* lam, int64_t n, double z, double N, int32_t f32,
                                   const LineArgs& lines, double* out, hipStream_t s);
hipError_t launch_gemm_i8(const GemmI8Args& a, hipStream_t s);

bool i8_supported(int K);
int i8_fused_rank(int k);
int i8_chunk_bytes(int K);
int i8_entries(int K);
hipError_t launch_convert_i8(int K, const ConvertI8Args& a, hipStream_t s);
hipError_t launch_likelihood_i8(int K, const LikelihoodI8Args& a, hipStream_t s);

struct ReduceArgs {
  int32_t q_count;
  const SpecInfo* info;
  const double* sample_ll;
  int64_t ld;
  int64_t S;
  double* ll_dla;
  double* zmin;
  double* zmax;
  int32_t* num_pixels;
};

hipError_t launch_prep(int K, const PrepArgs& a, hipStream_t s);
hipError_t launch_likelihood(int K, const LikelihoodArgs& a, hipStream_t s);
hipError_t launch_reduce(const ReduceArgs& a, hipStream_t s);
hipError_t launch_voigt_batch(const double* lambdas, int64_t n_padded, const double* z,
                              const double* N, int64_t count, int32_t num_lines,
                              const LineArgs& lines, double* out, hipStream_t s);
hipError_t launch_mvn_single(const double* y, const double* mu, const double* M_colmajor,
                             const double* d, int64_t n, int32_t k, double* out,
                             int32_t* status, hipStream_t s);
bool rank_supported(int K);
int fused_rank(int k);
int panel_row_doubles(int K);
int panel_lds_row_doubles(int K);
int scratch_doubles(int K);

// host-side table fitting (faddeeva_host.cpp)
void fit_core_table(int line, double* core);
void fit_wing_line(int line, double* wing);
double line_profile_error(int line);

}  // namespace gpdla
