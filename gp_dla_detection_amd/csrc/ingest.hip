// Spectrum ingest on gfx950: read_spec.m's derived columns and preload_qsos.m's numeric
// stage, batched over a CSR of the catalogue's spectra (FITS parsing stays on the host).
//
//   read_spec.m:27-28   wavelengths = 10.^loglam     single, rounded once from double (wavelength():
//                                                   exp2 with a rounding-boundary guard, else pow)
//                                                   -- the correctly rounded single over every float32
//                                                   loglam in [3.5, 4.1] (checked exhaustively against
//                                                   extended precision); MATLAB's own single pow is
//                                                   unpinned at the last ulp
//   read_spec.m:30-31   noise_variance = 1 ./ ivar   single IEEE division
//   read_spec.m:36-38   pixel_mask = ivar == 0 | bitget(and_mask, 24)
//   preload_qsos.m:19-21  entries with filter_flags > 0 are skipped (empty cells)
//   preload_qsos.m:26     rest = wavelengths / (1 + z)  (single: the double 1 + z rounded to single);
//                         the three range tests on rest become loglam intervals found once per
//                         spectrum (rest is monotone in loglam; see first_key_past), so only the cells'
//                         wavelengths need the pow
//   preload_qsos.m:29-33  nanmedian of the flux over unmasked pixels with rest in [1310, 1325]: the
//                         window's values gathered in LDS, NaNs dropped, bitonic-sorted (a radix
//                         select over the spectrum when more than kWindowCap), MATLAB's median
//                         (meanof(a, b) = a + (b - a) / 2 for finite same-sign a, b)
//   preload_qsos.m:36-49  bit 3 (value 4) when that median is NaN; bit 4 (value 8) when fewer than
//                         min_num_pixels unmasked pixels have rest in [911.75, 1215.75]
//   preload_qsos.m:51-54  normaliser; flux / median, noise_variance / median^2 (single)
//   preload_qsos.m:56-62  the loading range [910, 1217] plus the first unmasked pixel after its last
//                         and the last unmasked pixel before its first
//   preload_qsos.m:64-67  the selected pixels, in order (a block-wide ordered compaction)
//
// Three launches: the range ends as loglam keys (one wave per spectrum); then one 256-thread block
// per spectrum in each of two: the median, the flags,
// the loading range's ends and neighbours and the cell length; the host turns the lengths into CSR
// offsets; the second writes the cells (an order-preserving compaction over the span from the lower
// neighbour to the upper one: the selection is a mask, as in the reference, not assumed contiguous).
// HBM-bound elementwise work: loglam, ivar and and_mask read once per pixel (12 B), flux only in the
// normalisation window; the span's columns re-read and 13 B per selected pixel written.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/gpdla.h"
#include "internal.h"

namespace gpdla {
namespace {

#ifndef GPDLA_INGEST_SCAN_THREADS
#define GPDLA_INGEST_SCAN_THREADS 128          // with the 2,048 cap: 148 us per batch; 256 threads 159
#endif
#ifndef GPDLA_INGEST_WINDOW_CAP
#define GPDLA_INGEST_WINDOW_CAP 2048            // LDS per block 8 KiB: more spectra per CU
#endif
constexpr int kIngestThreads = GPDLA_INGEST_SCAN_THREADS;   // the scan's block
constexpr int kScanWaves = kIngestThreads / 64;
constexpr int kWindowCap = GPDLA_INGEST_WINDOW_CAP;            // median-set values per spectrum sorted in LDS (more: radix select)
#ifndef GPDLA_INGEST_SCAN_UNROLL
#define GPDLA_INGEST_SCAN_UNROLL 4
#endif
constexpr int kUnroll = GPDLA_INGEST_SCAN_UNROLL;   // scan rounds whose loads are issued together
#ifndef GPDLA_INGEST_WRITE_UNROLL
#define GPDLA_INGEST_WRITE_UNROLL 4           // write-pass rounds whose loads are issued together
#endif

struct IngestArgs {
  int64_t Q;
  const int64_t* off;                       // [Q + 1] input CSR
  const float* loglam;
  const float* flux;
  const float* ivar;
  const int32_t* and_mask;
  const double* z;
  const uint8_t* flags_in;
  gpdla_preload_params p;
  // pass-1 results per spectrum
  uint8_t* flags_out;
  float* median;
  int64_t* count;                           // cell length (0 when skipped or filtered)
  int64_t* ends;                            // [Q][4]: first, last of the loading range, after, before (-1 = none)
  int32_t* keys;                            // [Q][6]: the three ranges as loglam order keys [lo, hi)
  // pass-2 outputs
  const int64_t* out_off;                   // [Q + 1]
  float* w_out;
  float* f_out;
  float* nv_out;
  uint8_t* m_out;
  double* normalizers;
};

__device__ inline bool pixel_mask(const IngestArgs& a, int64_t i) {
  return a.ivar[i] == 0.0f || ((a.and_mask[i] >> (a.p.brightsky_bit - 1)) & 1);    // read_spec.m:36-38
}

// read_spec.m:28, 10.^loglam in single, correctly rounded: 2^(loglam log2 10) in double (relative error
// < 3e-15: the product's two roundings at |t| < 120 and exp2's ulp) rounded once to single -- the
// correctly rounded single unless the double lies within 1e-14 of a rounding boundary (a midpoint
// between singles; half that spacing below a power of two), where the double pow decides.
__device__ inline float wavelength(float loglam) {
  const double t = (double)loglam * 3.3219280948873623478703194;
  if (!(fabs(t) < 120.0)) return (float)pow(10.0, (double)loglam);               // NaN, inf, outside
  const double wd = exp2(t);
  const float w = (float)wd;
  const double h = ldexp(1.0, ilogbf(w) - 24);                                    // half an ulp of w
  const double r = fabs(wd - (double)w), tol = 1e-14 * wd;
  if (fabs(r - h) <= tol || fabs(r - 0.5 * h) <= tol) return (float)pow(10.0, (double)loglam);
  return w;
}

// The three rest-frame ranges of preload_qsos.m (:29 normalisation, :41 model, :56 loading) as
// intervals of loglam.  rest(L) = single(single(10^L) / single(1 + z)) (:26) is non-decreasing in L:
// the correctly rounded single 10^L is, and so are the IEEE division by a positive constant and the
// widening to double for the comparison.  So {L : lo <= rest(L) <= hi} is an interval of float32 L,
// found once per spectrum -- its ends are the first L with rest(L) >= lo and the first with
// rest(L) > hi -- and each pixel's test is two integer compares on its loglam's order key, exactly the
// reference's comparison with no per-pixel pow.  Order key: the float's bits, negatives mirrored, so
// that key order is float order (NaN keys land beyond +inf or below -inf and are excluded apart).
constexpr int kRanges = 3;
constexpr int32_t kKeyMin = (int32_t)0x807FFFFF;         // key(-inf)
constexpr int32_t kKeyNone = 0x7F800001;                 // one past key(+inf): "no such L"

__device__ inline int32_t order_key(float f) {
  const int32_t i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ inline float key_float(int32_t k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

__device__ inline bool past(float loglam, float one_pz, double end, bool strict) {
  const double r = (double)(wavelength(loglam) / one_pz);
  return strict ? r > end : r >= end;
}

// The first key whose L is past `end` (kKeyNone if none).  The step lies within an ulp or two of the
// double-precision estimate log10(end (1 + z)); lanes 10 j .. 10 j + 9 of a wave test the ten keys
// around it for end j (six ends, one ballot); an end whose step is not among its ten keys (a
// degenerate end or z) is found by its lane's binary search over every key.
__device__ inline int32_t find_key(double end, bool strict, float one_pz, unsigned group) {
  const int32_t c = order_key((float)log10(end * (double)one_pz)) - 5;
  if (group != 0 && !(group & 1)) return c + __ffs(group) - 1;
  int64_t lo = kKeyMin, hi = (int64_t)kKeyNone;                                   // answer in [lo, hi]
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (past(key_float((int32_t)mid), one_pz, end, strict)) hi = mid; else lo = mid + 1;
  }
  return (int32_t)lo;
}

enum : unsigned { kNormWindow = 1, kModelRange = 2, kLoadingRange = 4 };

__device__ inline unsigned range_bits(float loglam, const int32_t* keys) {
  const int32_t k = order_key(loglam);
  unsigned bits = 0;
#pragma unroll
  for (int r = 0; r < kRanges; ++r) bits |= (k >= keys[2 * r] && k < keys[2 * r + 1]) ? 1u << r : 0u;
  return isnan(loglam) ? 0u : bits;
}

// The six interval ends of each spectrum, one wave per spectrum (pass 0: the pow stays out of the
// scan's register budget).
constexpr int kKeySpectraPerBlock = 4;

__global__ __launch_bounds__(64 * kKeySpectraPerBlock) void preload_keys_kernel(IngestArgs a) {
  const int64_t q = (int64_t)blockIdx.x * kKeySpectraPerBlock + (threadIdx.x >> 6);
  if (q >= a.Q || a.flags_in[q] > 0) return;
  const double end[2 * kRanges] = {a.p.normalization_min_lambda, a.p.normalization_max_lambda, a.p.min_lambda,
                                   a.p.max_lambda, a.p.loading_min_lambda, a.p.loading_max_lambda};
  const float one_pz = (float)(1.0 + a.z[q]);
  const int lane = threadIdx.x & 63, j = min(lane / 10, 2 * kRanges - 1);
  const int32_t c = order_key((float)log10(end[j] * (double)one_pz)) - 5;
  const bool t = lane < 10 * 2 * kRanges && past(key_float(c + lane % 10), one_pz, end[j], j & 1);
  const uint64_t bal = __ballot(t);
  if (lane < 2 * kRanges)
    a.keys[q * 2 * kRanges + lane] = find_key(end[lane], lane & 1, one_pz, (unsigned)(bal >> (10 * lane)) & 0x3FFu);
}

template <typename T, typename Op>
__device__ inline T block_reduce(T v, T* red, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  T r = red[0];
#pragma unroll
  for (int w = 1; w < kScanWaves; ++w) r = op(r, red[w]);
  return r;
}

// A pixel of the median's set (preload_qsos.m:29-33): unmasked, in the normalisation window, flux
// not NaN (nanmedian).
__device__ inline bool in_window(const IngestArgs& a, int64_t i, const int32_t* kr) {
  return !pixel_mask(a, i) && (range_bits(a.loglam[i], kr) & kNormWindow) && !isnan(a.flux[i]);
}

// The k-th smallest (0-based) flux of the median's set when the set overflows LDS (a finely sampled
// spectrum): a radix select on the values' order keys, one bit per pass over the spectrum -- exact,
// and no sort.
__device__ float window_select(const IngestArgs& a, int64_t b, int64_t e, const int32_t* kr, int64_t k,
                               int64_t* red) {
  uint32_t prefix = 0, seen = 0;                  // the key bits decided so far, and which bits those are
  for (int bit = 31; bit >= 0; --bit) {
    int64_t zeros = 0;                            // set members matching the prefix with this bit clear
    for (int64_t i = b + threadIdx.x; i < e; i += kIngestThreads) {
      if (!in_window(a, i, kr)) continue;
      const uint32_t u = (uint32_t)order_key(a.flux[i]) ^ 0x80000000u;
      zeros += (u & seen) == prefix && !((u >> bit) & 1u);
    }
    zeros = block_reduce(zeros, red, [](int64_t x, int64_t y) { return x + y; });
    if (k >= zeros) {
      k -= zeros;
      prefix |= 1u << bit;
    }
    seen |= 1u << bit;
  }
  return key_float((int32_t)(prefix ^ 0x80000000u));
}

__global__ __launch_bounds__(kIngestThreads) void preload_scan_kernel(IngestArgs a) {
  __shared__ float win[kWindowCap];
  __shared__ int nwin;
  __shared__ int64_t red64[kScanWaves];
  __shared__ int32_t red32[kScanWaves];
  __shared__ int64_t red4[3][kScanWaves];
  const int64_t q = blockIdx.x;
  const int64_t b = a.off[q], e = a.off[q + 1];
  int64_t* ends = a.ends + q * 4;
  uint8_t flags = a.flags_in[q];
  if (flags > 0) {                                                                // :19-21
    if (threadIdx.x == 0) {
      a.flags_out[q] = flags;
      a.count[q] = 0;
      a.median[q] = NAN;
      ends[0] = ends[1] = ends[2] = ends[3] = -1;
    }
    return;
  }
  if (threadIdx.x == 0) nwin = 0;
  __syncthreads();
  int32_t kr[2 * kRanges];
#pragma unroll
  for (int j = 0; j < 2 * kRanges; ++j) kr[j] = a.keys[q * 2 * kRanges + j];
  int32_t nrange = 0;
  int64_t nload = 0, first = LLONG_MAX, last = -1;
  for (int64_t c = b + threadIdx.x; c < e; c += kIngestThreads * kUnroll) {
    float ll[kUnroll], iv[kUnroll];
    int32_t am[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {                                           // all loads first
      const int64_t i = c + u * kIngestThreads;
      const bool ok = i < e;
      ll[u] = ok ? a.loglam[i] : 0.0f;
      iv[u] = ok ? a.ivar[i] : 0.0f;
      am[u] = ok ? a.and_mask[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i = c + u * kIngestThreads;
      if (i >= e) break;
      const unsigned r = range_bits(ll[u], kr);
      const bool mask = iv[u] == 0.0f || ((am[u] >> (a.p.brightsky_bit - 1)) & 1);
      if (!mask && (r & kNormWindow)) {
        const float fl = a.flux[i];                                               // flux read in the window only
        if (!isnan(fl)) {
          const int slot = atomicAdd(&nwin, 1);                                  // :29-33 (order: sorted below)
          if (slot < kWindowCap) win[slot] = fl;
        }
      }
      nrange += !mask && (r & kModelRange);                                       // :41-43
      if (r & kLoadingRange) {                                                    // :56-57
        ++nload;
        first = min(first, i - b);
        last = max(last, i - b);
      }
    }
  }
  // the four counts in one barrier (which also completes the window gather)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nrange += __shfl_xor(nrange, o);
    nload += __shfl_xor(nload, o);
    first = min(first, (int64_t)__shfl_xor(first, o));
    last = max(last, (int64_t)__shfl_xor(last, o));
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red32[wave] = nrange;
    red4[0][wave] = nload;
    red4[1][wave] = first;
    red4[2][wave] = last;
  }
  __syncthreads();
  nrange = red32[0];
  nload = red4[0][0];
  first = red4[1][0];
  last = red4[2][0];
#pragma unroll
  for (int w = 1; w < kScanWaves; ++w) {
    nrange += red32[w];
    nload += red4[0][w];
    first = min(first, red4[1][w]);
    last = max(last, red4[2][w]);
  }
  const int n = nwin;
  float lo = NAN, hi = NAN;                       // the set's middle values (the same one for odd n)
  if (n > kWindowCap) {
    hi = window_select(a, b, e, kr, n / 2, red64);
    lo = (n & 1) ? hi : window_select(a, b, e, kr, n / 2 - 1, red64);
  } else if (n <= 64) {
    // the usual case (~50 values at SDSS sampling): wave 0 sorts in registers, the same compare-exchange
    // network as the LDS sort below (pairs (i, i ^ j) of np2 values, swap when (x_i > x_l) == up), so
    // the two give the same order, signed zeros included; no barrier
    if (wave == 0 && n > 0) {
      int np2 = 1;
      while (np2 < n) np2 <<= 1;
      float v = lane < n ? win[lane] : INFINITY;
      for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          const float o = __shfl_xor(v, j);
          const bool lower = (lane & j) == 0;
          const float xi = lower ? v : o, xl = lower ? o : v;
          if ((xi > xl) == ((lane & k) == 0)) v = o;
        }
      }
      hi = __shfl(v, n / 2);
      lo = __shfl(v, (n & 1) ? n / 2 : n / 2 - 1);
    }
  } else if (n > 0) {
    // bitonic sort of the window (padded with +inf to a power of two)
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + threadIdx.x; i < np2; i += kIngestThreads) win[i] = INFINITY;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < np2; i += kIngestThreads) {
          const int l = i ^ j;
          if (l > i) {
            const float x = win[i], y = win[l];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
              win[i] = y;
              win[l] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    hi = win[n / 2];
    lo = (n & 1) ? hi : win[n / 2 - 1];
  }
  float med = NAN;                                                                // median.m of an empty set
  if (n > 0) {
    if (n & 1) {
      med = hi;
    } else {                                                                      // median.m's meanof(a, b)
      const int slo = (lo > 0.0f) - (lo < 0.0f), shi = (hi > 0.0f) - (hi < 0.0f);   // MATLAB sign
      med = (slo == shi && isfinite(lo) && isfinite(hi)) ? lo + (hi - lo) / 2.0f : (lo + hi) / 2.0f;
    }
  }
  // the loading range's unmasked neighbours (:60-62).  No pixel outside [first, last] is in the loading
  // range (they are its extreme indices), so the neighbours are the nearest unmasked pixels on either
  // side: found 256 at a time outward from the range, stopping at the first chunk that holds one.
  int64_t after = LLONG_MAX, before = -1;
  // both sides in one reduction per round (2 barriers; one round unless 256 pixels in a row are masked)
  for (int64_t r = 0; last >= 0; r += kIngestThreads) {
    const int64_t ia = b + last + 1 + r + threadIdx.x, ib = b + first - 1 - r - threadIdx.x;
    const bool need_a = after == LLONG_MAX && b + last + 1 + r < e, need_b = before < 0 && b + first - 1 - r >= b;
    if (!need_a && !need_b) break;                                                // block-uniform
    int64_t va = need_a && ia < e && !pixel_mask(a, ia) ? ia - b : LLONG_MAX;
    int64_t vb = need_b && ib >= b && !pixel_mask(a, ib) ? ib - b : -1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      va = min(va, (int64_t)__shfl_xor(va, o));
      vb = max(vb, (int64_t)__shfl_xor(vb, o));
    }
    __syncthreads();                                                              // red4 reuse
    if (lane == 0) {
      red4[0][wave] = va;
      red4[1][wave] = vb;
    }
    __syncthreads();
    int64_t ta = red4[0][0], tb = red4[1][0];
#pragma unroll
    for (int w = 1; w < kScanWaves; ++w) {
      ta = min(ta, red4[0][w]);
      tb = max(tb, red4[1][w]);
    }
    if (need_a) after = ta;
    if (need_b) before = tb;
  }
  if (threadIdx.x != 0) return;
  ends[0] = last >= 0 ? first : -1;
  ends[1] = last;
  ends[2] = after == LLONG_MAX ? -1 : after;
  ends[3] = before;
  a.median[q] = med;
  if (isnan(med)) {                                                               // :36-39
    a.flags_out[q] = flags | 4;
    a.count[q] = 0;
    return;
  }
  if (nrange < a.p.min_num_pixels) {                                              // :46-49
    a.flags_out[q] = flags | 8;
    a.count[q] = 0;
    return;
  }
  a.flags_out[q] = flags;
  a.count[q] = nload + (ends[2] >= 0) + (ends[3] >= 0);                           // the cell length
}

#ifndef GPDLA_INGEST_WRITE_THREADS
#define GPDLA_INGEST_WRITE_THREADS 128          // 128 / 64: 108 us per batch, 256: 120, 512: 167
#endif
constexpr int kWriteThreads = GPDLA_INGEST_WRITE_THREADS;
constexpr int kWriteWaves = kWriteThreads / 64;

__global__ __launch_bounds__(kWriteThreads) void preload_write_kernel(IngestArgs a) {
  __shared__ int64_t wave_tot[kWriteWaves];
  const int64_t q = blockIdx.x;
  const int64_t n_out = a.out_off[q + 1] - a.out_off[q];
  if (n_out == 0) return;
  const int64_t b = a.off[q], e = a.off[q + 1];
  const int64_t* ends = a.ends + q * 4;
  const int64_t after = ends[2], before = ends[3];
  const int32_t klo = a.keys[q * 2 * kRanges + 4], khi = a.keys[q * 2 * kRanges + 5];
  const float med = a.median[q];
  const float med2 = med * med;                                                   // :54 (single)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t base = a.out_off[q];
  if (threadIdx.x == 0) a.normalizers[q] = (double)med;                           // :51
  // nothing outside [before or first, after or last] is selected
  const int64_t lo = b + (before >= 0 ? before : ends[0]), hi = b + (after >= 0 ? after : ends[1]) + 1;
  constexpr int kWU = GPDLA_INGEST_WRITE_UNROLL;
  for (int64_t c0 = lo; c0 < hi; c0 += kWriteThreads * kWU) {
    float w[kWU], fl[kWU], iv[kWU];
    int32_t am[kWU];
#pragma unroll
    for (int u = 0; u < kWU; ++u) {                                               // every column's loads first
      const int64_t i = c0 + u * kWriteThreads + threadIdx.x;
      const bool ok = i < hi;
      w[u] = ok ? a.loglam[i] : 0.0f;
      fl[u] = ok ? a.flux[i] : 0.0f;
      iv[u] = ok ? a.ivar[i] : 0.0f;
      am[u] = ok ? a.and_mask[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kWU; ++u) {
      const int64_t cu = c0 + u * kWriteThreads;
      if (cu >= hi) break;                                                        // block-uniform
      const int64_t i = cu + threadIdx.x;
      bool sel = false;
      if (i < hi) {
        const int64_t j = i - b;
        const int32_t k = order_key(w[u]);
        sel = j == after || j == before || (k >= klo && k < khi && !isnan(w[u]));
      }
      const uint64_t bal = __ballot(sel);
      const int before_me = __popcll(bal & ((1ull << lane) - 1));
      __syncthreads();
      if (lane == 0) wave_tot[wave] = __popcll(bal);
      __syncthreads();
      int64_t wo = 0;
      for (int k = 0; k < wave; ++k) wo += wave_tot[k];
      if (sel) {
        const int64_t o = base + wo + before_me;
        a.w_out[o] = wavelength(w[u]);                                            // :64-67
        a.f_out[o] = fl[u] / med;                                                 // :53
        a.nv_out[o] = (1.0f / iv[u]) / med2;                                      // read_spec.m:31, :54
        a.m_out[o] = iv[u] == 0.0f || ((am[u] >> (a.p.brightsky_bit - 1)) & 1);   // read_spec.m:36-38
      }
#pragma unroll
      for (int k = 0; k < kWriteWaves; ++k) base += wave_tot[k];
    }
  }
}

__global__ void read_spec_kernel(int64_t n, const float* loglam, const float* ivar, const int32_t* and_mask,
                                 int32_t brightsky_bit, float* w, float* nv, uint8_t* mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  w[i] = wavelength(loglam[i]);                                                   // read_spec.m:28
  nv[i] = 1.0f / ivar[i];                                                         // :31
  mask[i] = ivar[i] == 0.0f || ((and_mask[i] >> (brightsky_bit - 1)) & 1);        // :36-38
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace
}  // namespace gpdla

using namespace gpdla;

extern "C" {

int gpdla_read_spec_f32(int32_t device, int64_t n, const float* loglam, const float* ivar, const int32_t* and_mask,
                        float* wavelengths, float* noise_variance, uint8_t* pixel_mask) {
  if (n < 0 || (n > 0 && (!loglam || !ivar || !and_mask || !wavelengths || !noise_variance || !pixel_mask)))
    return set_error(GPDLA_EINVAL, "read_spec: null argument or negative length");
  if (int rc = check_device(device)) return rc;
  launch_times().reset();
  if (n == 0) return GPDLA_OK;
  HIP_TRY(hipSetDevice(device));
  DevBuf d_in, d_out;
  HIP_TRY(hipMalloc(&d_in.p, (size_t)n * 12));
  HIP_TRY(hipMalloc(&d_out.p, (size_t)n * 9));
  char* in = (char*)d_in.p;
  char* out = (char*)d_out.p;
  HIP_TRY(hipMemcpy(in, loglam, (size_t)n * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(in + n * 4, ivar, (size_t)n * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(in + n * 8, and_mask, (size_t)n * 4, hipMemcpyHostToDevice));
  launch_times().before();
  read_spec_kernel<<<(unsigned)((n + 255) / 256), 256>>>(n, (const float*)in, (const float*)(in + n * 4),
                                                         (const int32_t*)(in + n * 8), 24, (float*)out,
                                                         (float*)(out + n * 4), (uint8_t*)(out + n * 8));
  launch_times().after();
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(wavelengths, out, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(noise_variance, out + n * 4, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(pixel_mask, out + n * 8, (size_t)n, hipMemcpyDeviceToHost));
  launch_times().finish();
  return GPDLA_OK;
}

int gpdla_preload_qsos_f32(int32_t device, int64_t num_quasars, const int64_t* offsets, const float* flux,
                           const float* loglam, const float* ivar, const int32_t* and_mask, const double* z_qsos,
                           const gpdla_preload_params* params, uint8_t* filter_flags, int64_t* out_offsets,
                           float* out_wavelengths, float* out_flux, float* out_noise_variance,
                           uint8_t* out_pixel_mask, double* normalizers, float* medians) {
  if (num_quasars < 0 || !offsets || !params || !filter_flags || !out_offsets || !normalizers)
    return set_error(GPDLA_EINVAL, "preload_qsos: null argument");
  const int64_t Q = num_quasars, N = Q ? offsets[Q] : 0;
  if (N > 0 && (!flux || !loglam || !ivar || !and_mask || !out_wavelengths || !out_flux || !out_noise_variance ||
                !out_pixel_mask))
    return set_error(GPDLA_EINVAL, "preload_qsos: null pixel array");
  if (Q > 0 && !z_qsos) return set_error(GPDLA_EINVAL, "preload_qsos: null z_qsos");
  if (Q > 0 && offsets[0] != 0) return set_error(GPDLA_EINVAL, "preload_qsos: offsets[0] must be 0");
  for (int64_t q = 0; q < Q; ++q)
    if (offsets[q + 1] < offsets[q]) return set_error(GPDLA_EINVAL, "preload_qsos: offsets decrease at %lld", (long long)q);
  if (params->brightsky_bit < 1 || params->brightsky_bit > 32)
    return set_error(GPDLA_EINVAL, "preload_qsos: brightsky_bit %d outside 1..32", (int)params->brightsky_bit);
  if (int rc = check_device(device)) return rc;
  launch_times().reset();
  out_offsets[0] = 0;
  if (Q == 0) return GPDLA_OK;
  HIP_TRY(hipSetDevice(device));
  DevBuf d_off, d_pix, d_z, d_fl, d_res, d_ooff, d_out;
  HIP_TRY(hipMalloc(&d_off.p, (size_t)(Q + 1) * 8));
  HIP_TRY(hipMalloc(&d_pix.p, (size_t)N * 16 + 16));
  HIP_TRY(hipMalloc(&d_z.p, (size_t)Q * 8));
  HIP_TRY(hipMalloc(&d_fl.p, (size_t)Q * 2));
  HIP_TRY(hipMalloc(&d_res.p, (size_t)Q * 72));
  HIP_TRY(hipMalloc(&d_ooff.p, (size_t)(Q + 1) * 8));
  char* pix = (char*)d_pix.p;
  HIP_TRY(hipMemcpy(d_off.p, offsets, (size_t)(Q + 1) * 8, hipMemcpyHostToDevice));
  if (N > 0) {
    HIP_TRY(hipMemcpy(pix, flux, (size_t)N * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(pix + N * 4, loglam, (size_t)N * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(pix + N * 8, ivar, (size_t)N * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(pix + N * 12, and_mask, (size_t)N * 4, hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(d_z.p, z_qsos, (size_t)Q * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d_fl.p, filter_flags, (size_t)Q, hipMemcpyHostToDevice));
  char* res = (char*)d_res.p;
  IngestArgs a{};
  a.Q = Q;
  a.off = (const int64_t*)d_off.p;
  a.flux = (const float*)pix;
  a.loglam = (const float*)(pix + N * 4);
  a.ivar = (const float*)(pix + N * 8);
  a.and_mask = (const int32_t*)(pix + N * 12);
  a.z = (const double*)d_z.p;
  a.flags_in = (const uint8_t*)d_fl.p;
  a.flags_out = (uint8_t*)d_fl.p + Q;
  a.p = *params;
  a.median = (float*)res;
  a.count = (int64_t*)(res + Q * 8);           // 8-byte aligned: Q * 4 rounded by the 2x below
  a.ends = (int64_t*)(res + Q * 16);
  a.keys = (int32_t*)(res + Q * 48);
  // (median at [0, 4Q), count at [8Q, 16Q), ends at [16Q, 48Q), keys at [48Q, 72Q))
  launch_times().before();
  preload_keys_kernel<<<(unsigned)((Q + kKeySpectraPerBlock - 1) / kKeySpectraPerBlock), 64 * kKeySpectraPerBlock>>>(a);
  launch_times().after();
  HIP_TRY(hipGetLastError());
  launch_times().before();
  preload_scan_kernel<<<(unsigned)Q, kIngestThreads>>>(a);
  launch_times().after();
  HIP_TRY(hipGetLastError());
  std::vector<int64_t> count(Q);
  HIP_TRY(hipMemcpy(count.data(), a.count, (size_t)Q * 8, hipMemcpyDeviceToHost));
  for (int64_t q = 0; q < Q; ++q) out_offsets[q + 1] = out_offsets[q] + count[q];
  const int64_t M = out_offsets[Q];
  HIP_TRY(hipMemcpy(d_ooff.p, out_offsets, (size_t)(Q + 1) * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&d_out.p, (size_t)M * 13 + (size_t)Q * 8 + 16));
  char* out = (char*)d_out.p;
  a.out_off = (const int64_t*)d_ooff.p;
  a.w_out = (float*)out;
  a.f_out = (float*)(out + M * 4);
  a.nv_out = (float*)(out + M * 8);
  a.normalizers = (double*)(out + M * 12 + ((8 - (M * 12) % 8) % 8));
  a.m_out = (uint8_t*)a.normalizers + Q * 8;
  HIP_TRY(hipMemset(a.normalizers, 0, (size_t)Q * 8));                           // zeros(num_quasars, 1)
  launch_times().before();
  preload_write_kernel<<<(unsigned)Q, kWriteThreads>>>(a);
  launch_times().after();
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(filter_flags, a.flags_out, (size_t)Q, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(normalizers, a.normalizers, (size_t)Q * 8, hipMemcpyDeviceToHost));
  if (medians) HIP_TRY(hipMemcpy(medians, a.median, (size_t)Q * 4, hipMemcpyDeviceToHost));
  if (M > 0) {
    HIP_TRY(hipMemcpy(out_wavelengths, a.w_out, (size_t)M * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out_flux, a.f_out, (size_t)M * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out_noise_variance, a.nv_out, (size_t)M * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out_pixel_mask, a.m_out, (size_t)M, hipMemcpyDeviceToHost));
  }
  launch_times().finish();
  return GPDLA_OK;
}

}  // extern "C"
