// Spectrum ingest on gfx950: read_spec.m's derived columns and preload_qsos.m's numeric
// stage, batched over a CSR of the catalogue's spectra (FITS parsing stays on the host).
//
//   read_spec.m:27-28   wavelengths = 10.^loglam     single, rounded once: (float)pow(10.0, (double)loglam)
//                                                   -- the correctly rounded single over every float32
//                                                   loglam in [3.5, 4.1] (checked exhaustively against
//                                                   extended precision); MATLAB's own single pow is
//                                                   unpinned at the last ulp
//   read_spec.m:30-31   noise_variance = 1 ./ ivar   single IEEE division
//   read_spec.m:36-38   pixel_mask = ivar == 0 | bitget(and_mask, 24)
//   preload_qsos.m:19-21  entries with filter_flags > 0 are skipped (empty cells)
//   preload_qsos.m:26     rest = wavelengths / (1 + z)  (single: the double 1 + z rounded to single)
//   preload_qsos.m:29-33  nanmedian of the flux over unmasked pixels with rest in [1310, 1325]: the
//                         window's values gathered in LDS, NaNs dropped, bitonic-sorted, MATLAB's
//                         median (meanof(a, b) = a + (b - a) / 2 for finite same-sign a, b)
//   preload_qsos.m:36-49  bit 3 (value 4) when that median is NaN; bit 4 (value 8) when fewer than
//                         min_num_pixels unmasked pixels have rest in [911.75, 1215.75]
//   preload_qsos.m:51-54  normaliser; flux / median, noise_variance / median^2 (single)
//   preload_qsos.m:56-62  the loading range [910, 1217] plus the first unmasked pixel after its last
//                         and the last unmasked pixel before its first
//   preload_qsos.m:64-67  the selected pixels, in order (a block-wide ordered compaction)
//
// One 256-thread block per spectrum in each of two launches: the first finds the median, the flags,
// the loading range's ends and neighbours and the cell length; the host turns the lengths into CSR
// offsets; the second writes the cells (an order-preserving compaction: the selection is a mask, as in
// the reference, not assumed contiguous).  HBM-bound elementwise work: the input columns are read twice
// (16 B per pixel each time) and ~13 B per selected pixel written.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/gpdla.h"
#include "internal.h"

namespace gpdla {
namespace {

constexpr int kIngestThreads = 256;
constexpr int kWindowCap = 4096;            // normalisation-window values per spectrum held in LDS

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
  int32_t* status;                          // 1: a normalisation window over kWindowCap values
  // pass-2 outputs
  const int64_t* out_off;                   // [Q + 1]
  float* w_out;
  float* f_out;
  float* nv_out;
  uint8_t* m_out;
  double* normalizers;
};

struct PixelView {
  float w, nv, rest;
  bool mask;
};

__device__ inline PixelView pixel(const IngestArgs& a, int64_t i, float one_pz) {
  PixelView v;
  v.w = (float)pow(10.0, (double)a.loglam[i]);                                  // read_spec.m:28
  v.nv = 1.0f / a.ivar[i];                                                        // :31
  v.mask = a.ivar[i] == 0.0f || ((a.and_mask[i] >> (a.p.brightsky_bit - 1)) & 1); // :36-38
  v.rest = v.w / one_pz;                                                          // preload_qsos.m:26
  return v;
}

__device__ inline bool in_range(float r, double lo, double hi) { return (double)r >= lo && (double)r <= hi; }

template <typename T, typename Op>
__device__ inline T block_reduce(T v, T* red, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return op(op(red[0], red[1]), op(red[2], red[3]));
}

__global__ __launch_bounds__(kIngestThreads) void preload_scan_kernel(IngestArgs a) {
  __shared__ float win[kWindowCap];
  __shared__ int nwin;
  __shared__ int64_t red64[4];
  __shared__ int32_t red32[4];
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
  const float one_pz = (float)(1.0 + a.z[q]);
  int32_t nrange = 0;
  int64_t nload = 0, first = LLONG_MAX, last = -1;
  for (int64_t i = b + threadIdx.x; i < e; i += kIngestThreads) {
    const PixelView v = pixel(a, i, one_pz);
    const float fl = a.flux[i];
    if (!v.mask && in_range(v.rest, a.p.normalization_min_lambda, a.p.normalization_max_lambda) && !isnan(fl)) {
      const int slot = atomicAdd(&nwin, 1);                                      // :29-33 (order: sorted below)
      if (slot < kWindowCap) win[slot] = fl;
    }
    nrange += !v.mask && in_range(v.rest, a.p.min_lambda, a.p.max_lambda);       // :41-43
    if (in_range(v.rest, a.p.loading_min_lambda, a.p.loading_max_lambda)) {     // :56-57
      ++nload;
      first = min(first, i - b);
      last = max(last, i - b);
    }
  }
  nrange = block_reduce(nrange, red32, [](int32_t x, int32_t y) { return x + y; });
  nload = block_reduce(nload, red64, [](int64_t x, int64_t y) { return x + y; });
  first = block_reduce(first, red64, [](int64_t x, int64_t y) { return x < y ? x : y; });
  last = block_reduce(last, red64, [](int64_t x, int64_t y) { return x > y ? x : y; });
  __syncthreads();
  const int n = nwin;
  if (n > kWindowCap) {
    if (threadIdx.x == 0) {
      atomicOr(a.status, 1);
      a.flags_out[q] = flags;
      a.count[q] = 0;
    }
    return;
  }
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
  float med = NAN;                                                                // median.m of an empty set
  if (n > 0) {
    if (n & 1) {
      med = win[n / 2];
    } else {                                                                      // median.m's meanof(a, b)
      const float lo = win[n / 2 - 1], hi = win[n / 2];
      const int slo = (lo > 0.0f) - (lo < 0.0f), shi = (hi > 0.0f) - (hi < 0.0f);   // MATLAB sign
      med = (slo == shi && isfinite(lo) && isfinite(hi)) ? lo + (hi - lo) / 2.0f : (lo + hi) / 2.0f;
    }
  }
  // the loading range's unmasked neighbours (:60-62)
  int64_t after = LLONG_MAX, before = -1;
  if (last >= 0) {
    for (int64_t i = b + threadIdx.x; i < e; i += kIngestThreads) {
      const int64_t j = i - b;
      if (j > last || j < first) {
        const PixelView v = pixel(a, i, one_pz);
        if (!v.mask && !in_range(v.rest, a.p.loading_min_lambda, a.p.loading_max_lambda)) {
          if (j > last) after = min(after, j);
          if (j < first) before = max(before, j);
        }
      }
    }
  }
  after = block_reduce(after, red64, [](int64_t x, int64_t y) { return x < y ? x : y; });
  before = block_reduce(before, red64, [](int64_t x, int64_t y) { return x > y ? x : y; });
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

__global__ __launch_bounds__(kIngestThreads) void preload_write_kernel(IngestArgs a) {
  __shared__ int64_t wave_tot[4];
  const int64_t q = blockIdx.x;
  const int64_t n_out = a.out_off[q + 1] - a.out_off[q];
  if (n_out == 0) return;
  const int64_t b = a.off[q], e = a.off[q + 1];
  const int64_t* ends = a.ends + q * 4;
  const int64_t after = ends[2], before = ends[3];
  const float one_pz = (float)(1.0 + a.z[q]);
  const float med = a.median[q];
  const float med2 = med * med;                                                   // :54 (single)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t base = a.out_off[q];
  if (threadIdx.x == 0) a.normalizers[q] = (double)med;                           // :51
  for (int64_t c0 = b; c0 < e; c0 += kIngestThreads) {
    const int64_t i = c0 + threadIdx.x;
    bool sel = false;
    PixelView v{};
    if (i < e) {
      v = pixel(a, i, one_pz);
      const int64_t j = i - b;
      sel = in_range(v.rest, a.p.loading_min_lambda, a.p.loading_max_lambda) || j == after || j == before;
    }
    const uint64_t bal = __ballot(sel);
    const int before_me = __popcll(bal & ((1ull << lane) - 1));
    __syncthreads();
    if (lane == 0) wave_tot[wave] = __popcll(bal);
    __syncthreads();
    int64_t wo = 0;
    for (int w = 0; w < wave; ++w) wo += wave_tot[w];
    if (sel) {
      const int64_t o = base + wo + before_me;
      a.w_out[o] = v.w;                                                           // :64-67
      a.f_out[o] = a.flux[i] / med;                                               // :53
      a.nv_out[o] = v.nv / med2;                                                  // :54
      a.m_out[o] = v.mask;
    }
    base += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
  }
}

__global__ void read_spec_kernel(int64_t n, const float* loglam, const float* ivar, const int32_t* and_mask,
                                 int32_t brightsky_bit, float* w, float* nv, uint8_t* mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  w[i] = (float)pow(10.0, (double)loglam[i]);                                     // read_spec.m:28
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
  read_spec_kernel<<<(unsigned)((n + 255) / 256), 256>>>(n, (const float*)in, (const float*)(in + n * 4),
                                                         (const int32_t*)(in + n * 8), 24, (float*)out,
                                                         (float*)(out + n * 4), (uint8_t*)(out + n * 8));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(wavelengths, out, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(noise_variance, out + n * 4, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(pixel_mask, out + n * 8, (size_t)n, hipMemcpyDeviceToHost));
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
  out_offsets[0] = 0;
  if (Q == 0) return GPDLA_OK;
  HIP_TRY(hipSetDevice(device));
  DevBuf d_off, d_pix, d_z, d_fl, d_res, d_status, d_ooff, d_out;
  HIP_TRY(hipMalloc(&d_off.p, (size_t)(Q + 1) * 8));
  HIP_TRY(hipMalloc(&d_pix.p, (size_t)N * 16 + 16));
  HIP_TRY(hipMalloc(&d_z.p, (size_t)Q * 8));
  HIP_TRY(hipMalloc(&d_fl.p, (size_t)Q * 2));
  HIP_TRY(hipMalloc(&d_res.p, (size_t)Q * (4 + 8 + 32 + 8)));
  HIP_TRY(hipMalloc(&d_status.p, 4));
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
  HIP_TRY(hipMemset(d_status.p, 0, 4));
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
  a.status = (int32_t*)d_status.p;
  // (median at [0, 4Q), count at [8Q, 16Q), ends at [16Q, 48Q) within the Q * 52-byte block)
  preload_scan_kernel<<<(unsigned)Q, kIngestThreads>>>(a);
  HIP_TRY(hipGetLastError());
  std::vector<int64_t> count(Q);
  int32_t status = 0;
  HIP_TRY(hipMemcpy(count.data(), a.count, (size_t)Q * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&status, d_status.p, 4, hipMemcpyDeviceToHost));
  if (status & 1)
    return set_error(GPDLA_EUNSUPPORTED, "preload_qsos: a normalisation window holds more than %d pixels", kWindowCap);
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
  preload_write_kernel<<<(unsigned)Q, kIngestThreads>>>(a);
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
  return GPDLA_OK;
}

}  // extern "C"
