// generate_dla_samples.m:8-57 on gfx950: the DLA parameter samples every spectrum's
// likelihood sweep is evaluated on.
//
//   :8-9    scramble(haltonset(2), 'rr2')     halton_rr2_kernel: one thread per point, the radical
//                                             inverse digit by digit with each digit through the RR2
//                                             permutation (Kocis & Whiten 1997); MATLAB point 1 is
//                                             index 0 (the origin).  Integer digit work, then the same
//                                             IEEE operations in the same order as the checkers
//                                             (x += perm[d] * f; f /= b; no contraction): bit-exact.
//   :13     offsets = coordinate 1
//   :26-28  the catalogue's column densities  (host: the caller concatenates the non-empty cells)
//   :32-33  ksdensity(log_nhis, x)            kde_kernel: one block per grid point, a fixed-order
//                                             block reduction of the Gaussian kernel over the data, at
//                                             MATLAB's default bandwidth (MAD / 0.6745 (4 / 3n)^(1/5);
//                                             the two medians on the host, O(n) selection).
//   :34     polyfit(x, log(kde), 2)           host: economy Householder QR of the 1000 x 3 Vandermonde
//                                             system, p = R \ (Q' y), as MATLAB solves it.
//   :37-38  Z = integral(exp(polyval), 20, 25)  fit_integral: closed form (an erf difference) for a
//                                             concave fit, composite Gauss-Legendre otherwise.
//   :42-55  fzero(cdf - u_i, 20.5)            inverse_cdf_kernel: one thread per sample, bracketed
//                                             Newton on the mixture CDF to full double precision
//                                             (MATLAB's fzero / integral stop at their default
//                                             tolerances, 1e-6 relative for integral).
//   :57     nhi_samples = 10 .^ log_nhi_samples
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/gpdla.h"
#include "internal.h"

namespace gpdla {
namespace {

constexpr int kMaxHaltonDims = 16;
constexpr int kMaxHaltonBase = 64;
constexpr int kKdeThreads = 256;
constexpr int kFitPoints = 1000;   // generate_dla_samples.m:32

struct HaltonArgs {
  int64_t start, stride, num;
  int32_t dims;
  int32_t bases[kMaxHaltonDims];
  const int32_t* perms;           // [dims][kMaxHaltonBase]
  double* out;                    // [num][dims]
};

__global__ void halton_rr2_kernel(HaltonArgs a) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.num) return;
  const int64_t idx = a.start + j * a.stride;
  for (int d = 0; d < a.dims; ++d) {
    const int64_t b = a.bases[d];
    const int32_t* perm = a.perms + d * kMaxHaltonBase;
    int64_t i = idx;
    double x = 0.0, f = 1.0 / (double)b;
    while (i > 0) {
      const double term = (double)perm[i % b] * f;
      x = x + term;
      i /= b;
      f = f / (double)b;
    }
    a.out[j * a.dims + d] = x;
  }
}

__global__ __launch_bounds__(kKdeThreads) void kde_kernel(const double* data, int64_t n, double x0, double step,
                                                          double x_last, int32_t nx, double h, double* out) {
#pragma clang fp contract(off)
  __shared__ double red[kKdeThreads / 64];
  const int p = blockIdx.x;
  // np.linspace(fit_min, fit_max, 1000): i * step + start, the last point exactly the end
  const double x = p == nx - 1 ? x_last : (double)p * step + x0;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kKdeThreads) {
    const double u = (x - data[i]) / h;
    s += exp(-0.5 * u * u);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = (red[0] + red[1]) + (red[2] + red[3]);
    out[p] = tot / ((double)n * h * 2.5066282746310002);   // sqrt(2 pi)
  }
}

struct Prior {
  double c2, c1, c0;              // polyfit coefficients, highest power first (generate_dla_samples.m:34)
  double Z;                       // :37-38
  double alpha, umin, umax, fmin, fupper;
};

// 20-point Gauss-Legendre nodes / weights on [-1, 1] (the non-concave fit's quadrature; a concave fit,
// the case for any unimodal catalogue, integrates in closed form)
__host__ __device__ inline void gl20(int i, double& x, double& w) {
  // numpy.polynomial.legendre.leggauss(20), the non-negative half
  constexpr double X[10] = {0.07652652113349734, 0.2277858511416451, 0.37370608871541955, 0.5108670019508271,
                            0.636053680726515, 0.7463319064601508, 0.8391169718222188, 0.9122344282513258,
                            0.9639719272779138, 0.9931285991850949};
  constexpr double W[10] = {0.15275338713072578, 0.14917298647260366, 0.14209610931838187, 0.13168863844917653,
                            0.11819453196151825, 0.10193011981724026, 0.08327674157670467, 0.06267204833410944,
                            0.04060142980038622, 0.017614007139153273};
  const int k = i < 10 ? 9 - i : i - 10;
  x = i < 10 ? -X[k] : X[k];
  w = W[k];
}

// integral of exp(c2 t^2 + c1 t + c0) over [a, b] (unnormalized_pdf, generate_dla_samples.m:37)
__host__ __device__ inline double fit_integral(const Prior& p, double a, double b) {
  if (!(b > a)) return 0.0;
  if (p.c2 < 0) {
    const double s = sqrt(-p.c2), m = -p.c1 / (2 * p.c2);
    const double peak = exp(p.c0 - p.c1 * p.c1 / (4 * p.c2));
    return peak * 1.7724538509055159 / (2 * s) * (erf(s * (b - m)) - erf(s * (a - m)));
  }
  constexpr int kPanels = 64;
  const double hw = 0.5 * (b - a) / kPanels;
  double tot = 0.0;
  for (int q = 0; q < kPanels; ++q) {
    const double mid = a + (2 * q + 1) * hw;
    double acc = 0.0;
    for (int i = 0; i < 20; ++i) {
      double x, w;
      gl20(i, x, w);
      const double t = mid + hw * x;
      acc += w * exp((p.c2 * t + p.c1) * t + p.c0);
    }
    tot += acc * hw;
  }
  return tot;
}

// normalized_pdf and cdf (generate_dla_samples.m:42-46)
__host__ __device__ inline double prior_pdf(const Prior& p, double t) {
  const double uni = (t >= p.umin && t <= p.umax) ? 1.0 / (p.umax - p.umin) : 0.0;
  return p.alpha * exp((p.c2 * t + p.c1) * t + p.c0) / p.Z + (1 - p.alpha) * uni;
}

__host__ __device__ inline double prior_cdf(const Prior& p, double t) {
  const double fit = fit_integral(p, p.fmin, t) / p.Z;
  const double lo = p.fmin > p.umin ? p.fmin : p.umin;
  const double uni = t >= lo ? ((t < p.umax ? t : p.umax) - lo) / (p.umax - p.umin) : 0.0;
  return p.alpha * fit + (1 - p.alpha) * uni;
}

__global__ void inverse_cdf_kernel(Prior p, const double* halton, int32_t dims, int32_t coord, int64_t num,
                                   double* log_nhi, double* nhi) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= num) return;
  const double u = halton[j * dims + coord];
  constexpr double eps = 2.220446049250313e-16;
  double lo = p.fmin, hi = p.fupper;
  double t = 20.5 < lo ? lo : (20.5 > hi ? hi : 20.5);   // fzero's start point (:53)
  for (int it = 0; it < 200; ++it) {
    const double g = prior_cdf(p, t) - u;
    if (g <= 0) lo = t;
    else hi = t;
    const double d = prior_pdf(p, t);
    double tn = t - g / d;
    if (!isfinite(tn) || tn <= lo || tn >= hi) tn = 0.5 * (lo + hi);
    const bool done = fabs(tn - t) <= 4 * eps * fabs(t);
    t = tn;
    if (done || hi - lo <= 4 * eps * fabs(hi)) break;
  }
  if (u <= 0) t = p.fmin;
  log_nhi[j] = t;
  nhi[j] = pow(10.0, t);                                    // :57
}

// RR2 digit permutation: the bit-reversed integers 0 .. 2^m - 1 (m = ceil(log2 b)) that are below b
std::vector<int32_t> rr2_perm(int b) {
  int m = 1;
  while ((1 << m) < b) ++m;
  std::vector<int32_t> out;
  for (int i = 0; i < (1 << m); ++i) {
    int r = 0;
    for (int bit = 0; bit < m; ++bit)
      if (i >> bit & 1) r |= 1 << (m - 1 - bit);
    if (r < b) out.push_back(r);
  }
  return out;
}

// numpy / MATLAB median: the middle value, or the mean of the two middle values
double median_of(std::vector<double> v) {
  const size_t n = v.size(), h = n / 2;
  std::nth_element(v.begin(), v.begin() + h, v.end());
  const double hi = v[h];
  if (n % 2) return hi;
  const double lo = *std::max_element(v.begin(), v.begin() + h);
  return (lo + hi) / 2.0;
}

// polyfit(x, y, 2) as MATLAB computes it: economy QR of the Vandermonde matrix [x^2 x 1] by
// Householder reflections, then p = R \ (Q' y)
void polyfit2(const std::vector<double>& x, const std::vector<double>& y, double c[3]) {
  const size_t n = x.size();
  std::vector<double> A(n * 3), b(y);
  for (size_t i = 0; i < n; ++i) {
    A[i * 3 + 0] = x[i] * x[i];
    A[i * 3 + 1] = x[i];
    A[i * 3 + 2] = 1.0;
  }
  double R[3][3] = {};
  for (int j = 0; j < 3; ++j) {
    double nrm = 0.0;
    for (size_t i = j; i < n; ++i) nrm += A[i * 3 + j] * A[i * 3 + j];
    nrm = std::sqrt(nrm);
    const double alpha = A[j * 3 + j] > 0 ? -nrm : nrm;
    std::vector<double> v(n, 0.0);
    for (size_t i = j; i < n; ++i) v[i] = A[i * 3 + j];
    v[j] -= alpha;
    double vv = 0.0;
    for (size_t i = j; i < n; ++i) vv += v[i] * v[i];
    if (vv > 0) {
      for (int k = j; k < 3; ++k) {
        double s = 0.0;
        for (size_t i = j; i < n; ++i) s += v[i] * A[i * 3 + k];
        s = 2.0 * s / vv;
        for (size_t i = j; i < n; ++i) A[i * 3 + k] -= s * v[i];
      }
      double s = 0.0;
      for (size_t i = j; i < n; ++i) s += v[i] * b[i];
      s = 2.0 * s / vv;
      for (size_t i = j; i < n; ++i) b[i] -= s * v[i];
    }
    for (int k = j; k < 3; ++k) R[j][k] = A[j * 3 + k];
  }
  for (int j = 2; j >= 0; --j) {
    double s = b[j];
    for (int k = j + 1; k < 3; ++k) s -= R[j][k] * c[k];
    c[j] = s / R[j][j];
  }
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

int gpdla_halton_rr2_f64(int32_t device, int64_t start, int64_t stride, int64_t num, const int32_t* bases,
                         int32_t dims, double* out) {
  if (!bases || !out || num < 0 || start < 0 || stride < 1 || dims < 1 || dims > kMaxHaltonDims)
    return set_error(GPDLA_EINVAL, "halton: bad arguments (dims 1..%d, start >= 0, stride >= 1)", kMaxHaltonDims);
  for (int d = 0; d < dims; ++d)
    if (bases[d] < 2 || bases[d] > kMaxHaltonBase)
      return set_error(GPDLA_EINVAL, "halton: base %d outside 2..%d", (int)bases[d], kMaxHaltonBase);
  if (int rc = check_device(device)) return rc;
  launch_times().reset();
  if (num == 0) return GPDLA_OK;
  HIP_TRY(hipSetDevice(device));
  HaltonArgs a{};
  a.start = start;
  a.stride = stride;
  a.num = num;
  a.dims = dims;
  std::vector<int32_t> perms((size_t)dims * kMaxHaltonBase, 0);
  for (int d = 0; d < dims; ++d) {
    a.bases[d] = bases[d];
    const auto p = rr2_perm(bases[d]);
    std::copy(p.begin(), p.end(), perms.begin() + (size_t)d * kMaxHaltonBase);
  }
  DevBuf dperm, dout;
  HIP_TRY(hipMalloc(&dperm.p, perms.size() * 4));
  HIP_TRY(hipMalloc(&dout.p, (size_t)num * dims * 8));
  HIP_TRY(hipMemcpy(dperm.p, perms.data(), perms.size() * 4, hipMemcpyHostToDevice));
  a.perms = (const int32_t*)dperm.p;
  a.out = (double*)dout.p;
  launch_times().before();
  halton_rr2_kernel<<<(unsigned)((num + 255) / 256), 256>>>(a);
  launch_times().after();
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(out, dout.p, (size_t)num * dims * 8, hipMemcpyDeviceToHost));
  launch_times().finish();
  return GPDLA_OK;
}

int gpdla_generate_dla_samples_f64(int32_t device, const double* log_nhis, int64_t n_data, int64_t num_samples,
                                   const gpdla_dla_prior* prior, double* offset_samples, double* log_nhi_samples,
                                   double* nhi_samples, double* fit) {
  if (!log_nhis || !prior || !offset_samples || !log_nhi_samples || !nhi_samples || num_samples < 0)
    return set_error(GPDLA_EINVAL, "generate_dla_samples: null argument or negative sample count");
  if (n_data < 2) return set_error(GPDLA_EINVAL, "generate_dla_samples: need at least two catalogue column densities");
  if (!(prior->uniform_max > prior->uniform_min) || !(prior->fit_max > prior->fit_min) ||
      !(prior->fit_upper > prior->fit_min) || !(prior->alpha >= 0 && prior->alpha <= 1))
    return set_error(GPDLA_EINVAL, "generate_dla_samples: bad prior parameters");
  for (int64_t i = 0; i < n_data; ++i)
    if (!std::isfinite(log_nhis[i])) return set_error(GPDLA_EINVAL, "generate_dla_samples: non-finite log_nhis[%lld]", (long long)i);
  if (int rc = check_device(device)) return rc;
  launch_times().reset();
  HIP_TRY(hipSetDevice(device));
  // ksdensity's default bandwidth (host: two O(n) selections)
  std::vector<double> data(log_nhis, log_nhis + n_data);
  const double med = median_of(data);
  std::vector<double> dev(data.size());
  for (size_t i = 0; i < data.size(); ++i) dev[i] = std::fabs(data[i] - med);
  double sig = median_of(dev) / 0.6745;
  if (!(sig > 0)) sig = *std::max_element(data.begin(), data.end()) - *std::min_element(data.begin(), data.end());
  const double h = sig > 0 ? sig * std::pow(4.0 / (3.0 * (double)n_data), 0.2) : 1.0;
  // the KDE on the fit grid and the Halton points on the device
  const double x0 = prior->fit_min, x1 = prior->fit_max, step = (x1 - x0) / (kFitPoints - 1);
  DevBuf ddata, dkde, dhal, dperm, dlog, dnhi;
  HIP_TRY(hipMalloc(&ddata.p, (size_t)n_data * 8));
  HIP_TRY(hipMalloc(&dkde.p, kFitPoints * 8));
  HIP_TRY(hipMemcpy(ddata.p, data.data(), (size_t)n_data * 8, hipMemcpyHostToDevice));
  launch_times().before();
  kde_kernel<<<kFitPoints, kKdeThreads>>>((const double*)ddata.p, n_data, x0, step, x1, kFitPoints, h, (double*)dkde.p);
  launch_times().after();
  HIP_TRY(hipGetLastError());
  std::vector<double> kde(kFitPoints), xs(kFitPoints), ly(kFitPoints);
  HIP_TRY(hipMemcpy(kde.data(), dkde.p, kFitPoints * 8, hipMemcpyDeviceToHost));
  for (int i = 0; i < kFitPoints; ++i) {
    xs[i] = i == kFitPoints - 1 ? x1 : (double)i * step + x0;
    if (!(kde[i] > 0))
      return set_error(GPDLA_ENUMERIC, "generate_dla_samples: the density estimate is 0 at %.6f (log of 0)", xs[i]);
    ly[i] = std::log(kde[i]);
  }
  Prior p{};
  double c[3];
  polyfit2(xs, ly, c);                                                      // :34
  p.c2 = c[0];
  p.c1 = c[1];
  p.c0 = c[2];
  p.alpha = prior->alpha;
  p.umin = prior->uniform_min;
  p.umax = prior->uniform_max;
  p.fmin = prior->fit_min;
  p.fupper = prior->fit_upper;
  p.Z = 1.0;
  p.Z = fit_integral(p, p.fmin, p.fupper);                                  // :37-38
  if (!(p.Z > 0) || !std::isfinite(p.Z))
    return set_error(GPDLA_ENUMERIC, "generate_dla_samples: the fitted density does not normalise (Z = %g)", p.Z);
  if (fit) {
    fit[0] = p.c2;
    fit[1] = p.c1;
    fit[2] = p.c0;
    fit[3] = p.Z;
    fit[4] = h;
  }
  if (num_samples == 0) return GPDLA_OK;
  HaltonArgs a{};
  a.start = 0;
  a.stride = 1;
  a.num = num_samples;
  a.dims = 2;
  a.bases[0] = 2;
  a.bases[1] = 3;
  std::vector<int32_t> perms(2 * kMaxHaltonBase, 0);
  for (int d = 0; d < 2; ++d) {
    const auto q = rr2_perm(a.bases[d]);
    std::copy(q.begin(), q.end(), perms.begin() + d * kMaxHaltonBase);
  }
  HIP_TRY(hipMalloc(&dperm.p, perms.size() * 4));
  HIP_TRY(hipMalloc(&dhal.p, (size_t)num_samples * 2 * 8));
  HIP_TRY(hipMalloc(&dlog.p, (size_t)num_samples * 8));
  HIP_TRY(hipMalloc(&dnhi.p, (size_t)num_samples * 8));
  HIP_TRY(hipMemcpy(dperm.p, perms.data(), perms.size() * 4, hipMemcpyHostToDevice));
  a.perms = (const int32_t*)dperm.p;
  a.out = (double*)dhal.p;
  const unsigned grid = (unsigned)((num_samples + 255) / 256);
  launch_times().before();
  halton_rr2_kernel<<<grid, 256>>>(a);                                       // :8-9
  launch_times().after();
  HIP_TRY(hipGetLastError());
  launch_times().before();
  inverse_cdf_kernel<<<grid, 256>>>(p, (const double*)dhal.p, 2, 1, num_samples, (double*)dlog.p,
                                    (double*)dnhi.p);                        // :51-57
  launch_times().after();
  HIP_TRY(hipGetLastError());
  std::vector<double> hal((size_t)num_samples * 2);
  HIP_TRY(hipMemcpy(hal.data(), dhal.p, hal.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(log_nhi_samples, dlog.p, (size_t)num_samples * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(nhi_samples, dnhi.p, (size_t)num_samples * 8, hipMemcpyDeviceToHost));
  for (int64_t j = 0; j < num_samples; ++j) offset_samples[j] = hal[(size_t)j * 2];   // :13
  launch_times().finish();
  return GPDLA_OK;
}

}  // extern "C"
