// GP null-model training objective on gfx950: spectrum_loss.m (negative log likelihood of one
// centred rest-frame spectrum and its gradient wrt M, log omega, log c_0, log tau_0, log beta)
// summed over the training set as objective.m does.
//
// The per-spectrum work is the same Woodbury core as the hot path (B = I + M'D^-1 M, its
// Cholesky, K^-1 y = D^-1 y - D^-1 M B^-1 M'D^-1 y), plus the gradient terms; the identities
//   K^-1 M = D^-1 M B^-1                       (spectrum_loss.m:55, since C M = I - B^-1)
//   diag K^-1 = d^-1 - d^-2 diag(M B^-1 M')    (spectrum_loss.m:59)
// let one block per spectrum produce every term with k x k work per pixel and no n x n object.
// Per-spectrum partial gradients go to a [spectrum][...] buffer that a second kernel sums in
// spectrum order (objective.m:41-57's loop order; deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
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
  const double* log_omega;   // [P] (objective.m:25-26), or nullptr when omega2 is given
  const double* omega2;      // [P] spectrum_loss's omega2 argument directly, or nullptr
  double c_0, tau_0, beta;
  double* part_dM;           // [Q][k][P] per-spectrum dM (column-major per spectrum)
  double* part_dlo;          // [Q][P]
  double* part_s;            // [Q][kObjScalars]
};

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
  p.om2 = a.omega2 ? a.omega2[i] : exp(2 * a.log_omega[i]);     // objective.m:32
  p.tau = a.tau_0 * pow(lya, a.beta);                             // spectrum_loss.m:23
  p.absorb = exp(-p.tau);                                         // :24
  p.sf = 1 - p.absorb + a.c_0;                                    // :27
  p.an = p.om2 * (p.sf * p.sf);                                   // :28
  p.d = nv + p.an;                                                // :30
  return p;
}

// KB: compile-time bound on k (register arrays, unrolled loops); the rank itself is a.k <= KB
template <int KB>
__global__ __launch_bounds__(kObjThreads) void objective_spectrum_kernel(ObjArgs a) {
  extern __shared__ double sm[];
  const int P = a.P, k = a.k;
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.x;
  double* w = sm;              // [P] d^-1 (0 = excluded pixel)
  double* t = w + P;           // [P] D^-1 y, then K^-1 y
  double* B = t + P;           // [k][k]
  double* R = B + k * k;       // [k][k] upper Cholesky factor, then B^-1
  double* v = R + k * k;       // [k] M' D^-1 y
  double* s = v + k;           // [k] B^-1 M' D^-1 y  (= C y)
  double* g = s + k;           // [k] (K^-1 y)' M
  double* red = g + k;         // [8] block reductions
  __shared__ int s_bad;
  const double* y = a.y + q * a.ld;
  const double* lya = a.lya_1pz + q * a.ld;
  const double* nv = a.noise + q * a.ld;
  if (tid == 0) s_bad = 0;

  // pass 1: D^-1 and D^-1 y per pixel; sum log d; n
  double logd = 0.0, cnt = 0.0;
  for (int i = tid; i < P; i += kObjThreads) {
    const double yi = y[i];
    const bool valid = !(yi != yi);                               // objective.m:43 ~isnan
    double wi = 0.0, ti = 0.0;
    if (valid) {
      const PixelTerms p = pixel_terms(a, i, lya[i], nv[i]);
      wi = 1.0 / p.d;                                             // :32
      ti = wi * yi;                                               // :33
      logd += log(p.d);                                           // :44
      cnt += 1.0;
    }
    w[i] = wi;
    t[i] = ti;
  }
  logd = block_sum(logd, red);
  cnt = block_sum(cnt, red);

  // pass 2: B = M' (D^-1 M) + I (:41-42) and v = M' D^-1 y, one entry per thread
  const int ngram = k * (k + 1) / 2;
  for (int e = tid; e < ngram + k; e += kObjThreads) {
    double acc = 0.0;
    if (e < ngram) {
      int r = 0, start = 0;
      while (e >= start + (k - r)) { start += k - r; ++r; }
      const int c = r + (e - start);
      const double* Mr = a.M + (int64_t)r * P;
      const double* Mc = a.M + (int64_t)c * P;
      for (int i = 0; i < P; ++i) acc = fma(Mr[i], Mc[i] * w[i], acc);
      B[r * k + c] = acc + (r == c ? 1.0 : 0.0);
      B[c * k + r] = B[r * k + c];
    } else {
      const int r = e - ngram;
      const double* Mr = a.M + (int64_t)r * P;
      for (int i = 0; i < P; ++i) acc = fma(Mr[i], t[i], acc);
      v[r] = acc;
    }
  }
  __syncthreads();

  // pass 3 (wave 0): upper Cholesky R'R = B (:43), log det, B^-1 = R^-1 R^-T, s = B^-1 v
  if (tid < 64) {
    const int lane = tid;
    for (int r = lane; r < k * k; r += 64) R[r] = B[r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int p = 0; p < k; ++p) {
      const double dpp = R[p * k + p];
      if (!(dpp > 0.0) && lane == 0) s_bad = 1;
      const double rpp = sqrt(dpp);
      __builtin_amdgcn_wave_barrier();
      for (int c = p + 1 + lane; c < k; c += 64) R[p * k + c] /= rpp;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // trailing update R[r][c] -= R[p][r] R[p][c] for p < r <= c
      for (int idx = lane; idx < (k - p - 1) * (k - p - 1); idx += 64) {
        const int r = p + 1 + idx / (k - p - 1), c = p + 1 + idx % (k - p - 1);
        if (c >= r) R[r * k + c] = fma(-R[p * k + r], R[p * k + c], R[r * k + c]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) R[p * k + p] = rpp;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    double ldb = 0.0;
    for (int p = 0; p < k; ++p) ldb += log(R[p * k + p]);
    if (lane == 0) red[6] = 2 * ldb;                              // 2 sum log diag L (:44)
    // column j of B^-1 (lane j, in place in column j of B, which R has replaced): solve
    // R' z = e_j, then R x = z
    if (lane < k) {
      const int j = lane;
      for (int i = 0; i < k; ++i) {
        double acc = (i == j) ? 1.0 : 0.0;
        for (int m = 0; m < i; ++m) acc = fma(-R[m * k + i], B[m * k + j], acc);
        B[i * k + j] = acc / R[i * k + i];
      }
      for (int i = k - 1; i >= 0; --i) {
        double acc = B[i * k + j];
        for (int m = i + 1; m < k; ++m) acc = fma(-R[i * k + m], B[m * k + j], acc);
        B[i * k + j] = acc / R[i * k + i];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < k) {
      double acc = 0.0;
      for (int c = 0; c < k; ++c) acc = fma(B[lane * k + c], v[c], acc);
      s[lane] = acc;                                              // C y (:46-48)
    }
  }
  __syncthreads();
  const double* Bi = B;

  // pass 4: K^-1 y = D^-1 y - D^-1 M (C y) (:48); y' K^-1 y
  double yky = 0.0;
  for (int i = tid; i < P; i += kObjThreads) {
    const double wi = w[i];
    if (wi != 0.0) {
      double ms = 0.0;
      for (int r = 0; r < k; ++r) ms = fma(a.M[(int64_t)r * P + i] * wi, s[r], ms);
      const double ti = t[i] - ms;
      t[i] = ti;
      yky = fma(y[i], ti, yky);
    }
  }
  yky = block_sum(yky, red);  // (its barriers also publish t)

  // pass 5: g = (K^-1 y)' M (:55)
  for (int r = tid; r < k; r += kObjThreads) {
    const double* Mr = a.M + (int64_t)r * P;
    double acc = 0.0;
    for (int i = 0; i < P; ++i) acc = fma(t[i], Mr[i], acc);
    g[r] = acc;
  }
  __syncthreads();

  // pass 6: per pixel u = M_i B^-1, diag K^-1, dM row, d log omega, scalar gradient sums
  double sc0 = 0.0, stau = 0.0, sbeta = 0.0;
  double* dM = a.part_dM + q * (int64_t)k * P;
  double* dlo = a.part_dlo + q * (int64_t)P;
  for (int i = tid; i < P; i += kObjThreads) {
    const double wi = w[i];
    if (wi == 0.0) {
      for (int r = 0; r < k; ++r) dM[(int64_t)r * P + i] = 0.0;
      dlo[i] = 0.0;
      continue;
    }
    double Mi[KB];
#pragma unroll
    for (int r = 0; r < KB; ++r) Mi[r] = r < k ? a.M[(int64_t)r * P + i] : 0.0;
    const double ti = t[i];
    double qd = 0.0;
    for (int c = 0; c < k; ++c) {
      double u = 0.0;
#pragma unroll
      for (int r = 0; r < KB; ++r)
        if (r < k) u = fma(Mi[r], Bi[r * k + c], u);
      // qd += u * M_ic (M_ic = Mi[c], read back from memory: c is a runtime index)
      qd = fma(u, a.M[(int64_t)c * P + i], qd);
      // dM = -(K^-1 y (K^-1 y' M) - K^-1 M), K^-1 M = D^-1 M B^-1 (:54-55)
      dM[(int64_t)c * P + i] = -(ti * g[c] - wi * u);
    }
    const double dk = wi - wi * wi * qd;                          // diag K^-1 (:59)
    const PixelTerms p = pixel_terms(a, i, lya[i], nv[i]);
    dlo[i] = -(p.an * (ti * ti - dk));                            // :62
    const double da0 = a.c_0 * p.om2 * p.sf;                      // :65
    sc0 += -(ti * da0) * ti + dk * da0;                           // :66
    const double da1 = p.om2 * p.sf * p.tau * p.absorb;           // :69
    stau += -(ti * da1) * ti + dk * da1;                          // :70
    const double da2 = da1 * log(lya[i]) * a.beta;                // :73
    sbeta += -(ti * da2) * ti + dk * da2;                         // :74
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
    o[6] = 0.0;
    o[7] = 0.0;
  }
}

// sum the per-spectrum partials in spectrum order into the running totals (objective.m:46-52)
__global__ __launch_bounds__(256) void objective_sum_kernel(int64_t nq, int64_t per, const double* part,
                                                            double* total) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= per) return;
  double acc = total[e];
  for (int64_t q = 0; q < nq; ++q) acc += part[q * per + e];
  total[e] = acc;
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
  double* part_dM = nullptr;  // [batch][k][P]
  double* part_dlo = nullptr;
  double* part_s = nullptr;
  double* tot = nullptr;      // [k P + P + kObjScalars]
};

namespace {

int obj_fail(gpdla_objective* o, int rc) {
  gpdla_objective_destroy(o);
  return rc;
}

size_t obj_shared_bytes(int64_t P, int k) { return (size_t)(2 * P + 2 * k * k + 3 * k + 8) * sizeof(double); }

// one pass over all spectra with the M / log omega / (c_0, tau_0, beta) already in place
int obj_run(gpdla_objective* o, const double* dM_src, const double* lo_src, const double* om2_src,
            double c_0, double tau_0, double beta, double* host_tot) {
  const int64_t P = o->P;
  const int k = o->k;
  const int64_t per_dM = (int64_t)k * P;
  HIP_TRY(hipMemsetAsync(o->tot, 0, (per_dM + P + kObjScalars) * sizeof(double), o->stream));
  const size_t shm = obj_shared_bytes(P, k);
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
    a.log_omega = lo_src;
    a.omega2 = om2_src;
    a.c_0 = c_0;
    a.tau_0 = tau_0;
    a.beta = beta;
    a.part_dM = o->part_dM;
    a.part_dlo = o->part_dlo;
    a.part_s = o->part_s;
    const dim3 grid((unsigned)nq), blk(kObjThreads);
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
             : k <= 24 ? launch(objective_spectrum_kernel<24>)
             : k <= 32 ? launch(objective_spectrum_kernel<32>)
                       : launch(objective_spectrum_kernel<64>);
    if (rc) return rc;
    hipLaunchKernelGGL(objective_sum_kernel, dim3((unsigned)((per_dM + 255) / 256)), dim3(256), 0, o->stream,
                       nq, per_dM, (const double*)o->part_dM, o->tot);
    hipLaunchKernelGGL(objective_sum_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, o->stream,
                       nq, P, (const double*)o->part_dlo, o->tot + per_dM);
    hipLaunchKernelGGL(objective_sum_kernel, dim3(1), dim3(256), 0, o->stream, nq, (int64_t)kObjScalars,
                       (const double*)o->part_s, o->tot + per_dM + P);
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
  (void)hipFree(o->part_dM);
  (void)hipFree(o->part_dlo);
  (void)hipFree(o->part_s);
  (void)hipFree(o->tot);
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
  // spectra per launch: bounded by the partial-gradient buffer (<= 1 GiB)
  const int64_t per = (int64_t)(k + 1) * num_pixels + kObjScalars;
  o->batch = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(num_quasars, 1), (1LL << 27) / per));
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
      hipMalloc(&o->part_dM, (size_t)o->batch * k * num_pixels * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_dlo, (size_t)o->batch * num_pixels * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->part_s, (size_t)o->batch * kObjScalars * sizeof(double)) != hipSuccess ||
      hipMalloc(&o->tot, (size_t)per * sizeof(double)) != hipSuccess)
    return obj_fail(o, set_error(GPDLA_ENOMEM, "objective workspace allocation failed"));
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
