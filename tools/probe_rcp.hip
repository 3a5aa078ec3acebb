// Probe: accuracy of v_rcp_f64 (no Newton step) against IEEE 1/x, and its issue cost vs v_fma_f64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void acc_kernel(unsigned long long seed, int n, unsigned long long* maxulp, double* maxrel) {
  uint64_t s = seed ^ (blockIdx.x * 0x9E3779B97F4A7C15ull + threadIdx.x * 0xBF58476D1CE4E5B9ull);
  unsigned long long mu = 0;
  double mr = 0;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    // x in [1e-30, 1e30]: mantissa random, exponent in [-100, 100]
    const double m = 1.0 + (double)(s >> 12) * 0x1p-52;
    const int e = (int)((s & 255) % 201) - 100;
    const double x = __builtin_ldexp(m, e);
    const double r = __builtin_amdgcn_rcp(x);
    const double ref = 1.0 / x;
    const long long d = (long long)__double_as_longlong(r) - (long long)__double_as_longlong(ref);
    const unsigned long long ad = d < 0 ? -d : d;
    if (ad > mu) mu = ad;
    const double rel = fabs(r - ref) / ref;
    if (rel > mr) mr = rel;
  }
  atomicMax(maxulp, mu);
  // rel as bits (positive doubles order like integers)
  atomicMax((unsigned long long*)maxrel, (unsigned long long)__double_as_longlong(mr));
}

template <int MODE>
__global__ void rate_kernel(double* out, int iters) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = 1.0 + threadIdx.x * 1e-7 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) a[i] = __builtin_amdgcn_rcp(a[i]);
      else a[i] = fma(a[i], 0.999999, 1e-9);
    }
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  unsigned long long* mu; double* mr; double* out;
  hipMalloc(&mu, 8); hipMalloc(&mr, 8); hipMalloc(&out, 1024 * 256 * 8);
  hipMemset(mu, 0, 8); hipMemset(mr, 0, 8);
  acc_kernel<<<1024, 256>>>(12345, 4000, mu, mr);
  unsigned long long hmu; double hmr;
  hipMemcpy(&hmu, mu, 8, hipMemcpyDeviceToHost); hipMemcpy(&hmr, mr, 8, hipMemcpyDeviceToHost);
  printf("v_rcp_f64 vs IEEE 1/x over %d values: max |ulp diff| %llu, max rel err %.3e\n", 1024 * 256 * 4000, hmu, hmr);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) rate_kernel<0><<<2048, 256>>>(out, iters); else rate_kernel<1><<<2048, 256>>>(out, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double inst = 2048.0 * 4 * iters * 8;  // wave instructions
      if (rep) printf("%s: %.3f ms, %.2f wave-instr per SIMD-us (1024 SIMDs)\n", mode == 0 ? "v_rcp_f64" : "v_fma_f64", ms, inst / 1024 / (ms * 1e3));
    }
  }
  return 0;
}
