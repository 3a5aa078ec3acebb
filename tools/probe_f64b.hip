// Probe 2: fp64 MFMA vs VALU, concurrency, 4x4x4 form, clock.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0, unsigned long long* clk) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

__global__ __launch_bounds__(256) void mfma4_loop(double* out, int iters, double a0) {
  double acc[8][4];
  typedef double d4_t __attribute__((ext_vector_type(4)));
  d4_t c[8];
  for (int i = 0; i < 8; ++i) c[i] = (d4_t){0,0,0,0};
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i][0], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += c[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  (void)acc;
}

// Mixed: each wave does NACC MFMAs and NF fmas per iteration (independent).
template <int NF>
__global__ __launch_bounds__(256) void mixed_loop(double* out, int iters, double a0) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = a0 + i + threadIdx.x;
  double m = 0.999999, cc = 1e-7;
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < NF; ++f) x[(i + f) & 7] = fma(x[(i + f) & 7], m, cc);
    }
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a0) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = a0 + i + threadIdx.x;
  double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static float timeit(hipEvent_t e0, hipEvent_t e1) { float ms; hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); return ms; }

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  double* out; hipMalloc(&out, 256 * 64 * 256 * sizeof(double));
  unsigned long long* clk; hipMallocManaged(&clk, 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4000;
  for (int bpc : {1, 2, 4, 8}) {
    int blocks = p.multiProcessorCount * bpc;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0); mfma_loop<8><<<blocks, 256>>>(out, iters, 0.5, clk); hipEventRecord(e1);
      float ms = timeit(e0, e1);
      double fl = (double)blocks * 4 * iters * 8 * 2048.0;
      double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;
      if (rep) printf("bpc=%d mfma16 8acc: %.2f TF  (in-kernel clock %.2f GHz, cyc/mfma/wave=%.1f)\n", bpc, fl / ms / 1e9, ghz, (double)clk[0] / (iters * 8));
      hipEventRecord(e0); mfma_loop<16><<<blocks, 256>>>(out, iters / 2, 0.5, clk); hipEventRecord(e1);
      ms = timeit(e0, e1);
      if (rep) printf("bpc=%d mfma16 16acc: %.2f TF\n", bpc, fl / ms / 1e9);
      hipEventRecord(e0); mfma4_loop<<<blocks, 256>>>(out, iters, 0.5); hipEventRecord(e1);
      ms = timeit(e0, e1);
      fl = (double)blocks * 4 * iters * 8 * (4*4*4*2*16.0);
      if (rep) printf("bpc=%d mfma4x4x4: %.2f TF\n", bpc, fl / ms / 1e9);
      hipEventRecord(e0); fma_loop<<<blocks, 256>>>(out, iters * 4, 0.5); hipEventRecord(e1);
      ms = timeit(e0, e1);
      fl = (double)blocks * 256 * iters * 4 * 8 * 2;
      if (rep) printf("bpc=%d valu fma: %.2f TF\n", bpc, fl / ms / 1e9);
      hipEventRecord(e0); mixed_loop<4><<<blocks, 256>>>(out, iters, 0.5); hipEventRecord(e1);
      ms = timeit(e0, e1);
      double flm = (double)blocks * 4 * iters * 8 * 2048.0, flv = (double)blocks * 256 * iters * 8 * 4 * 2;
      if (rep) printf("bpc=%d mixed(8 mfma + 32 fma): %.3f ms mfma %.2f TF + valu %.2f TF\n", bpc, ms, flm / ms / 1e9, flv / ms / 1e9);
      hipEventRecord(e0); mixed_loop<8><<<blocks, 256>>>(out, iters, 0.5); hipEventRecord(e1);
      ms = timeit(e0, e1);
      flv = (double)blocks * 256 * iters * 8 * 8 * 2;
      if (rep) printf("bpc=%d mixed(8 mfma + 64 fma): %.3f ms mfma %.2f TF + valu %.2f TF\n", bpc, ms, flm / ms / 1e9, flv / ms / 1e9);
    }
  }
  return 0;
}
