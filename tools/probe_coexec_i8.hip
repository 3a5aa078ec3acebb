// Probe: do int8 MFMA (v_mfma_i32_16x16x64_i8) and fp64 VALU from DIFFERENT waves on one SIMD
// overlap?  768-thread blocks (12 waves, 3 per SIMD; wave w runs on SIMD w % 4): waves 0-7 (2 per
// SIMD) run role R0, waves 8-11 (1 per SIMD) role R1.
// role 0 = idle, 1 = int8 MFMA 16x16x64 chains x8, 2 = fp64 FMA chains x8 (16 per iteration),
// 3 = int8 MFMA chains x6 + 12 B of LDS reads per MFMA (the B-stationary GEMM's mix)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(768, 1) void probe(double* out, int iters, int r0, int r1, unsigned long long* cyc) {
  __shared__ v4i lds[4096];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int role = wave < 8 ? r0 : r1;
  for (int i = threadIdx.x; i < 4096; i += 768) lds[i] = (v4i){i, i + 1, i + 2, i + 3};
  __syncthreads();
  double s = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (role == 1 || role == 3) {
    v4i a = (v4i){(int)threadIdx.x, 3, 5, 7}, b = (v4i){1, (int)threadIdx.x, 2, 9};
    v4i acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = (v4i){i, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
      if (role == 3) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const v4i bb = lds[(lane + 64 * i + it) & 4095];
          acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bb, acc[i], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
      }
    }
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else if (role == 2) {
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    double acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = i * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { acc[i] = fma(acc[i], a, b); acc[i] = fma(acc[i], b, a); }
    }
    for (int i = 0; i < 8; ++i) s += acc[i];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0 && blockIdx.x == 0) cyc[wave] = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = ncu;
  hipMalloc(&out, (size_t)blocks * 768 * 8); hipMalloc(&cyc, 12 * 8);
  const int iters = 4000;
  struct C { int r0, r1; const char* name; } cs[] = {
      {1, 0, "I8MFMA x2 waves/SIMD"}, {1, 1, "I8MFMA x3 waves/SIMD"}, {0, 2, "F64 VALU x1 wave/SIMD"},
      {1, 2, "I8MFMA x2 + F64 VALU x1"}, {3, 0, "I8MFMA+LDS x2 waves/SIMD"}, {3, 2, "I8MFMA+LDS x2 + F64 x1"}};
  for (auto& c : cs) {
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(768), 0, 0, out, iters, c.r0, c.r1, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(768), 0, 0, out, iters, c.r0, c.r1, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[12]; hipMemcpy(h, cyc, 96, hipMemcpyDeviceToHost);
    // memtime ticks at 100 MHz: per-iteration cost of wave 0 (role R0) and wave 8 (role R1)
    printf("%-28s %8.3f ms  wave0 %8llu  wave8 %8llu ticks  (per iter: w0 %.3f, w8 %.3f)\n", c.name, ms, h[0], h[8],
           (double)h[0] / iters, (double)h[8] / iters);
  }
  return 0;
}
