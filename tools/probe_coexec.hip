// Probe: do fp64 MFMA and fp64 VALU from DIFFERENT waves on one SIMD overlap?
// 512-thread blocks (8 waves, 2 per SIMD): waves 0-3 run role R0, waves 4-7 role R1.
// role 0 = idle, 1 = MFMA f64 4x4x4 chain x8, 2 = VALU f64 FMA chains x8, 3 = VALU int32 chains x8
// (16 v_xad/v_add-class ops per iteration), 4 = VALU f32 FMA chains x8 (16 per iteration).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void probe(double* out, int iters, int r0, int r1, unsigned long long* cyc) {
  const int wave = threadIdx.x >> 6;
  const int role = wave < 4 ? r0 : r1;
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = i * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (role == 1) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
    }
  } else if (role == 2) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { acc[i] = fma(acc[i], a, b); acc[i] = fma(acc[i], b, a); }
    }
  } else if (role == 3) {
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x * 7u + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { u[i] = (u[i] ^ 0x9e3779b9u) + (unsigned)it; u[i] = (u[i] << 3) ^ (u[i] >> 5); }
    }
    for (int i = 0; i < 8; ++i) acc[i] += (double)u[i];
  } else if (role == 4) {
    float f[8];
    const float fa = 1.0f + threadIdx.x * 1e-7f, fb = 1.0f - threadIdx.x * 1e-7f;
    for (int i = 0; i < 8; ++i) f[i] = i * 1e-3f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { f[i] = fmaf(f[i], fa, fb); f[i] = fmaf(f[i], fb, fa); }
    }
    for (int i = 0; i < 8; ++i) acc[i] += f[i];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) cyc[wave] = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  const int blocks = 256;
  hipMalloc(&out, blocks * 512 * 8); hipMalloc(&cyc, 8 * 8);
  const int iters = 4000;
  struct C { int r0, r1; const char* name; } cs[] = {
      {1, 0, "MFMA x1 wave/SIMD"}, {1, 1, "MFMA x2 waves/SIMD"}, {2, 0, "VALU x1 wave/SIMD"},
      {2, 2, "VALU x2 waves/SIMD"}, {1, 2, "MFMA wave + VALU wave"}, {3, 0, "INT x1 wave/SIMD"},
      {1, 3, "MFMA wave + INT wave"}, {4, 0, "F32 x1 wave/SIMD"}, {1, 4, "MFMA wave + F32 wave"}};
  for (auto& c : cs) {
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(512), 0, 0, out, iters, c.r0, c.r1, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(512), 0, 0, out, iters, c.r0, c.r1, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[8]; hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
    // per-wave work: MFMA role 8*iters mfma (512 flop each... 4x4x4x4 blocks = 256 FMA = 512 flop)
    printf("%-24s %8.3f ms  wave0 %llu cyc  wave4 %llu cyc  (per inner iter: w0 %.1f, w4 %.1f)\n", c.name, ms,
           h[0], h[4], (double)h[0] / iters, (double)h[4] / iters);
  }
  return 0;
}
