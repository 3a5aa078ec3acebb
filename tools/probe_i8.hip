// Probe for an int8-MFMA (Ozaki-sliced) Gram contraction on gfx950:
//  1) operand lane maps of v_mfma_i32_16x16x64_i8 (exact integer data, two hypotheses for A/B)
//  2) issue rate of the i8 MFMA (1 and 2 waves/SIMD)
//  3) co-issue: an i8-MFMA wave and an f64-VALU wave on the same SIMD
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

// A: 16 x 64 (row i, k), B: 64 x 16 (k, col j), row-major int8 in global memory.
// Hypothesis h: lane l holds 16 bytes; element e (0..15) of lane l corresponds to
//   h=0: k = 16*(l>>4) + e
//   h=1: k = 8*(l>>4) + (e & 7) + 32*(e >> 3)
__device__ int kmap(int h, int l, int e) {
  return h == 0 ? 16 * (l >> 4) + e : 8 * (l >> 4) + (e & 7) + 32 * (e >> 3);
}

__global__ void layout_kernel(const signed char* A, const signed char* B, int* D, int h) {
  const int l = threadIdx.x;
  v4i a, b;
  signed char* pa = (signed char*)&a;
  signed char* pb = (signed char*)&b;
  for (int e = 0; e < 16; ++e) {
    int k = kmap(h, l, e);
    pa[e] = A[(l & 15) * 64 + k];
    pb[e] = B[k * 16 + (l & 15)];
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  // C/D map (dtype-independent on gfx950): col = l & 15, row = 4*(l>>4) + r
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__global__ __launch_bounds__(512) void rate_kernel(int* out, double* outd, int iters, int r0, int r1,
                                                   unsigned long long* cyc) {
  const int wave = threadIdx.x >> 6;
  const int role = wave < 4 ? r0 : r1;
  v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)threadIdx.x, 13, 17};
  v4i acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (v4i){i, 0, 0, 0};
  double x = 1.0 + threadIdx.x * 1e-9, y = 1.0 - threadIdx.x * 1e-9, dacc[8];
  for (int i = 0; i < 8; ++i) dacc[i] = i * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (role == 1) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
    }
  } else if (role == 2) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { dacc[i] = fma(dacc[i], x, y); dacc[i] = fma(dacc[i], y, x); }
    }
  } else if (role == 3) {  // int32 VALU (digit extraction class of work)
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x * (i + 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { u[i] = __builtin_amdgcn_ubfe(u[i], 3, 7) + (u[i] << 8); u[i] ^= it; }
    }
    for (int i = 0; i < 8; ++i) acc[i][0] += u[i];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
  double sd = 0;
  for (int i = 0; i < 8; ++i) { s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3]; sd += dacc[i]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  outd[blockIdx.x * blockDim.x + threadIdx.x] = sd;
  if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) cyc[wave] = t1 - t0;
}

int main() {
  // ---- 1) layout
  std::vector<signed char> A(16 * 64), B(64 * 16);
  srand(1);
  for (auto& v : A) v = (signed char)(rand() % 255 - 127);
  for (auto& v : B) v = (signed char)(rand() % 255 - 127);
  std::vector<int> ref(256, 0);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 64; ++k) ref[i * 16 + j] += A[i * 64 + k] * B[k * 16 + j];
  signed char *dA, *dB;
  int* dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  for (int h = 0; h < 2; ++h) {
    hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dD, h);
    std::vector<int> D(256);
    hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += D[i] != ref[i];
    printf("layout hypothesis %d: %d / 256 mismatches\n", h, bad);
  }
  // ---- 2,3) rates
  int* out;
  double* outd;
  unsigned long long* cyc;
  const int blocks = 1024;
  hipMalloc(&out, blocks * 512 * 4);
  hipMalloc(&outd, blocks * 512 * 8);
  hipMalloc(&cyc, 8 * 8);
  const int iters = 2000;
  struct C { int r0, r1; const char* name; } cs[] = {
      {1, 0, "i8 MFMA x1 wave/SIMD"}, {1, 1, "i8 MFMA x2 waves/SIMD"}, {2, 0, "f64 VALU x1 wave/SIMD"},
      {2, 2, "f64 VALU x2 waves/SIMD"}, {1, 2, "i8 MFMA wave + f64 VALU wave"},
      {3, 0, "i32 VALU x1 wave/SIMD"}, {1, 3, "i8 MFMA wave + i32 VALU wave"}};
  for (auto& c : cs) {
    hipLaunchKernelGGL(rate_kernel, dim3(blocks), dim3(512), 0, 0, out, outd, iters, c.r0, c.r1, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(rate_kernel, dim3(blocks), dim3(512), 0, 0, out, outd, iters, c.r0, c.r1, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[8];
    hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
    // i8 MFMA: 16*16*64 MAC = 32768 ops each; 8 per iter per wave
    double mfma_waves = (c.r0 == 1 ? 4 : 0) + (c.r1 == 1 ? 4 : 0);
    double tops = mfma_waves * blocks * 8.0 * iters * 32768 / (ms * 1e-3) / 1e12;
    double valu_waves = (c.r0 == 2 ? 4 : 0) + (c.r1 == 2 ? 4 : 0);
    double tf = valu_waves * blocks * 64 * 16.0 * iters * 2 / (ms * 1e-3) / 1e12;
    printf("%-32s %8.3f ms  w0 %.1f cyc/iter  w4 %.1f cyc/iter  i8 %.0f TOPS  f64 %.1f TF\n", c.name, ms,
           (double)h[0] / iters, (double)h[4] / iters, tops, tf);
  }
  return 0;
}
