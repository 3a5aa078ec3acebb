// Throughput probe: fp64 MFMA 16x16x4 and fp64 VALU FMA on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
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

int main() {
  int dev = 0; hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int blocks = p.multiProcessorCount * 8, threads = 256, iters = 4000;
  double* out; hipMalloc(&out, blocks * threads * sizeof(double));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0); mfma_loop<<<blocks, threads>>>(out, iters, 0.5); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * (threads / 64) * iters * 8 * (16.0 * 16 * 4 * 2);
    printf("mfma_f64_16x16x4: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
    hipEventRecord(e0); fma_loop<<<blocks, threads>>>(out, iters * 4, 0.5); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flops = (double)blocks * threads * iters * 4 * 8 * 2;
    printf("valu fma_f64: %.3f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
