// Probe: does rocBLAS run an int8 x int8 -> int32 GEMM at int8-MFMA rates on gfx950?
// (Input for the next-round plan: an Ozaki-sliced, exact fp64-class panel-GEMM path.)
// C (M x N, int32) = A^T (M x K, int8) * B (K x N, int8), the panel-GEMM shapes (M = Gram
// entries, N = samples, K = slots x slice pairs).  Also times rocblas_dgemm on the same M, N,
// K / pairs for comparison.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != 0) { printf("%s failed (%d) line %d\n", #x, (int)e_, __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 256;
  const int N = argc > 2 ? atoi(argv[2]) : 16384;
  const int K = argc > 3 ? atoi(argv[3]) : 832 * 15;
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  int8_t *A, *B;
  int32_t* C;
  CK(hipMalloc(&A, (size_t)M * K));
  CK(hipMalloc(&B, (size_t)K * N));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  std::vector<int8_t> ha((size_t)M * K), hb((size_t)K * N);
  for (auto& v : ha) v = (int8_t)(rand() % 255 - 127);
  for (auto& v : hb) v = (int8_t)(rand() % 255 - 127);
  CK(hipMemcpy(A, ha.data(), ha.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), hb.size(), hipMemcpyHostToDevice));
  const int32_t alpha = 1, beta = 0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int trans = 0; trans < 2; ++trans) {
    // A stored K x M (lda = K) and used transposed; B K x N (ldb = K)
    auto run = [&]() {
      return rocblas_gemm_ex(h, trans ? rocblas_operation_transpose : rocblas_operation_none,
                             rocblas_operation_none, M, N, K, &alpha, A, rocblas_datatype_i8_r,
                             trans ? K : M, B, rocblas_datatype_i8_r, K, &beta, C, rocblas_datatype_i32_r, M, C,
                             rocblas_datatype_i32_r, M, rocblas_datatype_i32_r, rocblas_gemm_algo_standard, 0, 0);
    };
    rocblas_status st = run();
    if (st != rocblas_status_success) {
      printf("int8 gemm_ex trans=%d: status %s\n", trans, rocblas_status_to_string(st));
      continue;
    }
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) run();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("int8 gemm_ex transA=%d M=%d N=%d K=%d: %.3f ms, %.0f TOPS\n", trans, M, N, K, ms,
           2.0 * M * N * K / (ms * 1e-3) / 1e12);
  }
  // dgemm on K / 15 for comparison (the f64 panel GEMM)
  const int Kd = K / 15;
  double *dA, *dB, *dC;
  CK(hipMalloc(&dA, (size_t)M * Kd * 8));
  CK(hipMalloc(&dB, (size_t)Kd * N * 8));
  CK(hipMalloc(&dC, (size_t)M * N * 8));
  hipMemset(dA, 0, (size_t)M * Kd * 8);
  hipMemset(dB, 0, (size_t)Kd * N * 8);
  const double one = 1, zero = 0;
  CK(rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, M, N, Kd, &one, dA, Kd, dB, Kd, &zero, dC, M));
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r)
    rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, M, N, Kd, &one, dA, Kd, dB, Kd, &zero, dC, M);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  printf("dgemm M=%d N=%d K=%d: %.3f ms, %.1f TFLOPS\n", M, N, Kd, ms, 2.0 * M * N * Kd / (ms * 1e-3) / 1e12);
  return 0;
}
