// Operand/result lane layout probe for fp64 MFMA forms on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void probe4(unsigned long long* out) {
  int l = threadIdx.x;
  for (int la = 0; la < 64; ++la)
    for (int lb = 0; lb < 64; ++lb) {
      double a = (l == la) ? 1.0 : 0.0, b = (l == lb) ? 1.0 : 0.0;
      double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
      unsigned long long m = __ballot(d != 0.0);
      if (l == 0) out[la * 64 + lb] = m;
    }
}
__global__ void probe16(unsigned long long* out) {
  int l = threadIdx.x;
  for (int la = 0; la < 64; ++la)
    for (int lb = 0; lb < 64; ++lb) {
      double a = (l == la) ? 1.0 : 0.0, b = (l == lb) ? 1.0 : 0.0;
      d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, (d4){0,0,0,0}, 0, 0, 0);
      for (int r = 0; r < 4; ++r) {
        unsigned long long m = __ballot(d[r] != 0.0);
        if (l == 0) out[(la * 64 + lb) * 4 + r] = m;
      }
    }
}
int main() {
  unsigned long long *o4, *o16;
  hipMallocManaged(&o4, 64 * 64 * 8); hipMallocManaged(&o16, 64 * 64 * 4 * 8);
  probe4<<<1, 64>>>(o4); probe16<<<1, 64>>>(o16); hipDeviceSynchronize();
  printf("4x4x4: la lb -> lanes\n");
  for (int la = 0; la < 64; ++la) for (int lb = 0; lb < 64; ++lb) if (o4[la * 64 + lb]) {
    printf("A%d B%d:", la, lb); for (int i = 0; i < 64; ++i) if (o4[la*64+lb] >> i & 1) printf(" %d", i); printf("\n"); }
  printf("16x16x4: la lb -> (reg lane)\n");
  for (int la = 0; la < 64; ++la) for (int lb = 0; lb < 64; ++lb) for (int r = 0; r < 4; ++r) if (o16[(la*64+lb)*4+r]) {
    printf("A%d B%d r%d:", la, lb, r); for (int i = 0; i < 64; ++i) if (o16[(la*64+lb)*4+r] >> i & 1) printf(" %d", i); printf("\n"); }
  return 0;
}
