// Verify v_mfma_i32_16x16x64_i8 lane maps: lane l holds A[l&15][16(l>>4) + j] and
// B[16(l>>4) + j][l&15] in byte j; D[4(l>>4) + i][l&15] in acc i.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __host__ int8_t aval(int m, int k) { return (int8_t)(((m * 37 + k * 11) % 255) - 127); }
__device__ __host__ int8_t bval(int k, int n) { return (int8_t)(((k * 53 + n * 29 + 7) % 251) - 125); }
__global__ void k(int* out) {
  const int l = threadIdx.x, r = l & 15, h = l >> 4;
  v4i A, B;
  for (int w = 0; w < 4; w++) {
    uint32_t a = 0, b = 0;
    for (int e = 0; e < 4; e++) {
      a |= (uint32_t)(uint8_t)aval(r, 16 * h + 4 * w + e) << (8 * e);
      b |= (uint32_t)(uint8_t)bval(16 * h + 4 * w + e, r) << (8 * e);
    }
    A[w] = (int)a; B[w] = (int)b;
  }
  v4i C = {};
  C = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, C, 0, 0, 0);
  for (int i = 0; i < 4; i++) out[(4 * h + i) * 16 + r] = C[i];
}
int main() {
  int* d; (void)hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < 16; m++) for (int n = 0; n < 16; n++) {
    int s = 0; for (int kk = 0; kk < 64; kk++) s += aval(m, kk) * bval(kk, n);
    if (s != h[m * 16 + n]) { if (bad < 5) printf("mismatch %d %d got %d want %d\n", m, n, h[m*16+n], s); bad++; }
  }
  printf("mfma_i32_16x16x64_i8 layout check: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad != 0;
}
