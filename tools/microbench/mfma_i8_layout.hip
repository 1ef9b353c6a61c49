// Verify the v_mfma_i32_32x32x32_i8 operand/accumulator lane maps assumed by the Poly1305
// MFMA design: lane l (r = l&31, h = l>>5) holds A[r][16h + j] and B[16h + j][r] in byte j of
// its 16-byte operand; D[row][col] with col = l&31, row = (i&3) + 8(i>>2) + 4h in acc i.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __host__ int8_t aval(int m, int k) { return (int8_t)(((m * 37 + k * 11) % 255) - 127); }
__device__ __host__ int8_t bval(int k, int n) { return (int8_t)(((k * 53 + n * 29 + 7) % 251) - 125); }

__global__ void k(int* out) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) { a[j] = aval(r, 16 * h + j); b[j] = bval(16 * h + j, r); }
  v4i A, B;
  for (int w = 0; w < 4; w++) {
    A[w] = (uint8_t)a[4*w] | ((uint8_t)a[4*w+1] << 8) | ((uint8_t)a[4*w+2] << 16) | ((uint32_t)(uint8_t)a[4*w+3] << 24);
    B[w] = (uint8_t)b[4*w] | ((uint8_t)b[4*w+1] << 8) | ((uint8_t)b[4*w+2] << 16) | ((uint32_t)(uint8_t)b[4*w+3] << 24);
  }
  v16i C = {};
  C = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, C, 0, 0, 0);
  for (int i = 0; i < 16; i++) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h, col = r;
    out[row * 32 + col] = C[i];
  }
}

int main() {
  int* d; (void)hipMalloc(&d, 32 * 32 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[1024]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < 32; m++)
    for (int n = 0; n < 32; n++) {
      int s = 0;
      for (int kk = 0; kk < 32; kk++) s += aval(m, kk) * bval(kk, n);
      if (s != h[m * 32 + n]) { if (bad < 5) printf("mismatch m=%d n=%d got %d want %d\n", m, n, h[m*32+n], s); bad++; }
    }
  printf("mfma_i32_32x32x32_i8 layout check: %s (%d mismatches) err=%s\n", bad ? "FAIL" : "OK", bad,
         hipGetErrorString(hipGetLastError()));
  return bad != 0;
}
