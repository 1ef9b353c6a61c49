// Component ceilings on gfx950: Salsa20/20 keystream blocks/s and Poly1305 Horner steps/s
// with everything in registers (no memory traffic).  Variants compare codegen choices.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "xs_salsa_asm.h"

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define QR(a, b, c, d) b ^= rotl(a + d, 7); c ^= rotl(b + a, 9); d ^= rotl(c + b, 13); a ^= rotl(d + c, 18);
__device__ __forceinline__ void rounds(uint32_t (&x)[16]) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]); QR(x[5], x[9], x[13], x[1]); QR(x[10], x[14], x[2], x[6]); QR(x[15], x[3], x[7], x[11]);
    QR(x[0], x[1], x[2], x[3]); QR(x[5], x[6], x[7], x[4]); QR(x[10], x[11], x[8], x[9]); QR(x[15], x[12], x[13], x[14]);
  }
}
__device__ __forceinline__ void rounds_nounroll(uint32_t (&x)[16]) {
#pragma unroll 1
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]); QR(x[5], x[9], x[13], x[1]); QR(x[10], x[14], x[2], x[6]); QR(x[15], x[3], x[7], x[11]);
    QR(x[0], x[1], x[2], x[3]); QR(x[5], x[6], x[7], x[4]); QR(x[10], x[11], x[8], x[9]); QR(x[15], x[12], x[13], x[14]);
  }
}

// V: 0 = 1 block/lane (unrolled), 1 = 2 blocks/lane interleaved, 2 = 1 block/lane rounds not unrolled
template <int V>
__global__ void __launch_bounds__(256) salsa_k(uint32_t* out, const uint32_t* __restrict__ key, int nblk) {
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = key[i];
  uint32_t acc = 0;
  const uint32_t base = (blockIdx.x * 256 + threadIdx.x) * 64;
  if constexpr (V == 1) {
    for (int b = 0; b < nblk; b += 2) {
      uint32_t x[16] = {0x61707865u, k[0], k[1], k[2], k[3], 0x3320646eu, k[5], k[6], base + b, 0, 0x79622d32u, k[4], k[5], k[6], k[7], 0x6b206574u};
      uint32_t y[16] = {0x61707865u, k[0], k[1], k[2], k[3], 0x3320646eu, k[5], k[6], base + b + 1, 0, 0x79622d32u, k[4], k[5], k[6], k[7], 0x6b206574u};
#pragma unroll
      for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]); QR(y[0], y[4], y[8], y[12]); QR(x[5], x[9], x[13], x[1]); QR(y[5], y[9], y[13], y[1]);
        QR(x[10], x[14], x[2], x[6]); QR(y[10], y[14], y[2], y[6]); QR(x[15], x[3], x[7], x[11]); QR(y[15], y[3], y[7], y[11]);
        QR(x[0], x[1], x[2], x[3]); QR(y[0], y[1], y[2], y[3]); QR(x[5], x[6], x[7], x[4]); QR(y[5], y[6], y[7], y[4]);
        QR(x[10], x[11], x[8], x[9]); QR(y[10], y[11], y[8], y[9]); QR(x[15], x[12], x[13], x[14]); QR(y[15], y[12], y[13], y[14]);
      }
      for (int i = 0; i < 16; i++) acc ^= x[i] + y[i];
    }
  } else {
    for (int b = 0; b < nblk; b++) {
      uint32_t x[16] = {0x61707865u, k[0], k[1], k[2], k[3], 0x3320646eu, k[5], k[6], base + b, 0, 0x79622d32u, k[4], k[5], k[6], k[7], 0x6b206574u};
      if constexpr (V == 0) rounds(x); else rounds_nounroll(x);
      for (int i = 0; i < 16; i++) acc ^= x[i] + k[i & 7];
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Same as salsa_k<2> but lane 0 of every workgroup stamps s_memtime / s_memrealtime.
__global__ void __launch_bounds__(256) salsa_clk(uint32_t* out, const uint32_t* __restrict__ key, int nblk,
                                                 unsigned long long* stamps) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = key[i];
  uint32_t acc = 0;
  const uint32_t base = (blockIdx.x * 256 + threadIdx.x) * 64;
  for (int b = 0; b < nblk; b++) {
    uint32_t x[16] = {0x61707865u, k[0], k[1], k[2], k[3], 0x3320646eu, k[5], k[6], base + b, 0, 0x79622d32u, k[4], k[5], k[6], k[7], 0x6b206574u};
    xs_salsa20_rounds_asm(x);
    for (int i = 0; i < 16; i++) acc ^= x[i] + k[i & 7];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { stamps[2 * blockIdx.x] = t1 - t0; stamps[2 * blockIdx.x + 1] = r1 - r0; }
}

// Poly1305 Horner with a wave-uniform multiplier (radix 2^26), as in xs_crypt.
constexpr uint32_t M26 = 0x3ffffff;
__global__ void __launch_bounds__(256) poly_k(uint32_t* out, const uint32_t* __restrict__ rr, int nchunk) {
  uint32_t m[5], s[5];
  for (int i = 0; i < 5; i++) { m[i] = rr[i] & M26; s[i] = m[i] * 5; }
  uint32_t h[5] = {threadIdx.x, 1, 2, 3, 4};
  uint32_t w0 = blockIdx.x, w1 = threadIdx.x * 7, w2 = 99, w3 = 12345;
  for (int c = 0; c < nchunk; c++) {
    w0 += c;
    h[0] += w0 & M26; h[1] += __builtin_amdgcn_alignbit(w1, w0, 26) & M26; h[2] += __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    h[3] += __builtin_amdgcn_alignbit(w3, w2, 14) & M26; h[4] += (w3 >> 8) | (1u << 24);
    uint64_t d0 = (uint64_t)h[0] * m[0] + (uint64_t)h[1] * s[4] + (uint64_t)h[2] * s[3] + (uint64_t)h[3] * s[2] + (uint64_t)h[4] * s[1];
    uint32_t o0 = (uint32_t)d0 & M26;
    uint64_t d1 = (d0 >> 26) + (uint64_t)h[0] * m[1] + (uint64_t)h[1] * m[0] + (uint64_t)h[2] * s[4] + (uint64_t)h[3] * s[3] + (uint64_t)h[4] * s[2];
    uint32_t o1 = (uint32_t)d1 & M26;
    uint64_t d2 = (d1 >> 26) + (uint64_t)h[0] * m[2] + (uint64_t)h[1] * m[1] + (uint64_t)h[2] * m[0] + (uint64_t)h[3] * s[4] + (uint64_t)h[4] * s[3];
    uint32_t o2 = (uint32_t)d2 & M26;
    uint64_t d3 = (d2 >> 26) + (uint64_t)h[0] * m[3] + (uint64_t)h[1] * m[2] + (uint64_t)h[2] * m[1] + (uint64_t)h[3] * m[0] + (uint64_t)h[4] * s[4];
    uint32_t o3 = (uint32_t)d3 & M26;
    uint64_t d4 = (d3 >> 26) + (uint64_t)h[0] * m[4] + (uint64_t)h[1] * m[3] + (uint64_t)h[2] * m[2] + (uint64_t)h[3] * m[1] + (uint64_t)h[4] * m[0];
    uint32_t o4 = (uint32_t)d4 & M26;
    uint32_t cc = (uint32_t)(d4 >> 26);
    o0 += cc * 5; cc = o0 >> 26; o0 &= M26; o1 += cc;
    h[0] = o0; h[1] = o1; h[2] = o2; h[3] = o3; h[4] = o4;
  }
  out[blockIdx.x * 256 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

template <class F> float timeit(F f) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f(); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0); for (int r = 0; r < 3; r++) f(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); return ms / 3;
}

int main() {
  uint32_t *d, *key; (void)hipMalloc(&d, (size_t)100000 * 256 * 4); (void)hipMalloc(&key, 64);
  (void)hipMemset(key, 0x5a, 64);
  const int grid = 100000;  // like 100k crypt blocks; each lane does 4 Salsa blocks = 1024 per WG
  float t0 = timeit([&] { salsa_k<0><<<grid, 256>>>(d, key, 4); });
  float t1 = timeit([&] { salsa_k<1><<<grid, 256>>>(d, key, 4); });
  float t2 = timeit([&] { salsa_k<2><<<grid, 256>>>(d, key, 4); });
  double nb = 100000.0 * 256 * 4;
  printf("err: %s\n", hipGetErrorString(hipGetLastError()));
  printf("salsa 1/lane unrolled : %.3f ms  %.2f GB/s keystream\n", t0, nb * 64 / (t0 * 1e6));
  printf("salsa 2/lane interleav: %.3f ms  %.2f GB/s keystream\n", t1, nb * 64 / (t1 * 1e6));
  printf("salsa 1/lane loop     : %.3f ms  %.2f GB/s keystream\n", t2, nb * 64 / (t2 * 1e6));
  unsigned long long* st; (void)hipMalloc(&st, 16 * 100000);
  float tc = timeit([&] { salsa_clk<<<grid, 256>>>(d, key, 4, st); });
  std::vector<unsigned long long> hs(200000);
  (void)hipMemcpy(hs.data(), st, 16 * 100000, hipMemcpyDeviceToHost);
  double sc = 0, sr = 0; for (int i = 0; i < 100000; i++) { sc += hs[2 * i]; sr += hs[2 * i + 1]; }
  printf("salsa ASM clk-stamped : %.3f ms  in-kernel clock %.3f GHz (memtime/memrealtime*100MHz)\n", tc, sc / sr * 0.1);
  float tp = timeit([&] { poly_k<<<grid, 256>>>(d, key, 16); });
  double nc = 100000.0 * 256 * 16;
  printf("poly horner (16/lane) : %.3f ms  %.2f GB/s authenticated\n", tp, nc * 16 / (tp * 1e6));
  return 0;
}
