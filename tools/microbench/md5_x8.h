// md5_x8.h -- DIAGNOSTIC ONLY (tools/microbench/md5_mb_rate.cpp): the 16-stream MD5 of
// rclone_amd/csrc/md5_x16.h restated over 8 lanes in 256-bit registers, to measure whether a
// host's 16 lanes are bound by vector throughput.  Not part of the library.
#pragma once
#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>

#include "../../rclone_amd/csrc/md5_x16.h"

namespace xs {

// The same over 8 lanes in 256-bit registers (AVX-512VL: ternary logic and rotate on ymm): half
// the work per block step, for CPUs where 16 lanes are bound by vector throughput rather than
// by the chain (then each of 8 lanes runs faster than each of 16).
inline bool md5_x8_supported() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl");
  return ok;
}

__attribute__((target("avx512f,avx512vl"))) inline void md5_x8_transpose8(const uint8_t* const p[8], int off,
                                                                           __m256i m[8]) {
  __m256i r[8], t[8], u[8];
  for (int i = 0; i < 8; i++) r[i] = _mm256_loadu_si256((const __m256i*)(p[i] + off));
  for (int i = 0; i < 8; i += 2) {
    t[i] = _mm256_unpacklo_epi32(r[i], r[i + 1]);
    t[i + 1] = _mm256_unpackhi_epi32(r[i], r[i + 1]);
  }
  for (int g = 0; g < 2; g++) {  // u[4g + j]: 128-bit half k = word 4k + j of rows 4g..4g+3
    u[4 * g + 0] = _mm256_unpacklo_epi64(t[4 * g], t[4 * g + 2]);
    u[4 * g + 1] = _mm256_unpackhi_epi64(t[4 * g], t[4 * g + 2]);
    u[4 * g + 2] = _mm256_unpacklo_epi64(t[4 * g + 1], t[4 * g + 3]);
    u[4 * g + 3] = _mm256_unpackhi_epi64(t[4 * g + 1], t[4 * g + 3]);
  }
  for (int j = 0; j < 4; j++) {
    m[j] = _mm256_permute2x128_si256(u[j], u[4 + j], 0x20);
    m[4 + j] = _mm256_permute2x128_si256(u[j], u[4 + j], 0x31);
  }
}

__attribute__((target("avx512f,avx512vl"))) inline void md5_x8_blocks(uint32_t st[4][8], const uint8_t* p[8],
                                                                       const uint32_t stride[8], size_t nblk) {
  __m256i a0 = _mm256_loadu_si256((const __m256i*)st[0]), b0 = _mm256_loadu_si256((const __m256i*)st[1]);
  __m256i c0 = _mm256_loadu_si256((const __m256i*)st[2]), d0 = _mm256_loadu_si256((const __m256i*)st[3]);
  const uint8_t* q[8];
  for (int i = 0; i < 8; i++) q[i] = p[i];
  for (; nblk; nblk--) {
    __m256i m[16];
    md5_x8_transpose8(q, 0, m);
    md5_x8_transpose8(q, 32, m + 8);
    for (int i = 0; i < 8; i++) q[i] += stride[i];
    __m256i a = a0, b = b0, c = c0, d = d0;
#define XS_MB(f, w, x, y, z, k, t, s)                                                                         \
  w = _mm256_add_epi32(w, _mm256_add_epi32(m[k], _mm256_set1_epi32((int)(t))));                             \
  w = _mm256_add_epi32(x, _mm256_rol_epi32(_mm256_add_epi32(w, _mm256_ternarylogic_epi32(x, y, z, f)), s))
    XS_MB(0xca, a, b, c, d, 0, 0xd76aa478, 7);
    XS_MB(0xca, d, a, b, c, 1, 0xe8c7b756, 12);
    XS_MB(0xca, c, d, a, b, 2, 0x242070db, 17);
    XS_MB(0xca, b, c, d, a, 3, 0xc1bdceee, 22);
    XS_MB(0xca, a, b, c, d, 4, 0xf57c0faf, 7);
    XS_MB(0xca, d, a, b, c, 5, 0x4787c62a, 12);
    XS_MB(0xca, c, d, a, b, 6, 0xa8304613, 17);
    XS_MB(0xca, b, c, d, a, 7, 0xfd469501, 22);
    XS_MB(0xca, a, b, c, d, 8, 0x698098d8, 7);
    XS_MB(0xca, d, a, b, c, 9, 0x8b44f7af, 12);
    XS_MB(0xca, c, d, a, b, 10, 0xffff5bb1, 17);
    XS_MB(0xca, b, c, d, a, 11, 0x895cd7be, 22);
    XS_MB(0xca, a, b, c, d, 12, 0x6b901122, 7);
    XS_MB(0xca, d, a, b, c, 13, 0xfd987193, 12);
    XS_MB(0xca, c, d, a, b, 14, 0xa679438e, 17);
    XS_MB(0xca, b, c, d, a, 15, 0x49b40821, 22);
    XS_MB(0xe4, a, b, c, d, 1, 0xf61e2562, 5);
    XS_MB(0xe4, d, a, b, c, 6, 0xc040b340, 9);
    XS_MB(0xe4, c, d, a, b, 11, 0x265e5a51, 14);
    XS_MB(0xe4, b, c, d, a, 0, 0xe9b6c7aa, 20);
    XS_MB(0xe4, a, b, c, d, 5, 0xd62f105d, 5);
    XS_MB(0xe4, d, a, b, c, 10, 0x02441453, 9);
    XS_MB(0xe4, c, d, a, b, 15, 0xd8a1e681, 14);
    XS_MB(0xe4, b, c, d, a, 4, 0xe7d3fbc8, 20);
    XS_MB(0xe4, a, b, c, d, 9, 0x21e1cde6, 5);
    XS_MB(0xe4, d, a, b, c, 14, 0xc33707d6, 9);
    XS_MB(0xe4, c, d, a, b, 3, 0xf4d50d87, 14);
    XS_MB(0xe4, b, c, d, a, 8, 0x455a14ed, 20);
    XS_MB(0xe4, a, b, c, d, 13, 0xa9e3e905, 5);
    XS_MB(0xe4, d, a, b, c, 2, 0xfcefa3f8, 9);
    XS_MB(0xe4, c, d, a, b, 7, 0x676f02d9, 14);
    XS_MB(0xe4, b, c, d, a, 12, 0x8d2a4c8a, 20);
    XS_MB(0x96, a, b, c, d, 5, 0xfffa3942, 4);
    XS_MB(0x96, d, a, b, c, 8, 0x8771f681, 11);
    XS_MB(0x96, c, d, a, b, 11, 0x6d9d6122, 16);
    XS_MB(0x96, b, c, d, a, 14, 0xfde5380c, 23);
    XS_MB(0x96, a, b, c, d, 1, 0xa4beea44, 4);
    XS_MB(0x96, d, a, b, c, 4, 0x4bdecfa9, 11);
    XS_MB(0x96, c, d, a, b, 7, 0xf6bb4b60, 16);
    XS_MB(0x96, b, c, d, a, 10, 0xbebfbc70, 23);
    XS_MB(0x96, a, b, c, d, 13, 0x289b7ec6, 4);
    XS_MB(0x96, d, a, b, c, 0, 0xeaa127fa, 11);
    XS_MB(0x96, c, d, a, b, 3, 0xd4ef3085, 16);
    XS_MB(0x96, b, c, d, a, 6, 0x04881d05, 23);
    XS_MB(0x96, a, b, c, d, 9, 0xd9d4d039, 4);
    XS_MB(0x96, d, a, b, c, 12, 0xe6db99e5, 11);
    XS_MB(0x96, c, d, a, b, 15, 0x1fa27cf8, 16);
    XS_MB(0x96, b, c, d, a, 2, 0xc4ac5665, 23);
    XS_MB(0x39, a, b, c, d, 0, 0xf4292244, 6);
    XS_MB(0x39, d, a, b, c, 7, 0x432aff97, 10);
    XS_MB(0x39, c, d, a, b, 14, 0xab9423a7, 15);
    XS_MB(0x39, b, c, d, a, 5, 0xfc93a039, 21);
    XS_MB(0x39, a, b, c, d, 12, 0x655b59c3, 6);
    XS_MB(0x39, d, a, b, c, 3, 0x8f0ccc92, 10);
    XS_MB(0x39, c, d, a, b, 10, 0xffeff47d, 15);
    XS_MB(0x39, b, c, d, a, 1, 0x85845dd1, 21);
    XS_MB(0x39, a, b, c, d, 8, 0x6fa87e4f, 6);
    XS_MB(0x39, d, a, b, c, 15, 0xfe2ce6e0, 10);
    XS_MB(0x39, c, d, a, b, 6, 0xa3014314, 15);
    XS_MB(0x39, b, c, d, a, 13, 0x4e0811a1, 21);
    XS_MB(0x39, a, b, c, d, 4, 0xf7537e82, 6);
    XS_MB(0x39, d, a, b, c, 11, 0xbd3af235, 10);
    XS_MB(0x39, c, d, a, b, 2, 0x2ad7d2bb, 15);
    XS_MB(0x39, b, c, d, a, 9, 0xeb86d391, 21);
#undef XS_MB
    a0 = _mm256_add_epi32(a0, a);
    b0 = _mm256_add_epi32(b0, b);
    c0 = _mm256_add_epi32(c0, c);
    d0 = _mm256_add_epi32(d0, d);
  }
  _mm256_storeu_si256((__m256i*)st[0], a0);
  _mm256_storeu_si256((__m256i*)st[1], b0);
  _mm256_storeu_si256((__m256i*)st[2], c0);
  _mm256_storeu_si256((__m256i*)st[3], d0);
}

}  // namespace xs
