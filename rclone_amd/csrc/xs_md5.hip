// MD5 of many byte streams in HBM, one lane per stream (RFC 1321).
//
// Why: crypt's Fs.put tees the ciphertext into the destination's hash (MD5 for
// backend/memory and most remotes, crypt.go:516-533) and cryptcheck re-encrypts the source
// with the stored nonce and MD5s the result (computeHashWithNonce, crypt.go:784-806).  With
// the cipher on the GPU the ciphertext is already in HBM; hashing it there returns 16 bytes
// per object instead of the whole ciphertext over PCIe.  MD5 is sequential within a
// stream, so the parallelism is across streams: lane i hashes stream i.
//
// Each stream is an optional 16-byte-multiple prefix held in the descriptor (the 32-byte
// crypt header "RCLONE\0\0" || nonce, which is never materialised in HBM) followed by `len`
// bytes at a 16-byte aligned offset of the source buffer (the wire body).  Every 16-byte
// chunk is therefore either wholly prefix or an aligned 16-byte load.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "xs_internal.h"

static_assert(sizeof(xs_md5_desc) == 64, "xs_md5_desc layout");

namespace xs {

namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

#define XS_MD5_STEP(f, a, b, c, d, m, k, s) a = b + rotl(a + (f) + (m) + (k), s)

__device__ __forceinline__ void md5_block(uint32_t st[4], const uint32_t m[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#define F1(b, c, d) (((b) & (c)) | (~(b) & (d)))
#define F2(b, c, d) (((b) & (d)) | ((c) & ~(d)))
#define F3(b, c, d) ((b) ^ (c) ^ (d))
#define F4(b, c, d) ((c) ^ ((b) | ~(d)))
  XS_MD5_STEP(F1(b, c, d), a, b, c, d, m[0], 0xd76aa478u, 7);
  XS_MD5_STEP(F1(a, b, c), d, a, b, c, m[1], 0xe8c7b756u, 12);
  XS_MD5_STEP(F1(d, a, b), c, d, a, b, m[2], 0x242070dbu, 17);
  XS_MD5_STEP(F1(c, d, a), b, c, d, a, m[3], 0xc1bdceeeu, 22);
  XS_MD5_STEP(F1(b, c, d), a, b, c, d, m[4], 0xf57c0fafu, 7);
  XS_MD5_STEP(F1(a, b, c), d, a, b, c, m[5], 0x4787c62au, 12);
  XS_MD5_STEP(F1(d, a, b), c, d, a, b, m[6], 0xa8304613u, 17);
  XS_MD5_STEP(F1(c, d, a), b, c, d, a, m[7], 0xfd469501u, 22);
  XS_MD5_STEP(F1(b, c, d), a, b, c, d, m[8], 0x698098d8u, 7);
  XS_MD5_STEP(F1(a, b, c), d, a, b, c, m[9], 0x8b44f7afu, 12);
  XS_MD5_STEP(F1(d, a, b), c, d, a, b, m[10], 0xffff5bb1u, 17);
  XS_MD5_STEP(F1(c, d, a), b, c, d, a, m[11], 0x895cd7beu, 22);
  XS_MD5_STEP(F1(b, c, d), a, b, c, d, m[12], 0x6b901122u, 7);
  XS_MD5_STEP(F1(a, b, c), d, a, b, c, m[13], 0xfd987193u, 12);
  XS_MD5_STEP(F1(d, a, b), c, d, a, b, m[14], 0xa679438eu, 17);
  XS_MD5_STEP(F1(c, d, a), b, c, d, a, m[15], 0x49b40821u, 22);

  XS_MD5_STEP(F2(b, c, d), a, b, c, d, m[1], 0xf61e2562u, 5);
  XS_MD5_STEP(F2(a, b, c), d, a, b, c, m[6], 0xc040b340u, 9);
  XS_MD5_STEP(F2(d, a, b), c, d, a, b, m[11], 0x265e5a51u, 14);
  XS_MD5_STEP(F2(c, d, a), b, c, d, a, m[0], 0xe9b6c7aau, 20);
  XS_MD5_STEP(F2(b, c, d), a, b, c, d, m[5], 0xd62f105du, 5);
  XS_MD5_STEP(F2(a, b, c), d, a, b, c, m[10], 0x02441453u, 9);
  XS_MD5_STEP(F2(d, a, b), c, d, a, b, m[15], 0xd8a1e681u, 14);
  XS_MD5_STEP(F2(c, d, a), b, c, d, a, m[4], 0xe7d3fbc8u, 20);
  XS_MD5_STEP(F2(b, c, d), a, b, c, d, m[9], 0x21e1cde6u, 5);
  XS_MD5_STEP(F2(a, b, c), d, a, b, c, m[14], 0xc33707d6u, 9);
  XS_MD5_STEP(F2(d, a, b), c, d, a, b, m[3], 0xf4d50d87u, 14);
  XS_MD5_STEP(F2(c, d, a), b, c, d, a, m[8], 0x455a14edu, 20);
  XS_MD5_STEP(F2(b, c, d), a, b, c, d, m[13], 0xa9e3e905u, 5);
  XS_MD5_STEP(F2(a, b, c), d, a, b, c, m[2], 0xfcefa3f8u, 9);
  XS_MD5_STEP(F2(d, a, b), c, d, a, b, m[7], 0x676f02d9u, 14);
  XS_MD5_STEP(F2(c, d, a), b, c, d, a, m[12], 0x8d2a4c8au, 20);

  XS_MD5_STEP(F3(b, c, d), a, b, c, d, m[5], 0xfffa3942u, 4);
  XS_MD5_STEP(F3(a, b, c), d, a, b, c, m[8], 0x8771f681u, 11);
  XS_MD5_STEP(F3(d, a, b), c, d, a, b, m[11], 0x6d9d6122u, 16);
  XS_MD5_STEP(F3(c, d, a), b, c, d, a, m[14], 0xfde5380cu, 23);
  XS_MD5_STEP(F3(b, c, d), a, b, c, d, m[1], 0xa4beea44u, 4);
  XS_MD5_STEP(F3(a, b, c), d, a, b, c, m[4], 0x4bdecfa9u, 11);
  XS_MD5_STEP(F3(d, a, b), c, d, a, b, m[7], 0xf6bb4b60u, 16);
  XS_MD5_STEP(F3(c, d, a), b, c, d, a, m[10], 0xbebfbc70u, 23);
  XS_MD5_STEP(F3(b, c, d), a, b, c, d, m[13], 0x289b7ec6u, 4);
  XS_MD5_STEP(F3(a, b, c), d, a, b, c, m[0], 0xeaa127fau, 11);
  XS_MD5_STEP(F3(d, a, b), c, d, a, b, m[3], 0xd4ef3085u, 16);
  XS_MD5_STEP(F3(c, d, a), b, c, d, a, m[6], 0x04881d05u, 23);
  XS_MD5_STEP(F3(b, c, d), a, b, c, d, m[9], 0xd9d4d039u, 4);
  XS_MD5_STEP(F3(a, b, c), d, a, b, c, m[12], 0xe6db99e5u, 11);
  XS_MD5_STEP(F3(d, a, b), c, d, a, b, m[15], 0x1fa27cf8u, 16);
  XS_MD5_STEP(F3(c, d, a), b, c, d, a, m[2], 0xc4ac5665u, 23);

  XS_MD5_STEP(F4(b, c, d), a, b, c, d, m[0], 0xf4292244u, 6);
  XS_MD5_STEP(F4(a, b, c), d, a, b, c, m[7], 0x432aff97u, 10);
  XS_MD5_STEP(F4(d, a, b), c, d, a, b, m[14], 0xab9423a7u, 15);
  XS_MD5_STEP(F4(c, d, a), b, c, d, a, m[5], 0xfc93a039u, 21);
  XS_MD5_STEP(F4(b, c, d), a, b, c, d, m[12], 0x655b59c3u, 6);
  XS_MD5_STEP(F4(a, b, c), d, a, b, c, m[3], 0x8f0ccc92u, 10);
  XS_MD5_STEP(F4(d, a, b), c, d, a, b, m[10], 0xffeff47du, 15);
  XS_MD5_STEP(F4(c, d, a), b, c, d, a, m[1], 0x85845dd1u, 21);
  XS_MD5_STEP(F4(b, c, d), a, b, c, d, m[8], 0x6fa87e4fu, 6);
  XS_MD5_STEP(F4(a, b, c), d, a, b, c, m[15], 0xfe2ce6e0u, 10);
  XS_MD5_STEP(F4(d, a, b), c, d, a, b, m[6], 0xa3014314u, 15);
  XS_MD5_STEP(F4(c, d, a), b, c, d, a, m[13], 0x4e0811a1u, 21);
  XS_MD5_STEP(F4(b, c, d), a, b, c, d, m[4], 0xf7537e82u, 6);
  XS_MD5_STEP(F4(a, b, c), d, a, b, c, m[11], 0xbd3af235u, 10);
  XS_MD5_STEP(F4(d, a, b), c, d, a, b, m[2], 0x2ad7d2bbu, 15);
  XS_MD5_STEP(F4(c, d, a), b, c, d, a, m[9], 0xeb86d391u, 21);
#undef F1
#undef F2
#undef F3
#undef F4
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
}
#undef XS_MD5_STEP

// 16-byte chunk q (byte offset 16q) of prefix || data; the prefix is read from the
// descriptor in global memory (a dynamically indexed local copy would go to scratch)
__device__ __forceinline__ uint4 chunk(const uint8_t* __restrict__ prefix, uint32_t prefix_len, uint64_t off,
                                       const uint8_t* __restrict__ src, uint64_t q) {
  const uint64_t p = 16u * q;
  if (p < prefix_len) return *reinterpret_cast<const uint4*>(prefix + p);
  return *reinterpret_cast<const uint4*>(src + off + (p - prefix_len));
}

__device__ __forceinline__ uint32_t byte_at(const uint8_t* __restrict__ prefix, uint32_t prefix_len, uint64_t off,
                                            const uint8_t* __restrict__ src, uint64_t p) {
  return p < prefix_len ? prefix[p] : src[off + (p - prefix_len)];
}

}  // namespace

__global__ void __launch_bounds__(64) xs_md5(const xs_md5_desc* __restrict__ descs, uint64_t n,
                                             const uint8_t* __restrict__ src, uint64_t src_len,
                                             uint8_t* __restrict__ digest, uint8_t* __restrict__ ok) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const xs_md5_desc& d = descs[i];
  const uint64_t off = d.off, len = d.len;
  const uint32_t plen = d.prefix_len;
  const uint8_t* prefix = d.prefix;
  const bool valid = plen <= 32u && (plen & 15u) == 0 && (off & 15u) == 0 && off <= src_len && len <= src_len - off;
  if (ok) ok[i] = valid ? 1 : 0;
  uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  if (valid) {
    const uint64_t total = plen + len;
    const uint64_t nfull = total >> 6;
    uint32_t m[16];
    // Full blocks, loads two blocks ahead of the compression (one lane's stream is a serial
    // chain: without the prefetch every block waited a whole HBM round trip).  Block 0 holds
    // the prefix; from block 1 on the stream is plain data at body + 64 b - prefix_len.
    const uint8_t* body = src + off - plen;
    uint4 A[4], B[4], C[4];
    auto fetch = [&](uint4 (&q)[4], uint64_t b) {
#pragma unroll
      for (int j = 0; j < 4; j++) q[j] = *reinterpret_cast<const uint4*>(body + 64u * b + 16u * j);
    };
    auto compress = [&](const uint4 (&q)[4]) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        m[4 * j] = q[j].x; m[4 * j + 1] = q[j].y; m[4 * j + 2] = q[j].z; m[4 * j + 3] = q[j].w;
      }
      md5_block(st, m);
    };
    if (nfull > 0) {
#pragma unroll
      for (int j = 0; j < 4; j++) A[j] = chunk(prefix, plen, off, src, j);
    }
    if (nfull > 1) fetch(B, 1);
#pragma unroll 1
    for (uint64_t b = 0; b < nfull; b += 3) {  // A, B, C rotate: no register moves, no early waits
      if (b + 2 < nfull) fetch(C, b + 2);
      compress(A);
      if (b + 1 >= nfull) break;
      if (b + 3 < nfull) fetch(A, b + 3);
      compress(B);
      if (b + 2 >= nfull) break;
      if (b + 4 < nfull) fetch(B, b + 4);
      compress(C);
    }
    // tail: remaining bytes, 0x80, zero pad, 64-bit little-endian bit length
    const uint32_t rem = (uint32_t)(total & 63u);
    const uint64_t base = nfull << 6;
    const uint64_t bits = total << 3;
    const int tail_blocks = rem < 56u ? 1 : 2;
#pragma unroll 1
    for (int t = 0; t < tail_blocks; t++) {
#pragma unroll
      for (int j = 0; j < 16; j++) m[j] = 0;
      for (uint32_t k = 0; k < 64u; k++) {
        const uint32_t pos = 64u * (uint32_t)t + k;  // position after base
        uint32_t v = 0;
        if (pos < rem) v = byte_at(prefix, plen, off, src, base + pos);
        else if (pos == rem) v = 0x80u;
        m[k >> 2] |= v << (8u * (k & 3u));
      }
      if (t == tail_blocks - 1) {
        m[14] = (uint32_t)bits;
        m[15] = (uint32_t)(bits >> 32);
      }
      md5_block(st, m);
    }
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(digest + 16u * i);
  o[0] = st[0];
  o[1] = st[1];
  o[2] = st[2];
  o[3] = st[3];
}

hipError_t launch_md5(const xs_md5_desc* d, uint64_t n, const uint8_t* src, uint64_t src_len, uint8_t* digest,
                      uint8_t* ok, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(xs_md5, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, stream, d, n, src, src_len, digest, ok);
  return hipGetLastError();
}

}  // namespace xs
