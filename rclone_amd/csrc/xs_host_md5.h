// xs_host_md5.h -- MD5 (RFC 1321) on a host core, for the objects the engine routes off the GPU's
// one-lane-per-object MD5 (xs_md5.hip): a single long stream runs ~10x faster on one CPU core
// than on one GPU lane, because MD5 is one dependency chain per stream.  The hash is the one
// crypt.put tees off the ciphertext (backend/crypt/crypt.go:516-533) and cryptcheck recomputes
// (crypt.go:784-806): MD5("RCLONE\0\0" || nonce || wire blocks).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace xs {

class HostMd5 {
 public:
  void update(const uint8_t* p, size_t len) {
    size_t have = (size_t)(n_ & 63);
    n_ += len;
    if (have) {
      size_t k = 64 - have < len ? 64 - have : len;
      memcpy(buf_ + have, p, k);
      p += k;
      len -= k;
      if (have + k < 64) return;
      blocks(buf_, 1);
    }
    if (len >= 64) {
      blocks(p, len / 64);
      p += len & ~(size_t)63;
      len &= 63;
    }
    memcpy(buf_, p, len);
  }
  // For an asynchronous block engine (md5_x16.h): the four state words, and the split of an
  // update into what must run here and the whole blocks the engine may run later.  begin_blocks
  // hashes the bytes completing a pending partial block, counts every byte and buffers the
  // trailing partial block; it returns the whole blocks in between (*nblk of them), which must be
  // applied to state() before the next update or final.
  uint32_t* state() { return h_; }
  const uint8_t* begin_blocks(const uint8_t* p, size_t len, size_t* nblk) {
    size_t have = (size_t)(n_ & 63);
    n_ += len;
    if (have) {
      size_t k = 64 - have < len ? 64 - have : len;
      memcpy(buf_ + have, p, k);
      p += k;
      len -= k;
      if (have + k == 64) blocks(buf_, 1);
      else {
        *nblk = 0;
        return p;
      }
    }
    *nblk = len / 64;
    memcpy(buf_, p + (len & ~(size_t)63), len & 63);
    return p;
  }
  void final(uint8_t out[16]) {
    const uint64_t bits = n_ * 8;
    uint8_t pad[72] = {0x80};
    const size_t have = (size_t)(n_ & 63);
    const size_t padlen = have < 56 ? 56 - have : 120 - have;
    update(pad, padlen);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (8 * i));
    update(lb, 8);
    memcpy(out, h_, 16);
  }

 private:
  uint32_t h_[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint8_t buf_[64];
  uint64_t n_ = 0;

  static inline uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

  void blocks(const uint8_t* p, size_t nblk) {
    uint32_t a0 = h_[0], b0 = h_[1], c0 = h_[2], d0 = h_[3];
    for (; nblk; nblk--, p += 64) {
      uint32_t m[16];
      memcpy(m, p, 64);  // little-endian host
      uint32_t a = a0, b = b0, c = c0, d = d0;
// The step is w = x + rol(w + f(x, y, z) + m + t, s) with x the newest word.  Everything that
// does not depend on x is added first, so the chain through x is as short as the function allows
// (one step's latency is the stream's rate: MD5 is one dependency chain):
//   F = z ^ (x & (y ^ z)): and, xor;  G = (x & z) + (y & ~z) (disjoint bits): the y & ~z half
//   joins the early sum, leaving one and;  H = x ^ (y ^ z): one xor;  I = y ^ (x | ~z): or, xor.
// XS_EARLY pins that order: clang otherwise re-associates the sum and puts an add back on the
// chain (its build ran ~20% below gcc's).
#define XS_EARLY(w) __asm__("" : "+r"(w))
#define XS_F(w, x, y, z, mk) w += (mk); XS_EARLY(w); w += (z) ^ ((x) & ((y) ^ (z)))
#define XS_G(w, x, y, z, mk) w += (mk) + ((y) & ~(z)); XS_EARLY(w); w += (x) & (z)
#define XS_H(w, x, y, z, mk) w += (mk); XS_EARLY(w); w += (x) ^ ((y) ^ (z))
#define XS_I(w, x, y, z, mk) w += (mk); XS_EARLY(w); w += (y) ^ ((x) | ~(z))
#define XS_STEP(f, w, x, y, z, k, t, s) \
  f(w, x, y, z, m[k] + (uint32_t)(t));   \
  w = x + rol(w, s)
      XS_STEP(XS_F, a, b, c, d, 0, 0xd76aa478, 7);
      XS_STEP(XS_F, d, a, b, c, 1, 0xe8c7b756, 12);
      XS_STEP(XS_F, c, d, a, b, 2, 0x242070db, 17);
      XS_STEP(XS_F, b, c, d, a, 3, 0xc1bdceee, 22);
      XS_STEP(XS_F, a, b, c, d, 4, 0xf57c0faf, 7);
      XS_STEP(XS_F, d, a, b, c, 5, 0x4787c62a, 12);
      XS_STEP(XS_F, c, d, a, b, 6, 0xa8304613, 17);
      XS_STEP(XS_F, b, c, d, a, 7, 0xfd469501, 22);
      XS_STEP(XS_F, a, b, c, d, 8, 0x698098d8, 7);
      XS_STEP(XS_F, d, a, b, c, 9, 0x8b44f7af, 12);
      XS_STEP(XS_F, c, d, a, b, 10, 0xffff5bb1, 17);
      XS_STEP(XS_F, b, c, d, a, 11, 0x895cd7be, 22);
      XS_STEP(XS_F, a, b, c, d, 12, 0x6b901122, 7);
      XS_STEP(XS_F, d, a, b, c, 13, 0xfd987193, 12);
      XS_STEP(XS_F, c, d, a, b, 14, 0xa679438e, 17);
      XS_STEP(XS_F, b, c, d, a, 15, 0x49b40821, 22);
      XS_STEP(XS_G, a, b, c, d, 1, 0xf61e2562, 5);
      XS_STEP(XS_G, d, a, b, c, 6, 0xc040b340, 9);
      XS_STEP(XS_G, c, d, a, b, 11, 0x265e5a51, 14);
      XS_STEP(XS_G, b, c, d, a, 0, 0xe9b6c7aa, 20);
      XS_STEP(XS_G, a, b, c, d, 5, 0xd62f105d, 5);
      XS_STEP(XS_G, d, a, b, c, 10, 0x02441453, 9);
      XS_STEP(XS_G, c, d, a, b, 15, 0xd8a1e681, 14);
      XS_STEP(XS_G, b, c, d, a, 4, 0xe7d3fbc8, 20);
      XS_STEP(XS_G, a, b, c, d, 9, 0x21e1cde6, 5);
      XS_STEP(XS_G, d, a, b, c, 14, 0xc33707d6, 9);
      XS_STEP(XS_G, c, d, a, b, 3, 0xf4d50d87, 14);
      XS_STEP(XS_G, b, c, d, a, 8, 0x455a14ed, 20);
      XS_STEP(XS_G, a, b, c, d, 13, 0xa9e3e905, 5);
      XS_STEP(XS_G, d, a, b, c, 2, 0xfcefa3f8, 9);
      XS_STEP(XS_G, c, d, a, b, 7, 0x676f02d9, 14);
      XS_STEP(XS_G, b, c, d, a, 12, 0x8d2a4c8a, 20);
      XS_STEP(XS_H, a, b, c, d, 5, 0xfffa3942, 4);
      XS_STEP(XS_H, d, a, b, c, 8, 0x8771f681, 11);
      XS_STEP(XS_H, c, d, a, b, 11, 0x6d9d6122, 16);
      XS_STEP(XS_H, b, c, d, a, 14, 0xfde5380c, 23);
      XS_STEP(XS_H, a, b, c, d, 1, 0xa4beea44, 4);
      XS_STEP(XS_H, d, a, b, c, 4, 0x4bdecfa9, 11);
      XS_STEP(XS_H, c, d, a, b, 7, 0xf6bb4b60, 16);
      XS_STEP(XS_H, b, c, d, a, 10, 0xbebfbc70, 23);
      XS_STEP(XS_H, a, b, c, d, 13, 0x289b7ec6, 4);
      XS_STEP(XS_H, d, a, b, c, 0, 0xeaa127fa, 11);
      XS_STEP(XS_H, c, d, a, b, 3, 0xd4ef3085, 16);
      XS_STEP(XS_H, b, c, d, a, 6, 0x04881d05, 23);
      XS_STEP(XS_H, a, b, c, d, 9, 0xd9d4d039, 4);
      XS_STEP(XS_H, d, a, b, c, 12, 0xe6db99e5, 11);
      XS_STEP(XS_H, c, d, a, b, 15, 0x1fa27cf8, 16);
      XS_STEP(XS_H, b, c, d, a, 2, 0xc4ac5665, 23);
      XS_STEP(XS_I, a, b, c, d, 0, 0xf4292244, 6);
      XS_STEP(XS_I, d, a, b, c, 7, 0x432aff97, 10);
      XS_STEP(XS_I, c, d, a, b, 14, 0xab9423a7, 15);
      XS_STEP(XS_I, b, c, d, a, 5, 0xfc93a039, 21);
      XS_STEP(XS_I, a, b, c, d, 12, 0x655b59c3, 6);
      XS_STEP(XS_I, d, a, b, c, 3, 0x8f0ccc92, 10);
      XS_STEP(XS_I, c, d, a, b, 10, 0xffeff47d, 15);
      XS_STEP(XS_I, b, c, d, a, 1, 0x85845dd1, 21);
      XS_STEP(XS_I, a, b, c, d, 8, 0x6fa87e4f, 6);
      XS_STEP(XS_I, d, a, b, c, 15, 0xfe2ce6e0, 10);
      XS_STEP(XS_I, c, d, a, b, 6, 0xa3014314, 15);
      XS_STEP(XS_I, b, c, d, a, 13, 0x4e0811a1, 21);
      XS_STEP(XS_I, a, b, c, d, 4, 0xf7537e82, 6);
      XS_STEP(XS_I, d, a, b, c, 11, 0xbd3af235, 10);
      XS_STEP(XS_I, c, d, a, b, 2, 0x2ad7d2bb, 15);
      XS_STEP(XS_I, b, c, d, a, 9, 0xeb86d391, 21);
#undef XS_STEP
#undef XS_I
#undef XS_H
#undef XS_G
#undef XS_F
#undef XS_EARLY
      a0 += a;
      b0 += b;
      c0 += c;
      d0 += d;
    }
    h_[0] = a0;
    h_[1] = b0;
    h_[2] = c0;
    h_[3] = d0;
  }
};

}  // namespace xs
