// scrypt.cpp -- key derivation for Cipher.Key (backend/crypt/cipher.go:231-252):
// scrypt(password, salt, N=16384, r=8, p=1, 80 bytes) -> dataKey[0:32] | nameKey[32:64] |
// nameTweak[64:80].  Host-only (once per remote).  The reference takes it from
// golang.org/x/crypto/scrypt v0.54.0; this is a restatement of RFC 7914 (PBKDF2-HMAC-SHA256 +
// Salsa20/8 BlockMix + ROMix), checked against cipher_test.go TestKey (:1609-1642).
#include <cstdint>
#include <cstring>
#include <vector>

namespace rc {

namespace {

struct Sha256 {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len = 0;
  size_t fill = 0;
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  Sha256() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, sizeof iv);
  }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
      uint32_t ch = (e & f) ^ (~e & g);
      uint32_t t1 = hh + S1 + ch + K[i] + w[i];
      uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
      uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      size_t take = 64 - fill < n ? 64 - fill : n;
      memcpy(buf + fill, p, take);
      fill += take; p += take; n -= take;
      if (fill == 64) { block(buf); fill = 0; }
    }
  }
  void final(uint8_t out[32]) {
    uint64_t bits = len * 8;
    uint8_t pad = 0x80;
    update(&pad, 1);
    uint8_t z = 0;
    while (fill != 56) update(&z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(lb, 8);
    for (int i = 0; i < 8; i++) {
      out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
      out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
    }
  }
};

void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* m1, size_t n1, const uint8_t* m2, size_t n2,
                 uint8_t out[32]) {
  uint8_t k[64] = {0};
  if (klen > 64) {
    Sha256 s; s.update(key, klen); s.final(k);
  } else {
    memcpy(k, key, klen);
  }
  uint8_t ipad[64], opad[64];
  for (int i = 0; i < 64; i++) { ipad[i] = k[i] ^ 0x36; opad[i] = k[i] ^ 0x5c; }
  uint8_t inner[32];
  Sha256 a; a.update(ipad, 64); a.update(m1, n1); if (n2) a.update(m2, n2); a.final(inner);
  Sha256 b; b.update(opad, 64); b.update(inner, 32); b.final(out);
}

// PBKDF2-HMAC-SHA256 with c = 1 (as scrypt uses it)
void pbkdf2_1(const uint8_t* pw, size_t pwlen, const uint8_t* salt, size_t slen, uint8_t* out, size_t olen) {
  for (uint32_t blk = 1; olen > 0; blk++) {
    uint8_t ctr[4] = {(uint8_t)(blk >> 24), (uint8_t)(blk >> 16), (uint8_t)(blk >> 8), (uint8_t)blk};
    uint8_t u[32];
    hmac_sha256(pw, pwlen, salt, slen, ctr, 4, u);
    size_t take = olen < 32 ? olen : 32;
    memcpy(out, u, take);
    out += take; olen -= take;
  }
}

inline uint32_t rl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void salsa8(uint32_t b[16]) {
  uint32_t x[16];
  memcpy(x, b, 64);
  for (int i = 0; i < 8; i += 2) {
    x[4] ^= rl(x[0] + x[12], 7);  x[8] ^= rl(x[4] + x[0], 9);   x[12] ^= rl(x[8] + x[4], 13);  x[0] ^= rl(x[12] + x[8], 18);
    x[9] ^= rl(x[5] + x[1], 7);   x[13] ^= rl(x[9] + x[5], 9);  x[1] ^= rl(x[13] + x[9], 13);  x[5] ^= rl(x[1] + x[13], 18);
    x[14] ^= rl(x[10] + x[6], 7); x[2] ^= rl(x[14] + x[10], 9); x[6] ^= rl(x[2] + x[14], 13);  x[10] ^= rl(x[6] + x[2], 18);
    x[3] ^= rl(x[15] + x[11], 7); x[7] ^= rl(x[3] + x[15], 9);  x[11] ^= rl(x[7] + x[3], 13);  x[15] ^= rl(x[11] + x[7], 18);
    x[1] ^= rl(x[0] + x[3], 7);   x[2] ^= rl(x[1] + x[0], 9);   x[3] ^= rl(x[2] + x[1], 13);   x[0] ^= rl(x[3] + x[2], 18);
    x[6] ^= rl(x[5] + x[4], 7);   x[7] ^= rl(x[6] + x[5], 9);   x[4] ^= rl(x[7] + x[6], 13);   x[5] ^= rl(x[4] + x[7], 18);
    x[11] ^= rl(x[10] + x[9], 7); x[8] ^= rl(x[11] + x[10], 9); x[9] ^= rl(x[8] + x[11], 13);  x[10] ^= rl(x[9] + x[8], 18);
    x[12] ^= rl(x[15] + x[14], 7); x[13] ^= rl(x[12] + x[15], 9); x[14] ^= rl(x[13] + x[12], 13); x[15] ^= rl(x[14] + x[13], 18);
  }
  for (int i = 0; i < 16; i++) b[i] += x[i];
}

// BlockMix_{Salsa20/8, r}: B (2r 64-byte blocks) -> Y
void blockmix(const uint32_t* B, uint32_t* Y, int r) {
  uint32_t X[16];
  memcpy(X, B + (2 * r - 1) * 16, 64);
  for (int i = 0; i < 2 * r; i++) {
    for (int j = 0; j < 16; j++) X[j] ^= B[i * 16 + j];
    salsa8(X);
    // even blocks to the first half, odd blocks to the second half
    memcpy(Y + ((i & 1) * r + i / 2) * 16, X, 64);
  }
}

}  // namespace

bool scrypt(const uint8_t* pw, size_t pwlen, const uint8_t* salt, size_t slen, uint64_t N, int r, int p,
            uint8_t* out, size_t olen) {
  if (N < 2 || (N & (N - 1)) || r <= 0 || p <= 0) return false;
  const size_t blen = (size_t)128 * r;
  std::vector<uint8_t> B((size_t)p * blen);
  pbkdf2_1(pw, pwlen, salt, slen, B.data(), B.size());
  std::vector<uint32_t> V((size_t)N * 32 * r), X(32 * r), Y(32 * r);
  for (int pi = 0; pi < p; pi++) {
    uint8_t* Bp = B.data() + (size_t)pi * blen;
    for (int i = 0; i < 32 * r; i++)
      X[i] = (uint32_t)Bp[4 * i] | (uint32_t)Bp[4 * i + 1] << 8 | (uint32_t)Bp[4 * i + 2] << 16 | (uint32_t)Bp[4 * i + 3] << 24;
    for (uint64_t i = 0; i < N; i++) {
      memcpy(&V[i * 32 * r], X.data(), 128 * r);
      blockmix(X.data(), Y.data(), r);
      X.swap(Y);
    }
    for (uint64_t i = 0; i < N; i++) {
      uint64_t j = X[(2 * r - 1) * 16] & (N - 1);
      for (int k = 0; k < 32 * r; k++) X[k] ^= V[j * 32 * r + k];
      blockmix(X.data(), Y.data(), r);
      X.swap(Y);
    }
    for (int i = 0; i < 32 * r; i++) {
      Bp[4 * i] = (uint8_t)X[i]; Bp[4 * i + 1] = (uint8_t)(X[i] >> 8);
      Bp[4 * i + 2] = (uint8_t)(X[i] >> 16); Bp[4 * i + 3] = (uint8_t)(X[i] >> 24);
    }
  }
  pbkdf2_1(pw, pwlen, B.data(), B.size(), out, olen);
  return true;
}

}  // namespace rc
