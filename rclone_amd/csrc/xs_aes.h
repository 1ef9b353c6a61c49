// AES-256 tables and key schedule shared by the EME kernel (xs_eme.hip) and the host key
// setup (names.cpp).  The S-box is computed at compile time from its definition (GF(2^8)
// inverse followed by the affine map, FIPS-197 §5.1.1); nothing is tabulated by hand.
//
// Word convention: a 16-byte AES state / round key is four little-endian uint32 columns,
// byte 4c+r (row r of column c) in bits 8r..8r+7 of word c.
#pragma once
#include <stdint.h>

namespace xs {
namespace aes {

constexpr uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

constexpr uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xt(a);
    b >>= 1;
  }
  return r;
}

struct Sbox {
  uint8_t fwd[256];
  uint8_t inv[256];
};

constexpr Sbox make_sbox() {
  Sbox t{};
  for (int x = 0; x < 256; x++) {
    // x^254 = x^-1 in GF(2^8) (0 -> 0)
    uint8_t r = 1, b = (uint8_t)x;
    for (int e = 254; e; e >>= 1) {
      if (e & 1) r = gmul(r, b);
      b = gmul(b, b);
    }
    if (x == 0) r = 0;
    uint8_t s = r, q = r;
    for (int i = 0; i < 4; i++) {
      q = (uint8_t)((q << 1) | (q >> 7));
      s ^= q;
    }
    s ^= 0x63;
    t.fwd[x] = s;
    t.inv[s] = (uint8_t)x;
  }
  return t;
}

constexpr uint32_t rotl32(uint32_t v, int k) { return (v << k) | (v >> (32 - k)); }

// MixColumns contribution of row-0 byte s: rows (2s, s, s, 3s).
constexpr uint32_t te0(uint8_t s) { return (uint32_t)xt(s) | (uint32_t)s << 8 | (uint32_t)s << 16 | (uint32_t)(xt(s) ^ s) << 24; }
// InvMixColumns contribution of row-0 byte i: rows (14i, 9i, 13i, 11i).
constexpr uint32_t td0(uint8_t i) {
  return (uint32_t)gmul(i, 14) | (uint32_t)gmul(i, 9) << 8 | (uint32_t)gmul(i, 13) << 16 | (uint32_t)gmul(i, 11) << 24;
}

// Kernel argument: encryption round keys, equivalent-inverse-cipher decryption round keys
// (FIPS-197 §5.3.5), the EME tweak (Cipher.nameTweak) -- 496 bytes.
struct EmeKey {
  uint32_t erk[60];
  uint32_t drk[60];
  uint32_t tweak[4];
};

// InvMixColumns of one column word.
inline uint32_t inv_mix_word(uint32_t w) {
  uint8_t a0 = (uint8_t)w, a1 = (uint8_t)(w >> 8), a2 = (uint8_t)(w >> 16), a3 = (uint8_t)(w >> 24);
  uint8_t r0 = gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9);
  uint8_t r1 = gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13);
  uint8_t r2 = gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11);
  uint8_t r3 = gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14);
  return (uint32_t)r0 | (uint32_t)r1 << 8 | (uint32_t)r2 << 16 | (uint32_t)r3 << 24;
}

// aes.NewCipher(nameKey) (cipher.go:249) for a 32-byte key: FIPS-197 §5.2 expansion.
inline void expand_key(const uint8_t key[32], const uint8_t tweak[16], EmeKey* k) {
  static constexpr Sbox S = make_sbox();
  uint32_t* w = k->erk;
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 | (uint32_t)key[4 * i + 2] << 16 |
           (uint32_t)key[4 * i + 3] << 24;
  uint8_t rcon = 1;
  for (int i = 8; i < 60; i++) {
    uint32_t t = w[i - 1];
    if (i % 8 == 0) {
      t = rotl32(t, 24);  // RotWord on little-endian bytes
      t = (uint32_t)S.fwd[t & 255] | (uint32_t)S.fwd[(t >> 8) & 255] << 8 | (uint32_t)S.fwd[(t >> 16) & 255] << 16 |
          (uint32_t)S.fwd[t >> 24] << 24;
      t ^= rcon;
      rcon = xt(rcon);
    } else if (i % 8 == 4) {
      t = (uint32_t)S.fwd[t & 255] | (uint32_t)S.fwd[(t >> 8) & 255] << 8 | (uint32_t)S.fwd[(t >> 16) & 255] << 16 |
          (uint32_t)S.fwd[t >> 24] << 24;
    }
    w[i] = w[i - 8] ^ t;
  }
  for (int r = 0; r <= 14; r++)
    for (int c = 0; c < 4; c++) {
      uint32_t v = k->erk[4 * (14 - r) + c];
      k->drk[4 * r + c] = (r == 0 || r == 14) ? v : inv_mix_word(v);
    }
  for (int c = 0; c < 4; c++)
    k->tweak[c] = (uint32_t)tweak[4 * c] | (uint32_t)tweak[4 * c + 1] << 8 | (uint32_t)tweak[4 * c + 2] << 16 |
                  (uint32_t)tweak[4 * c + 3] << 24;
}

}  // namespace aes
}  // namespace xs
