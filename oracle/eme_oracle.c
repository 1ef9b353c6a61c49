/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement of rclone crypt's file-name cipher, the checker
 * for the HIP EME kernel (rclone_amd/csrc/xs_eme.hip).  Never shipped, never measured.
 *
 * What it restates:
 *   - AES-256 block encrypt / decrypt (FIPS-197; Go crypto/aes, keyed by Cipher.Key,
 *     backend/crypt/cipher.go:249 `aes.NewCipher(c.nameKey[:])`), written from the spec in
 *     plain byte arithmetic (S-box computed from the GF(2^8) inverse, no tables copied).
 *   - EME (ECB-Mix-ECB, Halevi-Rogaway 2003) as implemented by github.com/rfjakob/eme v1.2.0
 *     (go.mod:78; not vendored under /root/reference): L = 2*E(0), L_j = 2^(j+1)*E(0) for the
 *     0-based block j, the mixing step MP = T xor sum PPP_j, MC = E(MP), M = MP xor MC,
 *     CCC_j = PPP_j xor 2^j*M (j >= 1), CCC_0 = MC xor T xor sum_{j>=1} CCC_j, C_j = E(CCC_j)
 *     xor L_j.  Decryption runs the same structure with AES decryption (L stays E(0)-based).
 *     Doubling in GF(2^128) is little-endian in bytes (byte 0 least significant, reduction
 *     0x87 into byte 0).  Called from cipher.go:288 (encryptSegment) and :312 (decryptSegment).
 *   - PKCS#7 pad/unpad to 16 (backend/crypt/pkcs7/pkcs7.go:20-63).
 * Pinned by the reference's own name vectors (cipher_test.go:207-271 TestEncryptSegment*,
 * zero key and tweak) and by OpenSSL AES-256-ECB fixtures (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <string.h>

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xt(a);
    b >>= 1;
  }
  return r;
}

static uint8_t SBOX[256], INV_SBOX[256];
static int tables_ready;

static void init_tables(void) {
  if (tables_ready) return;
  for (int x = 0; x < 256; x++) {
    uint8_t inv = 0;
    if (x) {
      for (int y = 1; y < 256; y++)
        if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    }
    /* affine transform: b ^ rotl(b,1) ^ rotl(b,2) ^ rotl(b,3) ^ rotl(b,4) ^ 0x63 */
    uint8_t b = inv, s = inv;
    for (int i = 0; i < 4; i++) {
      b = (uint8_t)((b << 1) | (b >> 7));
      s ^= b;
    }
    s ^= 0x63;
    SBOX[x] = s;
    INV_SBOX[s] = (uint8_t)x;
  }
  tables_ready = 1;
}

/* AES-256 key expansion: 15 round keys of 16 bytes (FIPS-197 §5.2). */
void orc_aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
  init_tables();
  memcpy(rk, key, 32);
  uint8_t rcon = 1;
  for (int i = 8; i < 60; i++) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 8 == 0) {
      uint8_t u = t[0];
      t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
      t[1] = SBOX[t[2]];
      t[2] = SBOX[t[3]];
      t[3] = SBOX[u];
      rcon = xt(rcon);
    } else if (i % 8 == 4) {
      for (int k = 0; k < 4; k++) t[k] = SBOX[t[k]];
    }
    for (int k = 0; k < 4; k++) rk[4 * i + k] = (uint8_t)(rk[4 * (i - 8) + k] ^ t[k]);
  }
}

/* state byte index = 4*column + row (FIPS-197 input order) */
void orc_aes256_encrypt(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16], t[16];
  for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[i]);
  for (int r = 1; r <= 14; r++) {
    for (int c = 0; c < 4; c++)
      for (int w = 0; w < 4; w++) t[4 * c + w] = SBOX[s[4 * ((c + w) & 3) + w]]; /* SubBytes+ShiftRows */
    if (r != 14) {
      for (int c = 0; c < 4; c++) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c + 0] = (uint8_t)(xt(a0) ^ xt(a1) ^ a1 ^ a2 ^ a3);
        s[4 * c + 1] = (uint8_t)(a0 ^ xt(a1) ^ xt(a2) ^ a2 ^ a3);
        s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xt(a2) ^ xt(a3) ^ a3);
        s[4 * c + 3] = (uint8_t)(xt(a0) ^ a0 ^ a1 ^ a2 ^ xt(a3));
      }
    } else {
      memcpy(s, t, 16);
    }
    for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
  }
  memcpy(out, s, 16);
}

void orc_aes256_decrypt(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16], t[16];
  init_tables();
  for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[224 + i]);
  for (int r = 13; r >= 0; r--) {
    for (int c = 0; c < 4; c++) /* InvShiftRows + InvSubBytes */
      for (int w = 0; w < 4; w++) t[4 * ((c + w) & 3) + w] = INV_SBOX[s[4 * c + w]];
    for (int i = 0; i < 16; i++) t[i] ^= rk[16 * r + i];
    if (r != 0) {
      for (int c = 0; c < 4; c++) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c + 0] = (uint8_t)(gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9));
        s[4 * c + 1] = (uint8_t)(gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13));
        s[4 * c + 2] = (uint8_t)(gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11));
        s[4 * c + 3] = (uint8_t)(gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14));
      }
    } else {
      memcpy(s, t, 16);
    }
  }
  memcpy(out, s, 16);
}

/* rfjakob/eme multByTwo: little-endian doubling in GF(2^128). */
static void dbl(uint8_t b[16]) {
  uint8_t carry = (uint8_t)(b[15] >> 7);
  for (int j = 15; j > 0; j--) b[j] = (uint8_t)((b[j] << 1) | (b[j - 1] >> 7));
  b[0] = (uint8_t)((b[0] << 1) ^ (carry ? 0x87 : 0));
}

static void xor16(uint8_t *d, const uint8_t *a, const uint8_t *b) {
  for (int i = 0; i < 16; i++) d[i] = (uint8_t)(a[i] ^ b[i]);
}

/* eme.Transform(aes(key), tweak, in[0:16*m], direction); direction 0 = encrypt, 1 = decrypt.
 * Returns 0, or -1 when m is outside [1, 128] (the reference panics there). */
int orc_eme_transform(const uint8_t key[32], const uint8_t tweak[16], const uint8_t *in, uint8_t *out,
                      int m, int direction) {
  if (m < 1 || m > 128) return -1;
  uint8_t rk[240], L[16], zero[16] = {0}, tmp[16], MP[16], MC[16], M[16];
  orc_aes256_expand(key, rk);
  orc_aes256_encrypt(rk, zero, L);
  uint8_t Lj[128][16];
  for (int j = 0; j < m; j++) {
    dbl(L);
    memcpy(Lj[j], L, 16);
  }
#define AES(o, i) (direction ? orc_aes256_decrypt(rk, i, o) : orc_aes256_encrypt(rk, i, o))
  for (int j = 0; j < m; j++) {
    xor16(tmp, in + 16 * j, Lj[j]);
    AES(out + 16 * j, tmp);
  }
  xor16(MP, out, tweak);
  for (int j = 1; j < m; j++) xor16(MP, MP, out + 16 * j);
  AES(MC, MP);
  xor16(M, MP, MC);
  for (int j = 1; j < m; j++) {
    dbl(M);
    xor16(out + 16 * j, out + 16 * j, M);
  }
  uint8_t C0[16];
  xor16(C0, MC, tweak);
  for (int j = 1; j < m; j++) xor16(C0, C0, out + 16 * j);
  memcpy(out, C0, 16);
  for (int j = 0; j < m; j++) {
    AES(tmp, out + 16 * j);
    xor16(out + 16 * j, tmp, Lj[j]);
  }
#undef AES
  return 0;
}

/* pkcs7.Pad(16, buf) into out (capacity len+16); returns the padded length. */
int64_t orc_pkcs7_pad(const uint8_t *in, int64_t len, uint8_t *out) {
  int pad = 16 - (int)(len % 16);
  memcpy(out, in, (size_t)len);
  for (int i = 0; i < pad; i++) out[len + i] = (uint8_t)pad;
  return len + pad;
}

/* pkcs7.Unpad(16, buf): returns the unpadded length or a negative code:
 * -1 NotFound, -2 NotAMultiple, -3 TooLong, -4 TooShort, -5 NotAllTheSame (pkcs7.go:8-14). */
int64_t orc_pkcs7_unpad(const uint8_t *buf, int64_t len) {
  if (len == 0) return -1;
  if (len % 16) return -2;
  int pad = buf[len - 1];
  if (pad > 16) return -3;
  if (pad == 0) return -4;
  for (int i = 0; i < pad; i++)
    if (buf[len - 1 - i] != pad) return -5;
  return len - pad;
}
