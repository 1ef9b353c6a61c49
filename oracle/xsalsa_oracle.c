/*
 * oracle/xsalsa_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the algorithm on rclone's crypt data path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg ONLY.  Nothing in
 * rclone_amd/ links or calls this file.
 *
 * What it restates (reference = /root/reference, rclone v1.76.0):
 *   - NaCl secretbox (XSalsa20 + Poly1305) as called at backend/crypt/cipher.go:737
 *     (secretbox.Seal) and :880 (secretbox.Open).  The primitive itself lives in the
 *     third-party module golang.org/x/crypto v0.54.0 (go.mod:98: nacl/secretbox,
 *     salsa20/salsa, internal/poly1305), which is NOT vendored in the reference; this
 *     file restates the published algorithm (Salsa20/20, HSalsa20, XSalsa20, Poly1305,
 *     secretbox = tag(16) || ciphertext, Poly1305 key = keystream bytes 0..31, message
 *     XORed with keystream from byte 32).
 *   - 24-byte little-endian nonce arithmetic: nonce.carry/increment/add
 *     backend/crypt/cipher.go:647-678.
 *   - crypt file framing: header = "RCLONE\0\0" || nonce (cipher.go:34-37, :712-714),
 *     one secretbox per <=65536-byte block, nonce incremented per block (cipher.go:726-741).
 *   - sizes: EncryptedSize / DecryptedSize cipher.go:1121-1146,
 *     calculateUnderlying cipher.go:935-965.
 *
 * Pinning: tests/test_oracle.py checks this code against the reference's own golden
 * vectors (file0/file1/file16, backend/crypt/cipher_test.go:1123-1140; nonce tables
 * :757-1005; size tables :685-727; calculateUnderlying table :1433-1483) and against
 * vectors produced by libsodium 1.0.18 (an independent implementation of the same
 * NaCl secretbox spec) committed under tests/golden/ by tests/golden/make_golden.py.
 *
 * Built by oracle/Makefile into oracle/build/liboracle.so (gcc -O3 -fopenmp).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_BLOCK_DATA 65536u
#define ORC_BLOCK_HDR 16u
#define ORC_BLOCK_SIZE (ORC_BLOCK_DATA + ORC_BLOCK_HDR)
#define ORC_FILE_HDR 32u

static const uint8_t file_magic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};

static inline uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void st32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* Salsa20/20 double rounds over x[16] in place. */
static void salsa_rounds(uint32_t x[16]) {
  for (int i = 0; i < 10; i++) {
    /* column round */
    x[4] ^= rotl(x[0] + x[12], 7);  x[8] ^= rotl(x[4] + x[0], 9);
    x[12] ^= rotl(x[8] + x[4], 13); x[0] ^= rotl(x[12] + x[8], 18);
    x[9] ^= rotl(x[5] + x[1], 7);   x[13] ^= rotl(x[9] + x[5], 9);
    x[1] ^= rotl(x[13] + x[9], 13); x[5] ^= rotl(x[1] + x[13], 18);
    x[14] ^= rotl(x[10] + x[6], 7); x[2] ^= rotl(x[14] + x[10], 9);
    x[6] ^= rotl(x[2] + x[14], 13); x[10] ^= rotl(x[6] + x[2], 18);
    x[3] ^= rotl(x[15] + x[11], 7); x[7] ^= rotl(x[3] + x[15], 9);
    x[11] ^= rotl(x[7] + x[3], 13); x[15] ^= rotl(x[11] + x[7], 18);
    /* row round */
    x[1] ^= rotl(x[0] + x[3], 7);   x[2] ^= rotl(x[1] + x[0], 9);
    x[3] ^= rotl(x[2] + x[1], 13);  x[0] ^= rotl(x[3] + x[2], 18);
    x[6] ^= rotl(x[5] + x[4], 7);   x[7] ^= rotl(x[6] + x[5], 9);
    x[4] ^= rotl(x[7] + x[6], 13);  x[5] ^= rotl(x[4] + x[7], 18);
    x[11] ^= rotl(x[10] + x[9], 7); x[8] ^= rotl(x[11] + x[10], 9);
    x[9] ^= rotl(x[8] + x[11], 13); x[10] ^= rotl(x[9] + x[8], 18);
    x[12] ^= rotl(x[15] + x[14], 7); x[13] ^= rotl(x[12] + x[15], 9);
    x[14] ^= rotl(x[13] + x[12], 13); x[15] ^= rotl(x[14] + x[13], 18);
  }
}

static void salsa_setup(uint32_t x[16], const uint8_t key[32], const uint8_t in16[16]) {
  x[0] = 0x61707865u; x[5] = 0x3320646eu; x[10] = 0x79622d32u; x[15] = 0x6b206574u;
  for (int i = 0; i < 4; i++) { x[1 + i] = ld32(key + 4 * i); x[11 + i] = ld32(key + 16 + 4 * i); }
  for (int i = 0; i < 4; i++) x[6 + i] = ld32(in16 + 4 * i);
}

/* HSalsa20: subkey = words 0,5,10,15,6,7,8,9 after 20 rounds, no feed-forward. */
void orc_hsalsa20(uint8_t out[32], const uint8_t key[32], const uint8_t nonce16[16]) {
  uint32_t x[16];
  salsa_setup(x, key, nonce16);
  salsa_rounds(x);
  static const int idx[8] = {0, 5, 10, 15, 6, 7, 8, 9};
  for (int i = 0; i < 8; i++) st32(out + 4 * i, x[idx[i]]);
}

/* One 64-byte Salsa20 keystream block for (key, 8-byte nonce, 64-bit counter). */
void orc_salsa20_block(uint8_t out[64], const uint8_t key[32], const uint8_t nonce8[8], uint64_t counter) {
  uint8_t in16[16];
  memcpy(in16, nonce8, 8);
  for (int i = 0; i < 8; i++) in16[8 + i] = (uint8_t)(counter >> (8 * i));
  uint32_t x[16], y[16];
  salsa_setup(x, key, in16);
  memcpy(y, x, sizeof x);
  salsa_rounds(x);
  for (int i = 0; i < 16; i++) st32(out + 4 * i, x[i] + y[i]);
}

/* Poly1305 one-time authenticator, radix 2^26 (textbook restatement). */
void orc_poly1305(uint8_t tag[16], const uint8_t *m, size_t len, const uint8_t key[32]) {
  const uint32_t r0 = ld32(key + 0) & 0x3ffffff, r1 = (ld32(key + 3) >> 2) & 0x3ffff03,
                 r2 = (ld32(key + 6) >> 4) & 0x3ffc0ff, r3 = (ld32(key + 9) >> 6) & 0x3f03fff,
                 r4 = (ld32(key + 12) >> 8) & 0x00fffff;
  const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
  while (len > 0) {
    uint8_t blk[16];
    uint32_t hibit = 1u << 24;
    size_t take = len < 16 ? len : 16;
    memcpy(blk, m, take);
    if (take < 16) { blk[take] = 1; memset(blk + take + 1, 0, 16 - take - 1); hibit = 0; }
    h0 += ld32(blk + 0) & 0x3ffffff;
    h1 += (ld32(blk + 3) >> 2) & 0x3ffffff;
    h2 += (ld32(blk + 6) >> 4) & 0x3ffffff;
    h3 += (ld32(blk + 9) >> 6) & 0x3ffffff;
    h4 += (ld32(blk + 12) >> 8) | hibit;
    uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff; d1 += c;
    c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff; d2 += c;
    c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff; d3 += c;
    c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff; d4 += c;
    c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff; h0 += c * 5;
    c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
    m += take; len -= take;
  }
  uint32_t c;
  c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
  c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
  c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
  c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
  c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
  /* g = h + 5 - 2^130; pick g when h >= p */
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1; /* all ones when g4 did not underflow, i.e. h >= p */
  h0 = (h0 & ~mask) | (g0 & mask); h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask); h3 = (h3 & ~mask) | (g3 & mask);
  h4 = (h4 & ~mask) | (g4 & mask);
  uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14), w3 = (h3 >> 18) | (h4 << 8);
  uint64_t f;
  f = (uint64_t)w0 + ld32(key + 16); st32(tag + 0, (uint32_t)f);
  f = (uint64_t)w1 + ld32(key + 20) + (f >> 32); st32(tag + 4, (uint32_t)f);
  f = (uint64_t)w2 + ld32(key + 24) + (f >> 32); st32(tag + 8, (uint32_t)f);
  f = (uint64_t)w3 + ld32(key + 28) + (f >> 32); st32(tag + 12, (uint32_t)f);
}

/* XOR msg with the XSalsa20 stream of (subkey, nonce[16:24]) starting at stream byte `skip`. */
static void xor_stream(uint8_t *out, const uint8_t *msg, size_t n, const uint8_t subkey[32],
                       const uint8_t nonce8[8], size_t skip) {
  uint8_t ks[64];
  size_t pos = skip;
  size_t i = 0;
  while (i < n) {
    uint64_t blk = pos / 64;
    size_t off = pos % 64;
    orc_salsa20_block(ks, subkey, nonce8, blk);
    for (; off < 64 && i < n; off++, i++, pos++) out[i] = msg[i] ^ ks[off];
  }
}

/* secretbox.Seal: out = tag(16) || ct(n).  (x/crypto nacl/secretbox; call site cipher.go:737) */
void orc_secretbox_seal(uint8_t *out, const uint8_t *msg, size_t n, const uint8_t nonce[24], const uint8_t key[32]) {
  uint8_t subkey[32], ks0[64];
  orc_hsalsa20(subkey, key, nonce);
  orc_salsa20_block(ks0, subkey, nonce + 16, 0);
  xor_stream(out + 16, msg, n, subkey, nonce + 16, 32);
  orc_poly1305(out, out + 16, n, ks0);
}

/* secretbox.Open: returns 0 and writes n-16 bytes on success; -1 (writes nothing) on auth failure. (cipher.go:880) */
int orc_secretbox_open(uint8_t *out, const uint8_t *box, size_t boxlen, const uint8_t nonce[24], const uint8_t key[32]) {
  if (boxlen < 16) return -1;
  uint8_t subkey[32], ks0[64], tag[16];
  orc_hsalsa20(subkey, key, nonce);
  orc_salsa20_block(ks0, subkey, nonce + 16, 0);
  orc_poly1305(tag, box + 16, boxlen - 16, ks0);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= tag[i] ^ box[i];
  if (diff) return -1;
  xor_stream(out, box + 16, boxlen - 16, subkey, nonce + 16, 32);
  return 0;
}

/* nonce.carry(i) cipher.go:647-658 */
void orc_nonce_carry(uint8_t n[24], int i) {
  for (; i < 24; i++) {
    uint8_t digit = n[i];
    uint8_t nd = (uint8_t)(digit + 1);
    n[i] = nd;
    if (nd >= digit) break;
  }
}
/* nonce.increment cipher.go:660-663 */
void orc_nonce_increment(uint8_t n[24]) { orc_nonce_carry(n, 0); }
/* nonce.add cipher.go:665-678 */
void orc_nonce_add(uint8_t n[24], uint64_t x) {
  uint16_t carry = 0;
  for (int i = 0; i < 8; i++) {
    uint8_t digit = n[i];
    uint8_t xd = (uint8_t)x;
    x >>= 8;
    carry = (uint16_t)(carry + digit + xd);
    n[i] = (uint8_t)carry;
    carry >>= 8;
  }
  if (carry != 0) orc_nonce_carry(n, 8);
}

/* EncryptedSize cipher.go:1121-1129 */
int64_t orc_encrypted_size(int64_t size) {
  int64_t blocks = size / ORC_BLOCK_DATA, residue = size % ORC_BLOCK_DATA;
  int64_t e = ORC_FILE_HDR + blocks * (int64_t)ORC_BLOCK_SIZE;
  if (residue != 0) e += ORC_BLOCK_HDR + residue;
  return e;
}
/* DecryptedSize cipher.go:1131-1146; returns -1 TooShort, -2 BadHeader */
int64_t orc_decrypted_size(int64_t size) {
  size -= ORC_FILE_HDR;
  if (size < 0) return -1;
  int64_t blocks = size / ORC_BLOCK_SIZE, residue = size % ORC_BLOCK_SIZE;
  int64_t d = blocks * ORC_BLOCK_DATA;
  if (residue != 0) {
    residue -= ORC_BLOCK_HDR;
    if (residue <= 0) return -2;
  }
  return d + residue;
}
/* calculateUnderlying cipher.go:935-965; out = {underlyingOffset, underlyingLimit, discard, blocks} */
void orc_calculate_underlying(int64_t offset, int64_t limit, int64_t out[4]) {
  int64_t blocks = offset / ORC_BLOCK_DATA, discard = offset % ORC_BLOCK_DATA;
  int64_t uoff = ORC_FILE_HDR + blocks * (int64_t)ORC_BLOCK_SIZE;
  int64_t ulim = -1;
  if (limit >= 0) {
    int64_t bytes_to_read = limit - (ORC_BLOCK_DATA - discard);
    int64_t blocks_to_read = 1;
    if (bytes_to_read > 0) {
      int64_t extra = bytes_to_read / ORC_BLOCK_DATA, end = bytes_to_read % ORC_BLOCK_DATA;
      if (end != 0) extra++;
      blocks_to_read += extra;
    }
    ulim = blocks_to_read * (int64_t)ORC_BLOCK_SIZE;
  }
  out[0] = uoff; out[1] = ulim; out[2] = discard; out[3] = blocks;
}

/* Whole-file encrypt mirroring encrypter framing (cipher.go:694-745): header then one
 * secretbox per 65536-byte block with the nonce incremented per block.  out must hold
 * orc_encrypted_size(len) bytes.  Blocks are independent, so this runs them in parallel. */
void orc_encrypt_file(uint8_t *out, const uint8_t *in, int64_t len, const uint8_t nonce0[24], const uint8_t key[32]) {
  memcpy(out, file_magic, 8);
  memcpy(out + 8, nonce0, 24);
  int64_t nblocks = (len + ORC_BLOCK_DATA - 1) / ORC_BLOCK_DATA;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblocks; b++) {
    uint8_t nonce[24];
    memcpy(nonce, nonce0, 24);
    orc_nonce_add(nonce, (uint64_t)b);
    int64_t n = len - b * (int64_t)ORC_BLOCK_DATA;
    if (n > ORC_BLOCK_DATA) n = ORC_BLOCK_DATA;
    orc_secretbox_seal(out + ORC_FILE_HDR + b * (int64_t)ORC_BLOCK_SIZE, in + b * (int64_t)ORC_BLOCK_DATA,
                       (size_t)n, nonce, key);
  }
}

/* Whole-file decrypt mirroring decrypter block semantics (cipher.go:793-898).
 * Returns plaintext length, or -1 too short (ErrorEncryptedFileTooShort), -2 bad magic,
 * -3 truncated block header (ErrorEncryptedFileBadHeader), -4 bad block
 * (ErrorEncryptedBadBlock; *bad_block = first failing block).  With pass_bad_blocks
 * a failing block is zero-filled instead. */
int64_t orc_decrypt_file(uint8_t *out, const uint8_t *in, int64_t len, const uint8_t key[32],
                         int pass_bad_blocks, int64_t *bad_block) {
  if (len < (int64_t)ORC_FILE_HDR) return -1;
  if (memcmp(in, file_magic, 8) != 0) return -2;
  const uint8_t *nonce0 = in + 8;
  int64_t body = len - ORC_FILE_HDR;
  int64_t nblocks = (body + ORC_BLOCK_SIZE - 1) / ORC_BLOCK_SIZE;
  int64_t first_bad = -1, first_short = -1;
  for (int64_t b = 0; b < nblocks; b++) {
    int64_t n = body - b * (int64_t)ORC_BLOCK_SIZE;
    if (n > ORC_BLOCK_SIZE) n = ORC_BLOCK_SIZE;
    if (n <= (int64_t)ORC_BLOCK_HDR) { first_short = b; nblocks = b; break; }
  }
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblocks; b++) {
    uint8_t nonce[24];
    memcpy(nonce, nonce0, 24);
    orc_nonce_add(nonce, (uint64_t)b);
    int64_t n = body - b * (int64_t)ORC_BLOCK_SIZE;
    if (n > ORC_BLOCK_SIZE) n = ORC_BLOCK_SIZE;
    uint8_t *dst = out + b * (int64_t)ORC_BLOCK_DATA;
    if (orc_secretbox_open(dst, in + ORC_FILE_HDR + b * (int64_t)ORC_BLOCK_SIZE, (size_t)n, nonce, key) != 0) {
      memset(dst, 0, (size_t)(n - ORC_BLOCK_HDR));
#pragma omp critical
      { if (first_bad < 0 || b < first_bad) first_bad = b; }
    }
  }
  if (first_bad >= 0 && !pass_bad_blocks) { if (bad_block) *bad_block = first_bad; return -4; }
  if (first_short >= 0) return -3;
  int64_t plain = orc_decrypted_size(len);
  return plain;
}

/* CPU baseline helper: seal `nblocks` independent full 65536-byte blocks laid out
 * contiguously, block i with nonce0 + i, output in wire layout (stride 65552).
 * Uses all OpenMP threads; returns the thread count used. */
int orc_seal_blocks(uint8_t *out, const uint8_t *in, int64_t nblocks, const uint8_t nonce0[24], const uint8_t key[32]) {
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(static)
    for (int64_t b = 0; b < nblocks; b++) {
      uint8_t nonce[24];
      memcpy(nonce, nonce0, 24);
      orc_nonce_add(nonce, (uint64_t)b);
      orc_secretbox_seal(out + b * (int64_t)ORC_BLOCK_SIZE, in + b * (int64_t)ORC_BLOCK_DATA, ORC_BLOCK_DATA, nonce, key);
    }
  }
  return threads;
}

/* CPU baseline helper: open `nblocks` wire blocks; ok[i] = 1 on success. */
int orc_open_blocks(uint8_t *out, uint8_t *ok, const uint8_t *in, int64_t nblocks, const uint8_t nonce0[24], const uint8_t key[32]) {
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(static)
    for (int64_t b = 0; b < nblocks; b++) {
      uint8_t nonce[24];
      memcpy(nonce, nonce0, 24);
      orc_nonce_add(nonce, (uint64_t)b);
      ok[b] = orc_secretbox_open(out + b * (int64_t)ORC_BLOCK_DATA, in + b * (int64_t)ORC_BLOCK_SIZE, ORC_BLOCK_SIZE, nonce, key) == 0;
    }
  }
  return threads;
}

/* Descriptor-mode batches (test checker for xs_seal_batch_dev / xs_open_batch_dev): each
 * descriptor is one secretbox of `len` bytes with its own 24-byte nonce, i.e. one
 * encrypter.Read block (cipher.go:737) / decrypter.fillBuffer block (cipher.go:880).  Same
 * 48-byte layout as xs_block_desc.  OpenMP over descriptors; returns the thread count. */
typedef struct orc_desc {
  uint64_t src_off;
  uint64_t dst_off;
  uint32_t len;
  uint32_t reserved;
  uint8_t nonce[24];
} orc_desc;

int orc_seal_desc(uint8_t *dst, const uint8_t *src, const orc_desc *d, int64_t n, const uint8_t key[32]) {
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; i++)
      orc_secretbox_seal(dst + d[i].dst_off, src + d[i].src_off, d[i].len, d[i].nonce, key);
  }
  return threads;
}

int orc_open_desc(uint8_t *dst, uint8_t *ok, const uint8_t *src, const orc_desc *d, int64_t n, const uint8_t key[32]) {
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; i++)
      ok[i] = orc_secretbox_open(dst + d[i].dst_off, src + d[i].src_off, (size_t)d[i].len + ORC_BLOCK_HDR, d[i].nonce, key) == 0;
  }
  return threads;
}
