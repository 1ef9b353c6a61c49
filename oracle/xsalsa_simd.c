/*
 * oracle/xsalsa_simd.c -- TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg.
 *
 * A vectorised CPU restatement of the same secretbox (XSalsa20 + Poly1305, call sites
 * backend/crypt/cipher.go:737 Seal, :880 Open) as oracle/xsalsa_oracle.c, so that the CPU
 * baseline is a tuned CPU path rather than the textbook one:
 *   - Salsa20/20 counter-parallel across SIMD lanes: 16 keystream blocks per AVX-512 pass
 *     (native 32-bit rotates), 8 per AVX2 pass; selected at run time (orc_simd_level);
 *   - Poly1305 in radix 2^44 with 64x64->128-bit products (three limbs, the usual 64-bit
 *     formulation), instead of the oracle's radix-2^26 32-bit limbs;
 *   - OpenMP over 64 KiB blocks, as the scalar oracle.
 * tests/test_oracle_simd.py checks it byte-for-byte against xsalsa_oracle.c (every AVX level the
 * host has, lengths 0..200 and whole blocks, tampered opens).  Nothing in rclone_amd/ links it.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define SB_DATA 65536u
#define SB_HDR 16u
#define SB_SIZE (SB_DATA + SB_HDR)

void orc_hsalsa20(uint8_t out[32], const uint8_t key[32], const uint8_t nonce16[16]);
void orc_nonce_add(uint8_t n[24], uint64_t x);

static inline uint32_t le32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t le64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* ------------------------------------------------------------------ Poly1305, radix 2^44 */
typedef unsigned __int128 u128;
#define M44 0xfffffffffffULL
#define M42 0x3ffffffffffULL

static void poly1305_44(uint8_t tag[16], const uint8_t *m, size_t len, const uint8_t key[32]) {
  const uint64_t t0 = le64(key), t1 = le64(key + 8);
  const uint64_t r0 = t0 & 0xffc0fffffffULL, r1 = ((t0 >> 44) | (t1 << 20)) & 0xfffffc0ffffULL,
                 r2 = (t1 >> 24) & 0x00ffffffc0fULL;
  const uint64_t s1 = r1 * (5 << 2), s2 = r2 * (5 << 2);
  uint64_t h0 = 0, h1 = 0, h2 = 0;
  while (len > 0) {
    uint8_t blk[16];
    const uint8_t *p = m;
    uint64_t hibit = 1ULL << 40;
    size_t take = 16;
    if (len < 16) {
      take = len;
      memcpy(blk, m, len);
      blk[len] = 1;
      memset(blk + len + 1, 0, 15 - len);
      p = blk;
      hibit = 0;
    }
    const uint64_t m0 = le64(p), m1 = le64(p + 8);
    h0 += m0 & M44;
    h1 += ((m0 >> 44) | (m1 << 20)) & M44;
    h2 += ((m1 >> 24) & M42) | hibit;
    const u128 d0 = (u128)h0 * r0 + (u128)h1 * s2 + (u128)h2 * s1;
    u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * s2;
    u128 d2 = (u128)h0 * r2 + (u128)h1 * r1 + (u128)h2 * r0;
    uint64_t c = (uint64_t)(d0 >> 44);
    h0 = (uint64_t)d0 & M44;
    d1 += c;
    c = (uint64_t)(d1 >> 44);
    h1 = (uint64_t)d1 & M44;
    d2 += c;
    c = (uint64_t)(d2 >> 42);
    h2 = (uint64_t)d2 & M42;
    h0 += c * 5;
    c = h0 >> 44;
    h0 &= M44;
    h1 += c;
    m += take;
    len -= take;
  }
  uint64_t c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  /* g = h + 5 - 2^130: take it when it does not underflow (h >= p) */
  uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
  uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
  uint64_t g2 = h2 + c - (1ULL << 42);
  const uint64_t take_g = (g2 >> 63) - 1;
  h0 = (h0 & ~take_g) | (g0 & take_g);
  h1 = (h1 & ~take_g) | (g1 & take_g);
  h2 = (h2 & ~take_g) | (g2 & take_g);
  /* + s (mod 2^128) */
  const uint64_t p0 = le64(key + 16), p1 = le64(key + 24);
  h0 += p0 & M44; c = h0 >> 44; h0 &= M44;
  h1 += (((p0 >> 44) | (p1 << 20)) & M44) + c; c = h1 >> 44; h1 &= M44;
  h2 += ((p1 >> 24) & M42) + c; h2 &= M42;
  const uint64_t w0 = h0 | (h1 << 44), w1 = (h1 >> 20) | (h2 << 24);
  memcpy(tag, &w0, 8);
  memcpy(tag + 8, &w1, 8);
}

/* ------------------------------------------------------------------ Salsa20, lane-parallel */
#define SIG0 0x61707865u
#define SIG1 0x3320646eu
#define SIG2 0x79622d32u
#define SIG3 0x6b206574u

#define QR(V, ADD, XOR, ROT, a, b, c, d)        \
  do {                                           \
    b = XOR(b, ROT(ADD(a, d), 7));               \
    c = XOR(c, ROT(ADD(b, a), 9));               \
    d = XOR(d, ROT(ADD(c, b), 13));              \
    a = XOR(a, ROT(ADD(d, c), 18));              \
  } while (0)
#define DOUBLE_ROUND(V, ADD, XOR, ROT, x)                          \
  do {                                                              \
    QR(V, ADD, XOR, ROT, x[0], x[4], x[8], x[12]);                  \
    QR(V, ADD, XOR, ROT, x[5], x[9], x[13], x[1]);                  \
    QR(V, ADD, XOR, ROT, x[10], x[14], x[2], x[6]);                 \
    QR(V, ADD, XOR, ROT, x[15], x[3], x[7], x[11]);                 \
    QR(V, ADD, XOR, ROT, x[0], x[1], x[2], x[3]);                   \
    QR(V, ADD, XOR, ROT, x[5], x[6], x[7], x[4]);                   \
    QR(V, ADD, XOR, ROT, x[10], x[11], x[8], x[9]);                 \
    QR(V, ADD, XOR, ROT, x[15], x[12], x[13], x[14]);               \
  } while (0)

/* 16 keystream blocks (counters ctr..ctr+15) of (subkey, nonce8) into ks[16][64] */
__attribute__((target("avx512f"))) static void salsa_x16(uint8_t ks[16 * 64], const uint32_t k[8], uint32_t n0,
                                                         uint32_t n1, uint64_t ctr) {
#define A512(a, b) _mm512_add_epi32(a, b)
#define X512(a, b) _mm512_xor_si512(a, b)
#define R512(v, n) _mm512_rol_epi32(v, n)
  __m512i x[16], y[16];
  const uint32_t in[16] = {SIG0, k[0], k[1], k[2], k[3], SIG1, n0, n1, 0, 0, SIG2, k[4], k[5], k[6], k[7], SIG3};
  for (int i = 0; i < 16; i++) x[i] = _mm512_set1_epi32((int)in[i]);
  const __m512i lanes = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  const __m512i lo = _mm512_add_epi32(_mm512_set1_epi32((int)(uint32_t)ctr), lanes);
  /* carry into the high word per lane */
  const __mmask16 wrap = _mm512_cmplt_epu32_mask(lo, _mm512_set1_epi32((int)(uint32_t)ctr));
  x[8] = lo;
  x[9] = _mm512_mask_add_epi32(_mm512_set1_epi32((int)(uint32_t)(ctr >> 32)), wrap,
                               _mm512_set1_epi32((int)(uint32_t)(ctr >> 32)), _mm512_set1_epi32(1));
  for (int i = 0; i < 16; i++) y[i] = x[i];
  for (int r = 0; r < 10; r++) DOUBLE_ROUND(512, A512, X512, R512, x);
  for (int i = 0; i < 16; i++) x[i] = _mm512_add_epi32(x[i], y[i]);
  /* 16x16 transpose (word i of lane j -> ks[64 j + 4 i]): 32-bit and 64-bit unpacks inside the
   * 128-bit lanes, then two 128-bit lane shuffles */
  __m512i t[16], u[16];
  for (int k = 0; k < 8; k++) {
    t[2 * k] = _mm512_unpacklo_epi32(x[2 * k], x[2 * k + 1]);
    t[2 * k + 1] = _mm512_unpackhi_epi32(x[2 * k], x[2 * k + 1]);
  }
  for (int m = 0; m < 4; m++) { /* u[4m + c], lane L: rows 4m..4m+3 at column 4L + c */
    u[4 * m + 0] = _mm512_unpacklo_epi64(t[4 * m], t[4 * m + 2]);
    u[4 * m + 1] = _mm512_unpackhi_epi64(t[4 * m], t[4 * m + 2]);
    u[4 * m + 2] = _mm512_unpacklo_epi64(t[4 * m + 1], t[4 * m + 3]);
    u[4 * m + 3] = _mm512_unpackhi_epi64(t[4 * m + 1], t[4 * m + 3]);
  }
  for (int c = 0; c < 4; c++) {
    const __m512i alo = _mm512_shuffle_i32x4(u[c], u[4 + c], 0x44), ahi = _mm512_shuffle_i32x4(u[c], u[4 + c], 0xEE);
    const __m512i blo = _mm512_shuffle_i32x4(u[8 + c], u[12 + c], 0x44),
                  bhi = _mm512_shuffle_i32x4(u[8 + c], u[12 + c], 0xEE);
    _mm512_store_si512((void *)(ks + 64 * (0 + c)), _mm512_shuffle_i32x4(alo, blo, 0x88));
    _mm512_store_si512((void *)(ks + 64 * (4 + c)), _mm512_shuffle_i32x4(alo, blo, 0xDD));
    _mm512_store_si512((void *)(ks + 64 * (8 + c)), _mm512_shuffle_i32x4(ahi, bhi, 0x88));
    _mm512_store_si512((void *)(ks + 64 * (12 + c)), _mm512_shuffle_i32x4(ahi, bhi, 0xDD));
  }
#undef A512
#undef X512
#undef R512
}

/* 8 keystream blocks (counters ctr..ctr+7) into ks[8][64] */
__attribute__((target("avx2"))) static void salsa_x8(uint8_t ks[8 * 64], const uint32_t k[8], uint32_t n0, uint32_t n1,
                                                     uint64_t ctr) {
#define A256(a, b) _mm256_add_epi32(a, b)
#define X256(a, b) _mm256_xor_si256(a, b)
#define R256(v, n) _mm256_or_si256(_mm256_slli_epi32(v, n), _mm256_srli_epi32(v, 32 - (n)))
  __m256i x[16], y[16];
  const uint32_t in[16] = {SIG0, k[0], k[1], k[2], k[3], SIG1, n0, n1, 0, 0, SIG2, k[4], k[5], k[6], k[7], SIG3};
  for (int i = 0; i < 16; i++) x[i] = _mm256_set1_epi32((int)in[i]);
  uint32_t lo[8], hi[8];
  for (int j = 0; j < 8; j++) {
    lo[j] = (uint32_t)(ctr + (uint64_t)j);
    hi[j] = (uint32_t)((ctr + (uint64_t)j) >> 32);
  }
  x[8] = _mm256_loadu_si256((const __m256i *)lo);
  x[9] = _mm256_loadu_si256((const __m256i *)hi);
  for (int i = 0; i < 16; i++) y[i] = x[i];
  for (int r = 0; r < 10; r++) DOUBLE_ROUND(256, A256, X256, R256, x);
  for (int i = 0; i < 16; i++) x[i] = _mm256_add_epi32(x[i], y[i]);
  /* two 8x8 transposes (words 0..7 and 8..15; word i of lane j -> ks[64 j + 4 i]) */
  for (int half = 0; half < 2; half++) {
    const __m256i *r = x + 8 * half;
    __m256i t[8], u[8];
    for (int k = 0; k < 4; k++) {
      t[2 * k] = _mm256_unpacklo_epi32(r[2 * k], r[2 * k + 1]);
      t[2 * k + 1] = _mm256_unpackhi_epi32(r[2 * k], r[2 * k + 1]);
    }
    for (int m = 0; m < 2; m++) {
      u[4 * m + 0] = _mm256_unpacklo_epi64(t[4 * m], t[4 * m + 2]);
      u[4 * m + 1] = _mm256_unpackhi_epi64(t[4 * m], t[4 * m + 2]);
      u[4 * m + 2] = _mm256_unpacklo_epi64(t[4 * m + 1], t[4 * m + 3]);
      u[4 * m + 3] = _mm256_unpackhi_epi64(t[4 * m + 1], t[4 * m + 3]);
    }
    for (int c = 0; c < 4; c++) {
      _mm256_store_si256((__m256i *)(ks + 64 * c + 32 * half), _mm256_permute2x128_si256(u[c], u[4 + c], 0x20));
      _mm256_store_si256((__m256i *)(ks + 64 * (4 + c) + 32 * half), _mm256_permute2x128_si256(u[c], u[4 + c], 0x31));
    }
  }
#undef A256
#undef X256
#undef R256
}

static int g_level = -1; /* forced level (tests) or -1: detect */

/* 2: AVX-512, 1: AVX2, 0: neither (the scalar oracle is then the baseline) */
int orc_simd_level(void) {
  if (g_level >= 0) return g_level;
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f")) return 2;
  if (__builtin_cpu_supports("avx2")) return 1;
  return 0;
}

/* tests: force a level (<= the detected one); -1 restores detection */
void orc_simd_force(int level) { g_level = level; }

/* XOR msg (n bytes) with the stream of (subkey, nonce8) from stream byte 32 on: the message starts
 * at keystream block 0 byte 32.  ks0 receives keystream block 0 (the Poly1305 key is bytes 0..31). */
static void xor_stream_simd(uint8_t *out, const uint8_t *msg, size_t n, const uint8_t subkey[32],
                            const uint8_t nonce8[8], uint8_t ks0[64], int level) {
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = le32(subkey + 4 * i);
  const uint32_t n0 = le32(nonce8), n1 = le32(nonce8 + 4);
  const int lanes = level >= 2 ? 16 : 8;
  uint8_t ks[16 * 64] __attribute__((aligned(64)));
  size_t done = 0;  /* message bytes written */
  uint64_t blk = 0; /* next keystream block */
  while (done < n || blk == 0) {
    if (level >= 2) salsa_x16(ks, k, n0, n1, blk);
    else salsa_x8(ks, k, n0, n1, blk);
    size_t from = 0;
    if (blk == 0) {
      memcpy(ks0, ks, 64);
      from = 32;
    }
    const size_t avail = (size_t)lanes * 64 - from;
    const size_t take = n - done < avail ? n - done : avail;
    for (size_t i = 0; i < take; i++) out[done + i] = msg[done + i] ^ ks[from + i];
    done += take;
    blk += (uint64_t)lanes;
  }
}

static void seal_one(uint8_t *out, const uint8_t *msg, size_t n, const uint8_t nonce[24], const uint8_t key[32],
                     int level) {
  uint8_t subkey[32], ks0[64];
  orc_hsalsa20(subkey, key, nonce);
  xor_stream_simd(out + 16, msg, n, subkey, nonce + 16, ks0, level);
  poly1305_44(out, out + 16, n, ks0);
}

static int open_one(uint8_t *out, const uint8_t *box, size_t boxlen, const uint8_t nonce[24], const uint8_t key[32],
                    int level) {
  if (boxlen < 16) return -1;
  uint8_t subkey[32], ks0[64], tag[16];
  orc_hsalsa20(subkey, key, nonce);
  /* keystream block 0 first (the Poly1305 key); the tag is checked before any output */
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = le32(subkey + 4 * i);
  {
    uint8_t ks[16 * 64] __attribute__((aligned(64)));
    if (level >= 2) salsa_x16(ks, k, le32(nonce + 16), le32(nonce + 20), 0);
    else salsa_x8(ks, k, le32(nonce + 16), le32(nonce + 20), 0);
    memcpy(ks0, ks, 64);
  }
  poly1305_44(tag, box + 16, boxlen - 16, ks0);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= tag[i] ^ box[i];
  if (diff) return -1;
  xor_stream_simd(out, box + 16, boxlen - 16, subkey, nonce + 16, ks0, level);
  return 0;
}

/* secretbox.Seal / Open, vectorised (falls back to level 1 code only when the CPU has AVX2) */
void orc_simd_secretbox_seal(uint8_t *out, const uint8_t *msg, size_t n, const uint8_t nonce[24],
                             const uint8_t key[32]) {
  seal_one(out, msg, n, nonce, key, orc_simd_level());
}

int orc_simd_secretbox_open(uint8_t *out, const uint8_t *box, size_t boxlen, const uint8_t nonce[24],
                            const uint8_t key[32]) {
  return open_one(out, box, boxlen, nonce, key, orc_simd_level());
}

/* Full 64 KiB blocks of one object (block i: nonce0 + i), OpenMP over blocks; returns threads used
 * (0 when the CPU has no AVX2: the caller uses the scalar oracle). */
int orc_simd_seal_blocks(uint8_t *out, const uint8_t *in, int64_t nblocks, const uint8_t nonce0[24],
                         const uint8_t key[32]) {
  const int level = orc_simd_level();
  if (level == 0) return 0;
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(static)
    for (int64_t b = 0; b < nblocks; b++) {
      uint8_t n[24];
      memcpy(n, nonce0, 24);
      orc_nonce_add(n, (uint64_t)b);
      seal_one(out + b * SB_SIZE, in + b * SB_DATA, SB_DATA, n, key, level);
    }
  }
  return threads;
}

int orc_simd_open_blocks(uint8_t *out, uint8_t *ok, const uint8_t *in, int64_t nblocks, const uint8_t nonce0[24],
                         const uint8_t key[32]) {
  const int level = orc_simd_level();
  if (level == 0) return 0;
  int threads = 1;
#pragma omp parallel
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
#pragma omp for schedule(static)
    for (int64_t b = 0; b < nblocks; b++) {
      uint8_t n[24];
      memcpy(n, nonce0, 24);
      orc_nonce_add(n, (uint64_t)b);
      ok[b] = open_one(out + b * SB_DATA, in + b * SB_SIZE, SB_SIZE, n, key, level) == 0;
      if (!ok[b]) memset(out + b * SB_DATA, 0, SB_DATA);
    }
  }
  return threads;
}

/* ------------------------------------------------------------------ generated object sets
 * The synthetic objects of BASELINE configs[1] and configs[3] are generated in HBM by
 * xs_fill_blocks_dev: 64-bit word w of global 64 KiB block g is SplitMix64 word g*8192 + w of
 * (seed), i.e. mix(seed + (g*8192 + w + 1) * golden) (rclone_amd/testdata.py).  Block g is sealed
 * with nonce0 + g (cipher.go:665-678 nonce.add, :737 secretbox.Seal).
 *
 * orc_simd_seal_gen regenerates that plaintext here for blocks g = first + j*stride (j < nblocks),
 * seals each one, writes the wire blocks to out when out != NULL (j-th block at out + j*65552) and
 * returns through tagsum[2] the order-independent tag digest the GPU harness reports: the sum mod
 * 2^64 of each tag's two little-endian 64-bit halves (rclone_amd/objectset.py tag_digest).  With
 * out == NULL nothing but the digest is kept, so a 1 TiB set (2^24 blocks) streams through 64 KiB
 * per thread.  nonces != NULL replaces nonce0 + g by nonces[24 j..24 j+23] (one-block objects, each with
 * its own nonce: configs[1]'s independent-object form).  Returns the OpenMP threads used, 0 when the
 * CPU has no AVX2. */
static inline uint64_t splitmix_word(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void orc_gen_block(uint8_t out[SB_DATA], uint64_t seed, uint64_t g) {
  uint64_t w[SB_DATA / 8];
  const uint64_t base = g * (SB_DATA / 8);
  for (uint64_t i = 0; i < SB_DATA / 8; i++) w[i] = splitmix_word(seed, base + i);
  memcpy(out, w, SB_DATA); /* little-endian host: word i -> bytes 8i..8i+7 */
}

int orc_simd_seal_gen(uint8_t *out, int64_t nblocks, uint64_t first, uint64_t stride, uint64_t seed,
                      const uint8_t nonce0[24], const uint8_t *nonces, const uint8_t key[32], uint64_t tagsum[2]) {
  const int level = orc_simd_level();
  if (level == 0) return 0;
  int threads = 1;
  uint64_t s0 = 0, s1 = 0;
#pragma omp parallel reduction(+ : s0, s1)
  {
#ifdef _OPENMP
#pragma omp single
    threads = omp_get_num_threads();
#endif
    uint8_t plain[SB_DATA] __attribute__((aligned(64)));
    uint8_t wire[SB_SIZE] __attribute__((aligned(64)));
#pragma omp for schedule(static)
    for (int64_t j = 0; j < nblocks; j++) {
      const uint64_t g = first + (uint64_t)j * stride;
      uint8_t n[24];
      if (nonces) {
        memcpy(n, nonces + (size_t)j * 24, 24);
      } else {
        memcpy(n, nonce0, 24);
        orc_nonce_add(n, g);
      }
      orc_gen_block(plain, seed, g);
      uint8_t *dst = out ? out + (size_t)j * SB_SIZE : wire;
      seal_one(dst, plain, SB_DATA, n, key, level);
      s0 += le64(dst);
      s1 += le64(dst + 8);
    }
  }
  tagsum[0] = s0;
  tagsum[1] = s1;
  return threads;
}

/* Windowed open, the CPU counterpart of a ranged read (cipher.go:972-1034 RangeSeek, then a short
 * Read): the tag is verified over the whole block (secretbox.Open needs every ciphertext byte), but
 * only the keystream blocks covering plaintext bytes [lo, hi) are generated and only those bytes of
 * out are written.  Returns 0 when authentic, -1 otherwise (out untouched).  The reference's Go path
 * decrypts the whole block (orc_simd_secretbox_open); this is the tuned CPU baseline beside the
 * GPU's windowed open (tools/seek_latency.cpp over tests/native/cpu_engine.cpp). */
int orc_simd_open_window(uint8_t *out, const uint8_t *box, size_t boxlen, const uint8_t nonce[24],
                         const uint8_t key[32], size_t lo, size_t hi) {
  const int level = orc_simd_level();
  if (boxlen < 16) return -1;
  const size_t n = boxlen - 16;
  if (hi > n) hi = n;
  uint8_t subkey[32], ks0[64], tag[16];
  orc_hsalsa20(subkey, key, nonce);
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = le32(subkey + 4 * i);
  const uint32_t n0 = le32(nonce + 16), n1 = le32(nonce + 20);
  uint8_t ks[16 * 64] __attribute__((aligned(64)));
  if (level >= 2) salsa_x16(ks, k, n0, n1, 0);
  else salsa_x8(ks, k, n0, n1, 0);
  memcpy(ks0, ks, 64);
  poly1305_44(tag, box + 16, n, ks0);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= tag[i] ^ box[i];
  if (diff) return -1;
  if (lo >= hi) return 0;
  /* plaintext byte i takes keystream byte i + 32 */
  const size_t lanes = level >= 2 ? 16 : 8;
  uint64_t blk = (lo + 32) / 64;
  size_t i = lo;
  while (i < hi) {
    if (level >= 2) salsa_x16(ks, k, n0, n1, blk);
    else salsa_x8(ks, k, n0, n1, blk);
    const size_t base = (size_t)blk * 64; /* stream offset of ks[0] */
    const size_t end = base + lanes * 64 - 32 < hi ? base + lanes * 64 - 32 : hi;
    for (; i < end; i++) out[i] = box[16 + i] ^ ks[i + 32 - base];
    blk += lanes;
  }
  return 0;
}

/* The crypt file (cipher.go:694-758 encrypter: "RCLONE\0\0" || nonce || sealed blocks, block j with
 * nonce + j) of an object whose plaintext is the SplitMix64 stream of `seed` (word k = mix(seed +
 * (k+1)*golden), little-endian, truncated to `size` bytes: tools/e2e_sync.cpp's tree files,
 * rclone_amd/testdata.py splitmix64_bytes).  out holds orc_encrypted_size(size) bytes.  Single
 * threaded (callers run many objects at once).  Returns 0, or -1 when the CPU has no AVX2. */
int orc_simd_encrypt_gen_file(uint8_t *out, uint64_t seed, uint64_t size, const uint8_t nonce0[24],
                              const uint8_t key[32]) {
  static const uint8_t magic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};
  const int level = orc_simd_level();
  if (level == 0) return -1;
  memcpy(out, magic, 8);
  memcpy(out + 8, nonce0, 24);
  uint64_t w[SB_DATA / 8];
  uint8_t *body = out + 32;
  for (uint64_t j = 0; j * SB_DATA < size; j++) {
    const uint64_t len = size - j * SB_DATA < SB_DATA ? size - j * SB_DATA : SB_DATA;
    const uint64_t words = (len + 7) / 8, base = j * (SB_DATA / 8);
    for (uint64_t i = 0; i < words; i++) w[i] = splitmix_word(seed, base + i);
    uint8_t n[24];
    memcpy(n, nonce0, 24);
    orc_nonce_add(n, j);
    seal_one(body + j * SB_SIZE, (const uint8_t *)w, len, n, key, level);
  }
  return 0;
}
