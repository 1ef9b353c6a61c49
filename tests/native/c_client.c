/* TEST INFRASTRUCTURE: a C11 client of librclone_crypt.so through the C half of the cgo binding,
 * integration/gpucipher/shim.c, compiled exactly as cgo would (-std=c11, the package's include
 * path, a stand-in _cgo_export.h).  The "Go side" -- goRead / goClose / goRangeSeek / goOpen, the
 * //export functions of gpucipher.go -- is played here by C functions that behave like them: a
 * handle table of small integers (runtime/cgo.Handle values 1, 2, ...), never pointers, and
 * reader / opener errors returned as codes >= RC_USER_BASE that must come back unchanged.  The
 * checks use only entry points that need no GPU (the header, error and nonce paths of cipher.go,
 * DecryptDataSeek's open callback, sizes, nonce arithmetic, the key derivation, host-only name
 * modes), so this runs in the CPU suite; tests/test_native_sanitize.py runs it.
 * Reference: librclone/librclone.go:22-104 (the reference's cgo precedent), backend/crypt/cipher.go. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "_cgo_export.h"
#include "rclone_crypt_gpu.h"

/* shim.c */
rc_reader gpucipher_reader(uintptr_t h, int closer, int range_seeker);
rc_encrypter *gpucipher_encrypt(rc_cipher *c, uintptr_t in, const uint8_t *nonce, int32_t *err);
rc_decrypter *gpucipher_decrypt(rc_cipher *c, uintptr_t rc, int range_seeker, int32_t *err);
rc_decrypter *gpucipher_decrypt_seek(rc_cipher *c, uintptr_t open_state, int64_t offset, int64_t limit, int32_t *err,
                                     int32_t *wrapped);
int32_t gpucipher_compute_hash(rc_cipher *c, uintptr_t src, int closer, const uint8_t *nonce, uint8_t *md5);
int32_t gpucipher_hash_batch(rc_cipher *c, uint64_t n, const uintptr_t *srcs, uint64_t n_nonces, const uint8_t *nonces,
                             uint8_t *md5, int32_t *errs);

static int failures = 0;
#define CHECK(c, msg)                          \
  do {                                         \
    if (!(c)) {                                \
      fprintf(stderr, "FAIL: %s\n", msg);      \
      failures++;                              \
    }                                          \
  } while (0)

/* ---- the "Go side": a handle table, like runtime/cgo.Handle (values 1, 2, ...) */
typedef struct {
  const uint8_t *p;
  int64_t n, pos;
  int32_t fail; /* returned instead of data once pos == n (RC_EOF for a clean end) */
  int reads, closes;
} box;
static box boxes[8];

int64_t goRead(uintptr_t h, uint8_t *p, int64_t n, int32_t *err) {
  box *b = &boxes[h];
  b->reads++;
  int64_t k = b->n - b->pos;
  if (k > n) k = n;
  if (k > 0) memcpy(p, b->p + b->pos, (size_t)k);
  b->pos += k;
  *err = (k == 0) ? b->fail : RC_NIL;
  return k;
}
int32_t goClose(uintptr_t h) {
  boxes[h].closes++;
  return RC_NIL;
}
int32_t goRangeSeek(uintptr_t h, int64_t offset, int32_t whence, int64_t limit) {
  (void)whence;
  (void)limit;
  boxes[h].pos = offset;
  return RC_NIL;
}
static int64_t open_calls[4][2];
static int nopen = 0, reopen_calls = 0;
int32_t goOpen(uintptr_t h, int64_t off, int64_t lim, rc_reader *out) {
  if (h == 100) { /* the first open serves a valid header (box 0, no RangeSeeker); the re-open fails */
    if (reopen_calls++ == 0) {
      *out = gpucipher_reader(0, 1, 0);
      return RC_NIL;
    }
    return RC_USER_BASE + 42;
  }
  if (nopen < 4) {
    open_calls[nopen][0] = off;
    open_calls[nopen][1] = lim;
  }
  nopen++;
  return (int32_t)(RC_USER_BASE + h); /* the opener fails with a Go error (code >= RC_USER_BASE) */
}

static void hex(const char *name, const uint8_t *p, int n) {
  printf("%s ", name);
  for (int i = 0; i < n; i++) printf("%02x", p[i]);
  printf("\n");
}

int main(void) {
  int32_t err = 0;
  rc_cipher *c = rc_cipher_new("potato", "", &err);
  CHECK(c && err == RC_NIL, "rc_cipher_new");
  if (!c) return 1;
  uint8_t dk[32], nk[32], nt[16];
  rc_cipher_keys(c, dk, nk, nt);
  hex("data_key", dk, 32);
  hex("name_key", nk, 32);
  hex("name_tweak", nt, 16);

  /* sizes (cipher.go:1121-1146) */
  CHECK(rc_encrypted_size(0) == 32 && rc_encrypted_size(1) == 49 && rc_encrypted_size(65536) == 65584 &&
            rc_encrypted_size(65537) == 65601,
        "EncryptedSize");
  CHECK(rc_decrypted_size(32, &err) == 0 && err == RC_NIL, "DecryptedSize(32)");
  rc_decrypted_size(48, &err);
  CHECK(err == RC_ERR_FILE_BAD_HEADER, "DecryptedSize(48) bad header");
  rc_decrypted_size(31, &err);
  CHECK(err == RC_ERR_FILE_TOO_SHORT, "DecryptedSize(31) too short");

  /* nonce arithmetic with full carry (cipher.go:647-678) */
  uint8_t n[24];
  memset(n, 0xFF, 24);
  rc_nonce_increment(n);
  int zero = 1;
  for (int i = 0; i < 24; i++) zero &= n[i] == 0;
  CHECK(zero, "nonce increment wraps all 24 bytes");
  memset(n, 0, 24);
  n[0] = 0xFF;
  rc_nonce_add(n, 1);
  CHECK(n[0] == 0 && n[1] == 1, "nonce add carry");

  /* newDecrypter errors close the source once; a reader error passes through unchanged */
  static const uint8_t bad_magic[40] = "RCLONX\0\0--------------------------------";
  boxes[1] = (box){bad_magic, 40, 0, RC_EOF, 0, 0};
  rc_decrypter *d = gpucipher_decrypt(c, 1, 0, &err);
  CHECK(!d && err == RC_ERR_BAD_MAGIC && boxes[1].closes == 1, "bad magic");
  boxes[2] = (box){bad_magic, 10, 0, RC_EOF, 0, 0};
  d = gpucipher_decrypt(c, 2, 0, &err);
  CHECK(!d && err == RC_ERR_FILE_TOO_SHORT && boxes[2].closes == 1, "too short");
  boxes[3] = (box){bad_magic, 5, 0, RC_USER_BASE + 7, 0, 0};
  d = gpucipher_decrypt(c, 3, 1, &err);
  CHECK(!d && err == RC_USER_BASE + 7 && boxes[3].closes == 1, "reader error passes through");
  printf("decrypter_errors %d %d %d\n", RC_ERR_BAD_MAGIC, RC_ERR_FILE_TOO_SHORT, RC_USER_BASE + 7);

  /* DecryptDataSeek: the opener's error passes through; open arguments as cipher.go:821-859 */
  int32_t wrapped = -1;
  d = gpucipher_decrypt_seek(c, 4, 0, -1, &err, &wrapped);
  CHECK(!d && err == RC_USER_BASE + 4 && wrapped == RC_NIL, "open error (offset 0)");
  d = gpucipher_decrypt_seek(c, 5, 100, 50, &err, &wrapped);
  CHECK(!d && err == RC_USER_BASE + 5, "open error (offset 100)");
  CHECK(nopen == 2 && open_calls[0][0] == 0 && open_calls[0][1] == -1 && open_calls[1][0] == 0 &&
            open_calls[1][1] == 32,
        "open arguments");

  /* the re-open at the seek offset fails: RC_ERR_REOPEN with the opener's own error behind it
   * (cipher.go:1011 wraps it with %w), the header reader closed once */
  static const uint8_t hdr32[32] = "RCLONE\0\0abcdefghijklmnopqrstuvwx";
  boxes[0] = (box){hdr32, 32, 0, RC_EOF, 0, 0};
  d = gpucipher_decrypt_seek(c, 100, 70000, -1, &err, &wrapped);
  CHECK(!d && err == RC_ERR_REOPEN && wrapped == RC_USER_BASE + 42 && reopen_calls == 2 && boxes[0].closes == 1,
        "re-open error wrapped");
  printf("reopen_wrapped %d %d\n", err, wrapped);

  /* computeHashWithNonce through the shim: a source failing before its first block returns its
   * error and is closed once; a nonce count that differs from the source count is refused before
   * any source is read.  No GPU work is needed for either. */
  static const uint8_t nonce24[24] = {9};
  uint8_t md5[16 * 3];
  boxes[1] = (box){NULL, 0, 0, RC_USER_BASE + 11, 0, 0};
  CHECK(gpucipher_compute_hash(c, 1, 1, nonce24, md5) == RC_USER_BASE + 11 && boxes[1].closes == 1,
        "compute hash: reader error, source closed");
  uintptr_t srcs[3] = {1, 2, 3};
  int32_t errs[3] = {0, 0, 0};
  uint8_t nonces[24 * 3] = {0};
  boxes[1] = (box){NULL, 0, 0, RC_USER_BASE + 11, 0, 0};
  boxes[2] = (box){NULL, 0, 0, RC_USER_BASE + 12, 0, 0};
  boxes[3] = (box){NULL, 0, 0, RC_UNEXPECTED_EOF, 0, 0};
  CHECK(gpucipher_hash_batch(c, 3, srcs, 2, nonces, md5, errs) == RC_ERR_INVALID && boxes[1].reads == 0,
        "hash batch: nonce count mismatch refused");
  CHECK(gpucipher_hash_batch(c, 3, srcs, 3, nonces, md5, errs) == RC_NIL && errs[0] == RC_USER_BASE + 11 &&
            errs[1] == RC_USER_BASE + 12 && errs[2] == RC_UNEXPECTED_EOF && boxes[1].closes == 1 &&
            boxes[2].closes == 1 && boxes[3].closes == 1,
        "hash batch: failing sources");
  printf("hash_batch_errs %d %d %d\n", errs[0], errs[1], errs[2]);

  /* encrypter: nonce from the cipher's random source, header served before any block */
  static const uint8_t rnd[24] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24};
  boxes[6] = (box){rnd, 24, 0, RC_EOF, 0, 0};
  rc_cipher_set_rand(c, gpucipher_reader(6, 0, 0));
  boxes[7] = (box){rnd, 0, 0, RC_EOF, 0, 0};
  rc_encrypter *e = gpucipher_encrypt(c, 7, NULL, &err);
  CHECK(e && err == RC_NIL, "encrypt_data");
  if (e) {
    uint8_t nonce[24], hdr[32];
    rc_encrypter_nonce(e, nonce);
    CHECK(!memcmp(nonce, rnd, 24), "nonce from the random source");
    int64_t got = rc_encrypter_read(e, hdr, 32, &err);
    CHECK(got == 32 && err == RC_NIL && !memcmp(hdr, "RCLONE\0\0", 8) && !memcmp(hdr + 8, rnd, 24), "header");
    CHECK(boxes[7].reads == 0, "no source read before the header is consumed");
    rc_encrypter_free(e);
  }
  boxes[6] = (box){rnd, 10, 0, RC_EOF, 0, 0};
  e = gpucipher_encrypt(c, 7, NULL, &err);
  CHECK(!e && err == RC_ERR_SHORT_NONCE, "short read of nonce");

  /* host-only name modes: obfuscate round trip, base32 encoding */
  rc_cipher_set_name_encryption(c, RC_NAME_OBFUSCATE, 1, RC_ENC_BASE32);
  const char *in[2] = {"hello/world.txt", "a"};
  uint64_t inl[2] = {15, 1};
  rc_names *r = NULL;
  CHECK(rc_names_run(c, RC_OP_ENCRYPT_FILE_NAME, 2, in, inl, &r) == RC_NIL, "obfuscate");
  if (r) {
    const char *s;
    uint64_t len;
    int32_t e2;
    int64_t arg;
    char enc[64];
    rc_names_get(r, 0, &s, &len, &e2, &arg);
    CHECK(e2 == RC_NIL && len < sizeof enc, "obfuscated name");
    memcpy(enc, s, len);
    enc[len] = 0;
    printf("obfuscated %s\n", enc);
    rc_names_free(r);
    const char *in2[1] = {enc};
    uint64_t in2l[1] = {len};
    CHECK(rc_names_run(c, RC_OP_DECRYPT_FILE_NAME, 1, in2, in2l, &r) == RC_NIL, "deobfuscate");
    if (r) {
      rc_names_get(r, 0, &s, &len, &e2, &arg);
      CHECK(e2 == RC_NIL && len == 15 && !memcmp(s, "hello/world.txt", 15), "deobfuscated name");
      rc_names_free(r);
    }
  }
  char b32[64];
  int64_t bl = rc_name_encode(RC_ENC_BASE32, (const uint8_t *)"hello", 5, b32, sizeof b32);
  CHECK(bl == 8 && !memcmp(b32, "d1imor3f", 8), "base32 encode");
  CHECK(strcmp(rc_error_string(RC_ERR_BAD_BLOCK), "failed to authenticate decrypted block - bad password?") == 0,
        "error string");
  /* keys derived on the Go side (Cipher.Key) installed directly */
  rc_cipher *z = rc_cipher_new(NULL, NULL, &err);
  CHECK(z && err == RC_NIL, "rc_cipher_new(NULL)");
  if (z) {
    uint8_t d2[32], n2[32], t2[16];
    rc_cipher_keys(z, d2, n2, t2);
    CHECK(d2[0] == 0 && d2[31] == 0, "empty password: zero keys");
    rc_cipher_set_keys(z, dk, nk, nt);
    rc_cipher_keys(z, d2, n2, t2);
    CHECK(!memcmp(d2, dk, 32) && !memcmp(n2, nk, 32) && !memcmp(t2, nt, 16), "rc_cipher_set_keys");
    rc_cipher_free(z);
  }
  rc_cipher_free(c);
  if (failures) return 1;
  printf("c client ok\n");
  return 0;
}
