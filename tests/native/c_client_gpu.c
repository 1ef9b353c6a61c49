/* TEST INFRASTRUCTURE: the data path of the cgo binding's C half (integration/gpucipher/shim.c)
 * on the GPU.  Same setup as c_client.c -- compiled as cgo compiles shim.c (-std=c11, the
 * package's include path, a stand-in _cgo_export.h), the Go //export functions played by C
 * functions over a table of integer handles -- but every call here seals or opens blocks on the
 * device through librclone_crypt.so:
 *
 *   gpucipher_encrypt       -> rc_encrypt_data / rc_encrypter_read   (cipher.go:694-758)
 *   rc_encrypter_set_md5    -> the TeeReader MD5 of Fs.put           (crypt.go:516-533)
 *   gpucipher_decrypt       -> rc_decrypt_data / rc_decrypter_read   (cipher.go:793-927)
 *   gpucipher_decrypt_seek  -> rc_decrypt_data_seek_ex, then RangeSeek (cipher.go:972-1039, :1112)
 *   gpucipher_compute_hash  -> computeHashWithNonce                  (crypt.go:784-806)
 *   gpucipher_hash_batch    -> the same, batched                     (cmd/cryptcheck/cryptcheck.go:67-117)
 *
 * Usage: c_client_gpu <manifest> [threads].  Manifest line 1: the data key (64 hex digits); then
 * one case per line: "<nonce hex> <plaintext path> <crypt file out path>".  For each case the
 * client writes the crypt file the encrypter produced (the test compares it with the reference's /
 * libsodium's fixture) and checks on its own that decrypting it, seeking into it and reading a
 * tampered copy behave as cipher.go does.  It prints one line per case:
 *   case <i> size <n> tee <md5> hash <md5> bad_block_at <bytes> opens <n>
 * then "batch <i> <md5>" per case, and "c client gpu ok" last when every check passed.
 * With threads > 1, that many threads run every case at once over the one shared cipher -- the
 * Go side's --transfers / --checkers goroutines calling through the shim concurrently, so the
 * engine coalesces their blocks into shared launches -- and every thread's crypt bytes, tee,
 * hash and batch digests must equal thread 0's (which are the ones printed and written). */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
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

static atomic_int failures;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      fprintf(stderr, "FAIL: ");        \
      fprintf(stderr, __VA_ARGS__);     \
      fprintf(stderr, "\n");            \
      failures++;                       \
    }                                   \
  } while (0)

/* ---- the "Go side": handles 1.. are readers (runtime/cgo.Handle values), OPENER_BASE +
 * MAXCASE * t + i the OpenRangeSeek of thread t's crypt file of case i (gpucipher.go goOpen).  Readers hand out at most `chunk`
 * bytes per Read, like a socket does: the library's ReadFill must gather whole blocks itself. */
typedef struct {
  const uint8_t *p;
  int64_t end, pos;
  int64_t full;  /* bytes behind p: a RangeSeek may move end up to here */
  int64_t chunk; /* max bytes per Read (0: no cap) */
  int32_t fail;  /* returned once pos == end (RC_EOF for a clean end) */
  int reads, closes, seeks;
} box;
#define MAXBOX 16384
#define OPENER_BASE 1000000u
static box boxes[MAXBOX];
static atomic_int nbox = 1; /* handle 0 unused: a cgo.Handle is never 0 */

static uintptr_t new_box(const uint8_t *p, int64_t pos, int64_t end, int64_t full, int64_t chunk) {
  const int h = atomic_fetch_add(&nbox, 1);
  if (h >= MAXBOX) {
    fprintf(stderr, "handle table full\n");
    exit(2);
  }
  boxes[h] = (box){p, end, pos, full, chunk, RC_EOF, 0, 0, 0};
  return (uintptr_t)h;
}

int64_t goRead(uintptr_t h, uint8_t *p, int64_t n, int32_t *err) {
  box *b = &boxes[h];
  b->reads++;
  int64_t k = b->end - b->pos;
  if (k > n) k = n;
  if (b->chunk > 0 && k > b->chunk) k = b->chunk;
  if (k > 0) memcpy(p, b->p + b->pos, (size_t)k);
  b->pos += k;
  *err = (k == 0) ? b->fail : RC_NIL;
  return k;
}
int32_t goClose(uintptr_t h) {
  boxes[h].closes++;
  return RC_NIL;
}

/* the cases (read-only once loaded) and each thread's results, its crypt files served by the openers */
typedef struct {
  uint8_t *plain;
  int64_t plain_n;
  uint8_t nonce[24];
} kase;
typedef struct {
  uint8_t *crypt;
  int64_t crypt_n, bad_at;
  uint8_t tee[16], hash[16], batch[16];
  int opens;
} result;
#define MAXCASE 128
#define MAXTHREADS 16
static kase cases[MAXCASE];
static result results[MAXTHREADS][MAXCASE];
static int ncases;

/* fs.RangeSeeker on a reader over a crypt file: offset/limit are underlying (crypt file) bytes */
int32_t goRangeSeek(uintptr_t h, int64_t offset, int32_t whence, int64_t limit) {
  box *b = &boxes[h];
  if (whence != 0) return RC_USER_BASE + 3;
  if (offset < 0 || offset > b->full) return RC_USER_BASE + 4;
  b->seeks++;
  b->pos = offset;
  b->end = (limit >= 0 && offset + limit < b->full) ? offset + limit : b->full;
  return RC_NIL;
}
/* OpenRangeSeek (cipher.go:77) over case i's crypt file: a fresh reader at offset, capped at
 * offset+limit as backend/memory's Open with a RangeOption would.  Even cases hand out an
 * fs.RangeSeeker (RangeSeek moves it, cipher.go:997), odd cases a plain ReadCloser (RangeSeek
 * closes it and opens again, cipher.go:1003-1014). */
int32_t goOpen(uintptr_t h, int64_t off, int64_t lim, rc_reader *out) {
  if (h < OPENER_BASE || h - OPENER_BASE >= (uintptr_t)MAXCASE * MAXTHREADS) return RC_USER_BASE + 1;
  const uintptr_t t = (h - OPENER_BASE) / MAXCASE, i = (h - OPENER_BASE) % MAXCASE;
  result *k = &results[t][i];
  k->opens++;
  if (off < 0 || off > k->crypt_n) return RC_USER_BASE + 2;
  int64_t end = k->crypt_n;
  if (lim >= 0 && off + lim < end) end = off + lim;
  *out = gpucipher_reader(new_box(k->crypt, off, end, k->crypt_n, 7000), 1, i % 2 == 0);
  return RC_NIL;
}

static uint8_t *slurp(const char *path, int64_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *p = (uint8_t *)malloc((size_t)sz + 1);
  if (p && fread(p, 1, (size_t)sz, f) != (size_t)sz) {
    free(p);
    p = NULL;
  }
  fclose(f);
  *n = sz;
  return p;
}

static int unhex(const char *s, uint8_t *out, int n) {
  if ((int)strlen(s) != 2 * n) return -1;
  for (int i = 0; i < n; i++) {
    unsigned v;
    if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
    out[i] = (uint8_t)v;
  }
  return 0;
}

static void hexs(char *dst, const uint8_t *p, int n) {
  for (int i = 0; i < n; i++) sprintf(dst + 2 * i, "%02x", p[i]);
}

/* Read a handle to its end in ragged request sizes, as a Go caller's io.Copy / ReadFull mix would.
 * Returns the bytes read; *err = the error that ended it (RC_EOF when clean). */
typedef int64_t (*read_fn)(void *h, uint8_t *p, int64_t n, int32_t *err);
static int64_t enc_read(void *h, uint8_t *p, int64_t n, int32_t *err) {
  return rc_encrypter_read((rc_encrypter *)h, p, n, err);
}
static int64_t dec_read(void *h, uint8_t *p, int64_t n, int32_t *err) {
  return rc_decrypter_read((rc_decrypter *)h, p, n, err);
}
static int64_t drain(read_fn rd, void *h, uint8_t *dst, int64_t cap, int32_t *err) {
  static const int64_t sizes[] = {1, 4096, 65552 * 2 + 7, 31, 65536, 100000};
  int64_t total = 0;
  for (int it = 0;; it++) {
    int64_t want = sizes[it % 6];
    if (want > cap - total) want = cap - total;
    if (want == 0) { /* the stream must be at its end: a read into a 1-byte scratch tells */
      uint8_t scratch[1];
      int64_t got = rd(h, scratch, 1, err);
      if (got != 0) *err = RC_ERR_INVALID;
      return total;
    }
    int64_t got = rd(h, dst + total, want, err);
    if (got < 0 || got > want) {
      *err = RC_ERR_INVALID;
      return total;
    }
    total += got;
    if (*err != RC_NIL) return total;
  }
}

/* every check of every case, on one thread, into results[t] */
typedef struct {
  rc_cipher *c;
  int t;
} job;

static void *run_cases(void *arg) {
  rc_cipher *c = ((job *)arg)->c;
  const int t = ((job *)arg)->t;
  const int n = ncases;
  int32_t err = RC_NIL;
  for (int i = 0; i < n; i++) {
    const kase *k = &cases[i];
    result *res = &results[t][i];
    const int64_t want_n = rc_encrypted_size(k->plain_n);
    const int64_t nblocks = (k->plain_n + 65535) / 65536;

    /* ---- encrypt: Fs.put's path, with the put tee MD5 taken by the encrypter */
    uintptr_t in = new_box(k->plain, 0, k->plain_n, k->plain_n, 5000);
    rc_encrypter *e = gpucipher_encrypt(c, in, k->nonce, &err);
    CHECK(e && err == RC_NIL, "case %d: gpucipher_encrypt %d", i, err);
    if (!e) continue;
    CHECK(rc_encrypter_set_md5(e, 1) == RC_NIL, "case %d: set md5", i);
    uint8_t en[24]; /* the nonce the object is stored under, visible before the first Read (crypt.go:529) */
    rc_encrypter_nonce(e, en);
    CHECK(!memcmp(en, k->nonce, 24), "case %d: encrypter nonce", i);
    res->crypt = (uint8_t *)malloc((size_t)want_n + 1);
    res->crypt_n = drain(enc_read, e, res->crypt, want_n + 1, &err);
    CHECK(err == RC_EOF && res->crypt_n == want_n, "case %d: encrypt read %lld of %lld, err %d", i,
          (long long)res->crypt_n, (long long)want_n, err);
    CHECK(rc_encrypter_md5(e, res->tee) == RC_NIL, "case %d: tee md5", i);
    rc_encrypter_free(e);

    /* ---- decrypt (DecryptData over an io.ReadCloser that is also a RangeSeeker) */
    uint8_t *back = (uint8_t *)malloc((size_t)k->plain_n + 1);
    uintptr_t rc = new_box(res->crypt, 0, res->crypt_n, res->crypt_n, 7000);
    rc_decrypter *d = gpucipher_decrypt(c, rc, 1, &err);
    CHECK(d && err == RC_NIL, "case %d: gpucipher_decrypt %d", i, err);
    if (d) {
      int64_t got = drain(dec_read, d, back, k->plain_n + 1, &err);
      CHECK(err == RC_EOF && got == k->plain_n && !memcmp(back, k->plain, (size_t)got),
            "case %d: decrypt round trip (%lld bytes, err %d)", i, (long long)got, err);
      CHECK(rc_decrypter_close(d) == RC_NIL && boxes[rc].closes == 1, "case %d: close once", i);
      CHECK(rc_decrypter_close(d) == RC_ERR_FILE_CLOSED, "case %d: second close", i);
      rc_decrypter_free(d);
    }

    /* ---- DecryptDataSeek (offset 70000, limit 50, clamped into small files), then a RangeSeek
     * on the same handle back to offset 1 without a limit (cipher.go:972-1034) */
    int64_t off = k->plain_n > 70050 ? 70000 : k->plain_n / 2;
    int64_t lim = 50;
    int32_t wrapped = -1;
    d = gpucipher_decrypt_seek(c, OPENER_BASE + (uintptr_t)(MAXCASE * t + i), off, lim, &err, &wrapped);
    CHECK(d && err == RC_NIL, "case %d: gpucipher_decrypt_seek %d (wrapped %d)", i, err, wrapped);
    if (d) {
      int64_t expect = k->plain_n - off < lim ? k->plain_n - off : lim;
      int64_t got = drain(dec_read, d, back, k->plain_n + 1, &err);
      CHECK(err == RC_EOF && got == expect && !memcmp(back, k->plain + off, (size_t)got),
            "case %d: seek window at %lld (%lld bytes, err %d)", i, (long long)off, (long long)got, err);
      if (k->plain_n > 0) {
        int64_t pos = rc_decrypter_range_seek(d, 1, 0, -1, &err);
        CHECK(err == RC_NIL && pos == 1, "case %d: RangeSeek(1) %d", i, err);
        got = drain(dec_read, d, back, k->plain_n + 1, &err);
        CHECK(err == RC_EOF && got == k->plain_n - 1 && !memcmp(back, k->plain + 1, (size_t)got),
              "case %d: read after RangeSeek (%lld bytes, err %d)", i, (long long)got, err);
      }
      rc_decrypter_close(d);
      rc_decrypter_free(d);
    }

    /* ---- tampered ciphertext: one byte of block nblocks/2's payload flipped.  The decrypter
     * returns every byte before that block, then ErrorEncryptedBadBlock (cipher.go:880-893),
     * which the Go side maps to the sentinel Register() installed for RC_ERR_BAD_BLOCK. */
    res->bad_at = -1;
    if (nblocks > 0) {
      const int64_t kb = nblocks / 2;
      uint8_t *tb = (uint8_t *)malloc((size_t)res->crypt_n);
      memcpy(tb, res->crypt, (size_t)res->crypt_n);
      tb[32 + kb * 65552 + 16] ^= 0x40;
      uintptr_t tr = new_box(tb, 0, res->crypt_n, res->crypt_n, 0);
      d = gpucipher_decrypt(c, tr, 0, &err);
      CHECK(d && err == RC_NIL, "case %d: decrypt tampered %d", i, err);
      if (d) {
        res->bad_at = drain(dec_read, d, back, k->plain_n + 1, &err);
        CHECK(err == RC_ERR_BAD_BLOCK && res->bad_at == kb * 65536 && !memcmp(back, k->plain, (size_t)res->bad_at),
              "case %d: tampered block %lld -> err %d after %lld bytes", i, (long long)kb, err,
              (long long)res->bad_at);
        CHECK(!strcmp(rc_error_string(err), "failed to authenticate decrypted block - bad password?"),
              "case %d: bad-block message", i);
        rc_decrypter_close(d);
        rc_decrypter_free(d);
      }
      /* a tampered tag (the block's first 16 bytes) fails the same way */
      memcpy(tb, res->crypt, (size_t)res->crypt_n);
      tb[32 + kb * 65552] ^= 0x01;
      tr = new_box(tb, 0, res->crypt_n, res->crypt_n, 0);
      d = gpucipher_decrypt(c, tr, 0, &err);
      if (d) {
        int64_t got = drain(dec_read, d, back, k->plain_n + 1, &err);
        CHECK(err == RC_ERR_BAD_BLOCK && got == kb * 65536, "case %d: tampered tag", i);
        rc_decrypter_close(d);
        rc_decrypter_free(d);
      }
      free(tb);
    }
    free(back);

    /* ---- computeHashWithNonce, one object (the cryptcheck checker's call) */
    uintptr_t src = new_box(k->plain, 0, k->plain_n, k->plain_n, 3000);
    CHECK(gpucipher_compute_hash(c, src, 1, k->nonce, res->hash) == RC_NIL && boxes[src].closes == 1,
          "case %d: compute hash", i);
    CHECK(!memcmp(res->hash, res->tee, 16), "case %d: computeHashWithNonce == put's tee MD5", i);
  }

  /* ---- computeHashWithNonce batched over every case (HashBatchWithNonce) */
  uintptr_t *srcs = (uintptr_t *)malloc(sizeof(uintptr_t) * (size_t)(n ? n : 1));
  uint8_t *nonces = (uint8_t *)malloc(24 * (size_t)(n ? n : 1));
  uint8_t *md5 = (uint8_t *)malloc(16 * (size_t)(n ? n : 1));
  int32_t *errs = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  for (int i = 0; i < n; i++) {
    srcs[i] = new_box(cases[i].plain, 0, cases[i].plain_n, cases[i].plain_n, 9000);
    memcpy(nonces + 24 * i, cases[i].nonce, 24);
  }
  CHECK(gpucipher_hash_batch(c, (uint64_t)n, srcs, (uint64_t)n, nonces, md5, errs) == RC_NIL, "hash batch");
  for (int i = 0; i < n; i++) {
    CHECK(errs[i] == RC_NIL && boxes[srcs[i]].closes == 1, "batch %d: err %d", i, errs[i]);
    memcpy(results[t][i].batch, md5 + 16 * i, 16);
  }
  free(srcs);
  free(nonces);
  free(md5);
  free(errs);
  return NULL;
}

int main(int argc, char **argv) {
  if (argc != 2 && argc != 3) {
    fprintf(stderr, "usage: c_client_gpu <manifest> [threads]\n");
    return 2;
  }
  const int nthreads = argc == 3 ? atoi(argv[2]) : 1;
  if (nthreads < 1 || nthreads > MAXTHREADS) return 2;
  FILE *mf = fopen(argv[1], "r");
  if (!mf) return 2;
  char keyhex[80], nhex[80], ppath[4096], opath[4096];
  uint8_t key[32], zero[32] = {0};
  if (fscanf(mf, "%79s", keyhex) != 1 || unhex(keyhex, key, 32)) return 2;
  int n = 0;
  static char outs[MAXCASE][4096];
  while (n < MAXCASE && fscanf(mf, "%79s %4095s %4095s", nhex, ppath, opath) == 3) {
    kase *k = &cases[n];
    if (unhex(nhex, k->nonce, 24)) return 2;
    k->plain = slurp(ppath, &k->plain_n);
    if (!k->plain) return 2;
    memcpy(outs[n], opath, sizeof opath);
    n++;
  }
  fclose(mf);
  ncases = n;

  /* one Cipher with keys from the Go side's Cipher.Key (New(dataKey, nameKey, nameTweak, ..)),
   * shared by every thread as rclone shares it between its goroutines */
  int32_t err = RC_NIL;
  rc_cipher *c = rc_cipher_new(NULL, NULL, &err);
  if (!c) return 2;
  rc_cipher_set_keys(c, key, zero, zero);

  job jobs[MAXTHREADS];
  pthread_t th[MAXTHREADS];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job){c, t};
    if (nthreads == 1) run_cases(&jobs[t]);
    else if (pthread_create(&th[t], NULL, run_cases, &jobs[t]) != 0) return 2;
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);

  /* every thread produced thread 0's bytes and digests */
  for (int t = 1; t < nthreads; t++)
    for (int i = 0; i < n; i++) {
      const result *a = &results[0][i], *b = &results[t][i];
      CHECK(a->crypt && b->crypt && a->crypt_n == b->crypt_n && !memcmp(a->crypt, b->crypt, (size_t)a->crypt_n) &&
                !memcmp(a->tee, b->tee, 16) && !memcmp(a->hash, b->hash, 16) && !memcmp(a->batch, b->batch, 16) &&
                a->bad_at == b->bad_at && a->opens == b->opens,
            "thread %d case %d differs from thread 0", t, i);
    }
  for (int i = 0; i < n; i++) {
    const result *r = &results[0][i];
    FILE *of = fopen(outs[i], "wb");
    if (of) {
      if (r->crypt) fwrite(r->crypt, 1, (size_t)r->crypt_n, of);
      fclose(of);
    }
    char th_[33], hh[33];
    hexs(th_, r->tee, 16);
    hexs(hh, r->hash, 16);
    printf("case %d size %lld tee %s hash %s bad_block_at %lld opens %d\n", i, (long long)cases[i].plain_n, th_, hh,
           (long long)r->bad_at, r->opens);
  }
  for (int i = 0; i < n; i++) {
    char bh[33];
    hexs(bh, results[0][i].batch, 16);
    printf("batch %d %s\n", i, bh);
  }
  if (nthreads > 1) printf("threads %d consistent\n", nthreads);
  rc_cipher_free(c);
  if (atomic_load(&failures)) {
    fprintf(stderr, "%d failures\n", atomic_load(&failures));
    return 1;
  }
  printf("c client gpu ok\n");
  return 0;
}
