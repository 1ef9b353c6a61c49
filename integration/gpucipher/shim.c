// shim.c -- the C half of the cgo binding `package gpucipher` (gpucipher.go): the callbacks
// librclone_crypt.so calls are C functions that forward to the Go exports, carrying the
// runtime/cgo.Handle of the Go reader / opener as an integer.  The library only passes `user`
// back (include/rclone_crypt_gpu.h), so Go never converts an integer into unsafe.Pointer -- the
// pattern `go test -race` (checkptr) accepts.  cgo compiles this file as C with the package's
// CFLAGS; it must not live in the preamble of the file holding the //export functions (cgo
// forbids definitions there).  tests/native builds it with -std=c11 -Werror against a stand-in
// _cgo_export.h and drives it from a C client.
#include <stdint.h>
#include <stdlib.h>

#include "_cgo_export.h" /* goRead, goClose, goRangeSeek, goOpen */
#include "rclone_crypt_gpu.h"

static int64_t shim_read(void *user, uint8_t *p, int64_t n, int32_t *err) {
  return goRead((uintptr_t)user, p, n, err);
}
static int32_t shim_close(void *user) { return goClose((uintptr_t)user); }
static int32_t shim_range_seek(void *user, int64_t offset, int32_t whence, int64_t limit) {
  return goRangeSeek((uintptr_t)user, offset, whence, limit);
}
static int32_t shim_open(void *user, int64_t offset, int64_t limit, rc_reader *out) {
  return goOpen((uintptr_t)user, offset, limit, out);
}

/* io.Reader (+ io.Closer, + fs.RangeSeeker) behind handle h */
rc_reader gpucipher_reader(uintptr_t h, int closer, int range_seeker) {
  rc_reader r;
  r.read = shim_read;
  r.close = closer ? shim_close : NULL;
  r.range_seek = range_seeker ? shim_range_seek : NULL;
  r.user = (void *)h;
  return r;
}

/* newEncrypter (cipher.go:694): nonce NULL -> from the cipher's random source */
rc_encrypter *gpucipher_encrypt(rc_cipher *c, uintptr_t in, const uint8_t *nonce, int32_t *err) {
  return rc_encrypt_data(c, gpucipher_reader(in, 0, 0), nonce, err);
}

/* newDecrypter (cipher.go:793) over an io.ReadCloser */
rc_decrypter *gpucipher_decrypt(rc_cipher *c, uintptr_t rc, int range_seeker, int32_t *err) {
  return rc_decrypt_data(c, gpucipher_reader(rc, 1, range_seeker), err);
}

/* DecryptDataSeek (cipher.go:1112): open_state is the handle of the Go OpenRangeSeek; *wrapped gets
 * the opener's error behind RC_ERR_REOPEN (the %w operand, cipher.go:1011) */
rc_decrypter *gpucipher_decrypt_seek(rc_cipher *c, uintptr_t open_state, int64_t offset, int64_t limit,
                                     int32_t *err, int32_t *wrapped) {
  return rc_decrypt_data_seek_ex(c, shim_open, (void *)open_state, offset, limit, err, wrapped);
}

/* computeHashWithNonce (crypt.go:784), one object: src is the handle of an io.Reader, closed after
 * use when it is an io.Closer (closer != 0) */
int32_t gpucipher_compute_hash(rc_cipher *c, uintptr_t src, int closer, const uint8_t *nonce, uint8_t *md5) {
  return rc_compute_hash_with_nonce(c, gpucipher_reader(src, closer, 0), nonce, md5);
}

/* computeHashWithNonce (crypt.go:784) batched: srcs[i] handles of io.Readers, closed after use.
 * n_nonces is len(nonces) on the Go side: a mismatch is refused before any source is read. */
int32_t gpucipher_hash_batch(rc_cipher *c, uint64_t n, const uintptr_t *srcs, uint64_t n_nonces,
                             const uint8_t *nonces, uint8_t *md5, int32_t *errs) {
  if (n_nonces != n) return RC_ERR_INVALID;
  rc_reader *r = (rc_reader *)malloc((n ? n : 1) * sizeof *r);
  if (!r) return RC_ERR_INVALID;
  for (uint64_t i = 0; i < n; i++) r[i] = gpucipher_reader(srcs[i], 1, 0);
  const int32_t rc = rc_hash_batch_with_nonce(c, n, r, nonces, md5, errs);
  free(r);
  return rc;
}
