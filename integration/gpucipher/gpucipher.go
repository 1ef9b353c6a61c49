// Package gpucipher runs rclone's crypt data cipher -- XSalsa20-Poly1305 over every 64 KiB
// block, backend/crypt/cipher.go:681-1118 -- on AMD MI355X GPUs through librclone_crypt.so
// (include/rclone_crypt_gpu.h).  It is the Go half of the drop-in: backend/crypt keeps its
// Fs/Object surface and routes encryptData / newEncrypter / DecryptData / DecryptDataSeek here
// when the crypt option `gpu` allows it (INTEGRATION.md).  The C half is shim.c.
//
// Readers, closers and openers cross the C ABI as runtime/cgo.Handle values carried in the
// library's opaque `user` field by shim.c; the Go side only ever sees them as integers.  Errors
// cross as small codes: the crypt sentinels (cipher.go:44-58) map to the values Register was
// given, io.EOF / io.ErrUnexpectedEOF to themselves, and any other error a reader or opener
// returned comes back as the identical Go value at the position cipher.go would return it.
package gpucipher

/*
#cgo CFLAGS: -I${SRCDIR}/../../../rclone_amd_native/include
#cgo LDFLAGS: -L${SRCDIR}/../../../rclone_amd_native/rclone_amd -lrclone_crypt -Wl,-rpath,${SRCDIR}/../../../rclone_amd_native/rclone_amd
#include <stdlib.h>
#include "rclone_crypt_gpu.h"

// shim.c
rc_reader gpucipher_reader(uintptr_t h, int closer, int range_seeker);
rc_encrypter *gpucipher_encrypt(rc_cipher *c, uintptr_t in, const uint8_t *nonce, int32_t *err);
rc_decrypter *gpucipher_decrypt(rc_cipher *c, uintptr_t rc, int range_seeker, int32_t *err);
rc_decrypter *gpucipher_decrypt_seek(rc_cipher *c, uintptr_t open_state, int64_t offset, int64_t limit, int32_t *err,
                                     int32_t *wrapped);
int32_t gpucipher_compute_hash(rc_cipher *c, uintptr_t src, int closer, const uint8_t *nonce, uint8_t *md5);
int32_t gpucipher_hash_batch(rc_cipher *c, uint64_t n, const uintptr_t *srcs, uint64_t n_nonces, const uint8_t *nonces,
                             uint8_t *md5, int32_t *errs);
*/
import "C"

import (
	"context"
	"encoding/hex"
	"errors"
	"fmt"
	"io"
	"runtime"
	"runtime/cgo"
	"sync"
	"unsafe"

	"github.com/rclone/rclone/fs"
)

// ---------------------------------------------------------------------------- errors

var (
	sentinelMu sync.RWMutex
	sentinels  = map[C.int32_t]error{}
)

// Register maps the library's sentinel codes onto backend/crypt's own error values
// (cipher.go:44-58), so callers comparing errors with == keep working.
func Register(tooShort, badHeader, badMagic, badBlock, closed, badSeek error) {
	sentinelMu.Lock()
	defer sentinelMu.Unlock()
	sentinels[C.RC_ERR_FILE_TOO_SHORT] = tooShort
	sentinels[C.RC_ERR_FILE_BAD_HEADER] = badHeader
	sentinels[C.RC_ERR_BAD_MAGIC] = badMagic
	sentinels[C.RC_ERR_BAD_BLOCK] = badBlock
	sentinels[C.RC_ERR_FILE_CLOSED] = closed
	sentinels[C.RC_ERR_BAD_SEEK] = badSeek
}

// errTable holds the Go errors produced by the readers / openers of one handle; C sees index
// codes >= RC_USER_BASE.  The library may return a code again and again (a finished stream's
// sticky error, cipher.go:748-758 / :1042-1052), so entries stay for the handle's life; an error
// value seen before gets its old code back, so the table grows only with distinct errors (a
// reader that keeps failing the same way adds one entry, not one per call).
type errTable struct {
	mu   sync.Mutex
	errs []error
}

func (t *errTable) code(err error) C.int32_t {
	switch {
	case err == nil:
		return C.RC_NIL
	case err == io.EOF:
		return C.RC_EOF
	case err == io.ErrUnexpectedEOF:
		return C.RC_UNEXPECTED_EOF
	}
	t.mu.Lock()
	defer t.mu.Unlock()
	for i := len(t.errs) - 1; i >= 0; i-- {
		if sameError(t.errs[i], err) {
			return C.int32_t(C.RC_USER_BASE + i)
		}
	}
	t.errs = append(t.errs, err)
	return C.int32_t(C.RC_USER_BASE + len(t.errs) - 1)
}

// sameError: the identical error value (== on comparable dynamic types; never panics).
func sameError(a, b error) (same bool) {
	defer func() {
		if recover() != nil {
			same = false
		}
	}()
	return a == b
}

func (t *errTable) err(code C.int32_t) error {
	switch {
	case code == C.RC_NIL:
		return nil
	case code == C.RC_EOF:
		return io.EOF
	case code == C.RC_UNEXPECTED_EOF:
		return io.ErrUnexpectedEOF
	case code >= C.RC_USER_BASE:
		t.mu.Lock()
		defer t.mu.Unlock()
		return t.errs[int(code-C.RC_USER_BASE)]
	}
	sentinelMu.RLock()
	e, ok := sentinels[code]
	sentinelMu.RUnlock()
	if ok {
		return e
	}
	return errors.New(C.GoString(C.rc_error_string(code)))
}

// ---------------------------------------------------------------------------- callbacks

type readerBox struct {
	r       io.Reader
	t       *errTable
	s       *openState // the decrypter's state (its RangeSeek context), nil for an encrypter's source
	readErr bool       // a Read returned an error other than io.EOF
}

//export goRead
func goRead(h C.uintptr_t, p *C.uint8_t, n C.int64_t, errp *C.int32_t) C.int64_t {
	b := cgo.Handle(h).Value().(*readerBox)
	buf := unsafe.Slice((*byte)(unsafe.Pointer(p)), int(n)) // library-owned pinned staging
	got, err := b.r.Read(buf)
	if err != nil && err != io.EOF {
		b.readErr = true
	}
	*errp = b.t.code(err)
	return C.int64_t(got)
}

//export goClose
func goClose(h C.uintptr_t) C.int32_t {
	b := cgo.Handle(h).Value().(*readerBox)
	code := C.int32_t(C.RC_NIL)
	if c, ok := b.r.(io.Closer); ok {
		code = b.t.code(c.Close())
	}
	if b.s != nil {
		// the library closes a reader once and never uses it again (Close, or RangeSeek
		// replacing it, cipher.go:1004-1015): drop it now instead of at the decrypter's end
		b.s.forget(cgo.Handle(h))
	}
	return code
}

//export goRangeSeek
func goRangeSeek(h C.uintptr_t, offset C.int64_t, whence C.int32_t, limit C.int64_t) C.int32_t {
	b := cgo.Handle(h).Value().(*readerBox)
	rs := b.r.(fs.RangeSeeker) // only registered when the reader is one (cipher.go:997)
	ctx := context.TODO()
	if b.s != nil {
		b.s.mu.Lock()
		if b.s.ctx != nil {
			ctx = b.s.ctx // the ctx of the Decrypter.RangeSeek call in progress (cipher.go:999)
		}
		b.s.mu.Unlock()
	}
	_, err := rs.RangeSeek(ctx, int64(offset), int(whence), int64(limit))
	return b.t.code(err)
}

// OpenRangeSeek is backend/crypt's opener (cipher.go:77).
type OpenRangeSeek func(ctx context.Context, offset, limit int64) (io.ReadCloser, error)

type openState struct {
	ctx     context.Context
	open    OpenRangeSeek
	t       *errTable
	mu      sync.Mutex
	handles map[cgo.Handle]struct{} // readers handed to C and not yet closed by it
}

func (s *openState) newReader(r io.Reader, closer bool) C.rc_reader {
	hd := cgo.NewHandle(&readerBox{r: r, t: s.t, s: s})
	s.mu.Lock()
	if s.handles == nil {
		s.handles = map[cgo.Handle]struct{}{}
	}
	s.handles[hd] = struct{}{}
	s.mu.Unlock()
	_, seeker := r.(fs.RangeSeeker)
	return C.gpucipher_reader(C.uintptr_t(hd), cbool(closer), cbool(seeker))
}

// forget deletes a reader's handle once the library has closed it (each handle is deleted once).
func (s *openState) forget(hd cgo.Handle) {
	s.mu.Lock()
	_, live := s.handles[hd]
	delete(s.handles, hd)
	s.mu.Unlock()
	if live {
		hd.Delete()
	}
}

// release deletes every handle still held (idempotent).
func (s *openState) release() {
	s.mu.Lock()
	hs := s.handles
	s.handles = nil
	s.mu.Unlock()
	for hd := range hs {
		hd.Delete()
	}
}

//export goOpen
func goOpen(h C.uintptr_t, offset, limit C.int64_t, out *C.rc_reader) C.int32_t {
	s := cgo.Handle(h).Value().(*openState)
	s.mu.Lock()
	ctx := s.ctx
	s.mu.Unlock()
	rc, err := s.open(ctx, int64(offset), int64(limit))
	if err != nil {
		return s.t.code(err)
	}
	*out = s.newReader(rc, true)
	return C.RC_NIL
}

func cbool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}

// ---------------------------------------------------------------------------- cipher

// Cipher is the GPU half of one crypt Cipher: its data key and options, and the engines of
// the process (spread over every MI355X of the node, RCLONE_AMD_DEVICES).
type Cipher struct {
	h *C.rc_cipher
}

// Available reports whether librclone_crypt found a HIP device ("gpu = auto").
func Available() bool { return C.xs_device_count() > 0 }

// New wraps keys already derived by Cipher.Key (cipher.go:231-252).
func New(dataKey, nameKey *[32]byte, nameTweak *[16]byte, passBadBlocks bool) (*Cipher, error) {
	var e C.int32_t
	h := C.rc_cipher_new(nil, nil, &e) // empty password: zero keys, no scrypt
	if h == nil {
		return nil, fmt.Errorf("gpucipher: %s", C.GoString(C.rc_error_string(e)))
	}
	C.rc_cipher_set_keys(h, (*C.uint8_t)(unsafe.Pointer(&dataKey[0])), (*C.uint8_t)(unsafe.Pointer(&nameKey[0])),
		(*C.uint8_t)(unsafe.Pointer(&nameTweak[0])))
	C.rc_cipher_set_pass_bad_blocks(h, C.int32_t(cbool(passBadBlocks)))
	c := &Cipher{h: h}
	runtime.SetFinalizer(c, func(c *Cipher) { C.rc_cipher_free(c.h) })
	return c, nil
}

// ComputeHashWithNonce is computeHashWithNonce (crypt.go:784-806) for MD5 after src.Open: in is
// read to EOF, sealed with nonce on the GPU -- concurrent checkers' seals share launches -- and
// "RCLONE\0\0" || nonce || wire blocks is MD5'd on host cores; in is closed when it is an
// io.Closer (the library does what `defer fs.CheckClose(in, &err)` does).  It returns what the
// reference returns from that point: ("", "failed to hash data: %w") for a read error, the hex
// digest and nil, or the hex digest with the close error.  crypt.go's change, after src.Open:
//
//	if f.cipher.gpu != nil && hashType == hash.MD5 {
//		return f.cipher.gpu.ComputeHashWithNonce((*[24]byte)(&nonce), in)
//	}
//	defer fs.CheckClose(in, &err) // the Go path, unchanged
func (c *Cipher) ComputeHashWithNonce(nonce *[24]byte, in io.Reader) (hashStr string, err error) {
	var sum [16]byte
	t := &errTable{}
	box := &readerBox{r: in, t: t}
	hd := cgo.NewHandle(box)
	defer hd.Delete()
	_, closer := in.(io.Closer)
	rc := C.gpucipher_compute_hash(c.h, C.uintptr_t(hd), cbool(closer), (*C.uint8_t)(unsafe.Pointer(&nonce[0])),
		(*C.uint8_t)(unsafe.Pointer(&sum[0])))
	runtime.KeepAlive(c)
	switch {
	case rc == C.RC_NIL:
		return hex.EncodeToString(sum[:]), nil
	case rc == C.RC_ERR_GPU:
		return "", fmt.Errorf("failed to hash data: gpucipher: %s", C.GoString(C.xs_last_error()))
	case box.readErr || !closer:
		return "", fmt.Errorf("failed to hash data: %w", t.err(rc)) // io.Copy's error
	default:
		return hex.EncodeToString(sum[:]), t.err(rc) // every read succeeded: CheckClose's error
	}
}

// ---------------------------------------------------------------------------- encrypter

// Encrypter is an io.Reader of the encrypted stream (cipher.go:681 encrypter).
type Encrypter struct {
	c    *Cipher
	h    *C.rc_encrypter
	t    *errTable
	hd   cgo.Handle
	done sync.Once // hd deleted: the stream has finished and the library reads its source no more
}

// NewEncrypter is newEncrypter(in, nonce) (cipher.go:694).  The nonce must be given: the
// caller draws it from c.cryptoRand exactly as the Go path does, so Nonce() is the initial
// nonce before the first Read (crypt.go:536, :727).
func (c *Cipher) NewEncrypter(in io.Reader, nonce *[24]byte) (*Encrypter, error) {
	t := &errTable{}
	hd := cgo.NewHandle(&readerBox{r: in, t: t})
	var e C.int32_t
	h := C.gpucipher_encrypt(c.h, C.uintptr_t(hd), (*C.uint8_t)(unsafe.Pointer(&nonce[0])), &e)
	if h == nil {
		hd.Delete()
		return nil, t.err(e)
	}
	fh := &Encrypter{c: c, h: h, t: t, hd: hd}
	runtime.SetFinalizer(fh, func(fh *Encrypter) {
		C.rc_encrypter_free(fh.h)
		fh.release()
	})
	return fh, nil
}

func (fh *Encrypter) release() { fh.done.Do(fh.hd.Delete) }

// SetMD5 makes the encrypter take crypt.put's ciphertext hash itself (crypt.go:516-533), hashed
// on host workers while the wrapped Put reads; call it before the first Read.  put then skips its
// TeeReader and uses MD5() as srcHash.
func (fh *Encrypter) SetMD5() error {
	rc := C.rc_encrypter_set_md5(fh.h, 1)
	runtime.KeepAlive(fh)
	if rc != C.RC_NIL {
		return errors.New("gpucipher: SetMD5 after the first Read")
	}
	return nil
}

// MD5 is the MD5 of exactly the bytes Read has returned (hasher.Sums() of the TeeReader).
func (fh *Encrypter) MD5() (sum [16]byte, err error) {
	rc := C.rc_encrypter_md5(fh.h, (*C.uint8_t)(unsafe.Pointer(&sum[0])))
	runtime.KeepAlive(fh)
	if rc != C.RC_NIL {
		return sum, errors.New("gpucipher: MD5 without SetMD5")
	}
	return sum, nil
}

// Read as per io.Reader (cipher.go:719): the library copies into p and never retains it.
func (fh *Encrypter) Read(p []byte) (int, error) {
	if len(p) == 0 {
		return 0, nil
	}
	var e C.int32_t
	n := C.rc_encrypter_read(fh.h, (*C.uint8_t)(unsafe.Pointer(&p[0])), C.int64_t(len(p)), &e)
	err := fh.t.err(e)
	if err != nil {
		// finish (cipher.go:748-758): the stream is over, the library never reads the source
		// again -- drop its handle now rather than when the finalizer runs
		fh.release()
	}
	runtime.KeepAlive(fh)
	return int(n), err
}

// Nonce is fh.nonce: the initial nonce before the first Read, the next block's after.
func (fh *Encrypter) Nonce() (n [24]byte) {
	C.rc_encrypter_nonce(fh.h, (*C.uint8_t)(unsafe.Pointer(&n[0])))
	runtime.KeepAlive(fh)
	return n
}

// ---------------------------------------------------------------------------- decrypter

// Decrypter is io.ReadCloser + io.Seeker + fs.RangeSeeker of plaintext (cipher.go:776
// decrypter, :69-74 ReadSeekCloser).
type Decrypter struct {
	c    *Cipher
	h    *C.rc_decrypter
	s    *openState
	hd   cgo.Handle // of s (DecryptDataSeek only)
	done sync.Once  // Go handles released (Close, or the finalizer as a backstop)
}

func (c *Cipher) newDecrypter(s *openState, h *C.rc_decrypter, hd cgo.Handle) *Decrypter {
	fh := &Decrypter{c: c, h: h, s: s, hd: hd}
	runtime.SetFinalizer(fh, func(fh *Decrypter) {
		C.rc_decrypter_free(fh.h)
		fh.release()
	})
	return fh
}

// release drops the reader and opener handles.  Once closed the library calls none of them:
// Read, Seek and RangeSeek return ErrorFileClosed (cipher.go:1069-1087).
func (fh *Decrypter) release() {
	fh.done.Do(func() {
		fh.s.release()
		if fh.hd != 0 {
			fh.hd.Delete()
		}
	})
}

// DecryptData is newDecrypter(rc) (cipher.go:793, :1099).
func (c *Cipher) DecryptData(rc io.ReadCloser) (*Decrypter, error) {
	s := &openState{t: &errTable{}}
	r := s.newReader(rc, true)
	var e C.int32_t
	h := C.rc_decrypt_data(c.h, r, &e)
	if h == nil {
		err := s.t.err(e)
		s.release()
		return nil, err
	}
	return c.newDecrypter(s, h, 0), nil
}

// DecryptDataSeek is newDecrypterSeek (cipher.go:821, :1112): open is called with the
// underlying (offset, limit) exactly as the reference calls it.
func (c *Cipher) DecryptDataSeek(ctx context.Context, open OpenRangeSeek, offset, limit int64) (*Decrypter, error) {
	s := &openState{ctx: ctx, open: open, t: &errTable{}}
	hd := cgo.NewHandle(s)
	var e, w C.int32_t
	h := C.gpucipher_decrypt_seek(c.h, C.uintptr_t(hd), C.int64_t(offset), C.int64_t(limit), &e, &w)
	runtime.KeepAlive(c)
	if h == nil {
		err := s.t.err(e)
		if e == C.RC_ERR_REOPEN || e == C.RC_ERR_SHORT_NONCE {
			// the opener's own error, wrapped with %w as cipher.go:1011 does, so errors.Is /
			// fserrors.Cause still see context.Canceled, fs.ErrorObjectNotFound, ...
			err = wrap(e, s.t.err(w))
		}
		s.release()
		hd.Delete()
		return nil, err
	}
	return c.newDecrypter(s, h, hd), nil
}

func wrap(code C.int32_t, inner error) error {
	switch code {
	case C.RC_ERR_REOPEN:
		return fmt.Errorf("couldn't reopen file with offset and limit: %w", inner)
	case C.RC_ERR_SHORT_NONCE:
		return fmt.Errorf("short read of nonce: %w", inner)
	}
	return inner
}

func (fh *Decrypter) toErr(code C.int32_t) error {
	if code == C.RC_ERR_REOPEN || code == C.RC_ERR_SHORT_NONCE {
		return wrap(code, fh.s.t.err(C.rc_decrypter_wrapped_error(fh.h)))
	}
	return fh.s.t.err(code)
}

// Read as per io.Reader (cipher.go:901).
func (fh *Decrypter) Read(p []byte) (int, error) {
	if len(p) == 0 {
		return 0, nil
	}
	var e C.int32_t
	n := C.rc_decrypter_read(fh.h, (*C.uint8_t)(unsafe.Pointer(&p[0])), C.int64_t(len(p)), &e)
	err := fh.toErr(e)
	runtime.KeepAlive(fh)
	return int(n), err
}

// RangeSeek (cipher.go:972).
func (fh *Decrypter) RangeSeek(ctx context.Context, offset int64, whence int, limit int64) (int64, error) {
	fh.s.mu.Lock()
	fh.s.ctx = ctx
	fh.s.mu.Unlock()
	var e C.int32_t
	n := C.rc_decrypter_range_seek(fh.h, C.int64_t(offset), C.int32_t(whence), C.int64_t(limit), &e)
	err := fh.toErr(e)
	runtime.KeepAlive(fh)
	return int64(n), err
}

// Seek as per io.Seeker (cipher.go:1037).
func (fh *Decrypter) Seek(offset int64, whence int) (int64, error) {
	return fh.RangeSeek(context.TODO(), offset, whence, -1)
}

// Close (cipher.go:1069): closes the underlying reader once; ErrorFileClosed afterwards.  The
// reader and opener handles are released here (idempotently); the finalizer only frees the
// library handle, and releases the Go handles of a Decrypter that was never closed.
func (fh *Decrypter) Close() error {
	err := fh.toErr(C.rc_decrypter_close(fh.h))
	fh.release()
	runtime.KeepAlive(fh)
	return err
}

// Nonce is fh.nonce (the next block's nonce; the initial nonce right after DecryptData).
func (fh *Decrypter) Nonce() (n [24]byte) {
	C.rc_decrypter_nonce(fh.h, (*C.uint8_t)(unsafe.Pointer(&n[0])))
	runtime.KeepAlive(fh)
	return n
}

// ---------------------------------------------------------------------------- cryptcheck

// HashBatchWithNonce is computeHashWithNonce (crypt.go:784) for MD5 over many sources at once:
// each source is read to EOF, closed (fs.CheckClose), sealed with its nonce and its crypt file
// MD5'd on the GPU.  errs[i] is the reference's "failed to hash data: %w" for a failing source.
func (c *Cipher) HashBatchWithNonce(nonces [][24]byte, srcs []io.ReadCloser) (sums [][16]byte, errs []error, err error) {
	n := len(srcs)
	if len(nonces) != n {
		// fewer nonces would hash sources with zero nonces and report false differences
		return nil, nil, fmt.Errorf("gpucipher: %d nonces for %d sources", len(nonces), n)
	}
	if n == 0 {
		return nil, nil, nil
	}
	t := &errTable{}
	handles := unsafe.Slice((*C.uintptr_t)(C.malloc(C.size_t(n)*C.size_t(unsafe.Sizeof(C.uintptr_t(0))))), n)
	defer C.free(unsafe.Pointer(&handles[0]))
	hds := make([]cgo.Handle, n)
	for i, s := range srcs {
		hds[i] = cgo.NewHandle(&readerBox{r: s, t: t})
		handles[i] = C.uintptr_t(hds[i])
	}
	defer func() {
		for _, h := range hds {
			h.Delete()
		}
	}()
	flat := make([]byte, 24*n)
	for i := range nonces {
		copy(flat[24*i:], nonces[i][:])
	}
	md5 := make([]byte, 16*n)
	codes := make([]C.int32_t, n)
	rc := C.gpucipher_hash_batch(c.h, C.uint64_t(n), &handles[0], C.uint64_t(len(nonces)),
		(*C.uint8_t)(unsafe.Pointer(&flat[0])), (*C.uint8_t)(unsafe.Pointer(&md5[0])), &codes[0])
	runtime.KeepAlive(c) // the finalizer must not free c.h while the batch runs
	if rc != C.RC_NIL {
		return nil, nil, fmt.Errorf("gpucipher: %s", C.GoString(C.xs_last_error()))
	}
	sums, errs = make([][16]byte, n), make([]error, n)
	for i := range sums {
		copy(sums[i][:], md5[16*i:])
		if codes[i] != C.RC_NIL {
			errs[i] = fmt.Errorf("failed to hash data: %w", t.err(codes[i]))
		}
	}
	return sums, errs, nil
}
