/*
 * rclone_crypt_gpu.h -- C ABI of the MI355X (gfx950) crypt-overlay data path.
 *
 * Drop-in boundary for rclone's backend/crypt data cipher (reference v1.76.0,
 * /root/reference).  Two layers, both plain C (pointers + sizes, no torch/HIP types):
 *
 *  1. xs_*  -- the primitive seam.  Batched NaCl secretbox over crypt blocks, replacing the
 *     per-block calls secretbox.Seal (backend/crypt/cipher.go:737) and secretbox.Open
 *     (cipher.go:880) of x/crypto v0.54.0.  Block i of an object uses nonce0 + i
 *     (nonce.add, cipher.go:665-678).  Wire layout of a block: tag(16) || ciphertext(n),
 *     blocks back to back with stride 65552 (cipher.go:39-40, EncryptedSize :1121).
 *     *_dev entry points take device pointers and a hipStream_t passed as void*.
 *     xs_engine_* take host pointers (pinned via xs_host_alloc for full speed) and
 *     overlap H2D / kernels / D2H on side streams.
 *
 *  2. rc_*  -- the cipher.go data API itself (Cipher, EncryptData, DecryptData,
 *     DecryptDataSeek, RangeSeek, EncryptedSize, DecryptedSize, nonce arithmetic) with the
 *     same argument meaning, error values and error precedence, io.Reader expressed as
 *     a C callback.  This is what a cgo binding of backend/crypt would call.
 *
 * Thread safety: xs_*_dev are reentrant (callers own workspace and stream); an xs_engine
 * serialises its own calls; rc_* handles serialise per handle like the reference's fh.mu
 * (cipher.go:682, :778) and may be used from many threads at once.
 */
#ifndef RCLONE_CRYPT_GPU_H
#define RCLONE_CRYPT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XS_BLOCK_DATA 65536u /* blockDataSize cipher.go:39 */
#define XS_BLOCK_HDR 16u     /* blockHeaderSize = secretbox.Overhead cipher.go:38 */
#define XS_BLOCK_SIZE 65552u /* blockSize cipher.go:40 */
#define XS_FILE_HDR 32u      /* fileHeaderSize cipher.go:37 */

/* xs_* return codes */
#define XS_OK 0
#define XS_ERR_INVALID (-1) /* bad argument / size / alignment */
#define XS_ERR_HIP (-2)     /* HIP runtime error (see xs_last_error) */
#define XS_ERR_NOMEM (-3)
#define XS_ERR_NODEV (-4)

/* One crypt block of a batch (descriptor mode).  Offsets are bytes from the src / dst
 * base pointers.  Seal: src_off -> plaintext, dst_off -> wire block (tag first).
 * Open: src_off -> wire block (tag first), dst_off -> plaintext.  len = plaintext bytes
 * (1..65536).  Payload addresses (plaintext and ciphertext = wire + 16) must be 16-byte
 * aligned.  reserved: 0 (the engine uses it internally for ranged opens; the *_batch_dev entry
 * points ignore it). */
typedef struct xs_block_desc {
  uint64_t src_off;
  uint64_t dst_off;
  uint32_t len;
  uint32_t reserved;
  uint8_t nonce[24];
} xs_block_desc;

/* One MD5 stream for xs_md5_batch_dev: prefix[0:prefix_len] (prefix_len 0, 16 or 32 -- the
 * 32-byte crypt header "RCLONE\0\0" || nonce, cipher.go:34-37) followed by len bytes at byte
 * offset off (16-byte aligned) of the source buffer. */
typedef struct xs_md5_desc {
  uint64_t off;
  uint64_t len;
  uint8_t prefix[32];  /* 16-byte aligned within the (16-byte aligned) descriptor array */
  uint32_t prefix_len;
  uint32_t reserved[3];
} xs_md5_desc;  /* 64 bytes */

const char *xs_version(void);
/* sha256 (hex) of the sources and build flags the library was compiled from
   (rclone_amd/build.py build_sources_sha256); "unstamped" for a build outside it. */
const char *xs_build_id(void);
/* Last error message of the calling thread ("" if none). */
const char *xs_last_error(void);
/* Number of HIP devices (0 when none; never fails). */
int xs_device_count(void);
/* Device workspace bytes needed for a batch of nblocks (per-block key schedule). */
size_t xs_workspace_bytes(uint64_t nblocks);

/* Seal a contiguous plaintext object range: blocks first_block.. of an object whose block 0
 * uses nonce0.  d_plain holds plain_len bytes (block i at i*65536); d_body receives the
 * wire blocks (block i at i*65552; EncryptedSize(plain_len)-32 bytes for a whole object).
 * Replaces the secretbox.Seal loop of encrypter.Read (cipher.go:719-745). */
int xs_seal_object_dev(const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                       const void *d_plain, uint64_t plain_len, void *d_body, void *d_workspace,
                       void *stream);
/* Open wire blocks (body_len bytes, block i at i*65552) into d_plain (block i at i*65536).
 * d_ok[i] = 1 if block i authenticated, else 0 and that block's plaintext is zero-filled
 * (secretbox.Open failure, cipher.go:880-893).  Every block must hold > 16 bytes.
 * Unlike x/crypto's Open, which writes nothing on failure, the kernels decrypt and verify in one
 * pass: a failed block's unauthenticated plaintext is in the destination between its stores and
 * the zero-fill, both inside the same launch.  Read the destination only after the call's work
 * has completed (stream-ordered here; the engine calls below return after completion), never
 * concurrently with it.  This applies to every open entry point of this header. */
int xs_open_object_dev(const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                       const void *d_body, uint64_t body_len, void *d_plain, uint8_t *d_ok,
                       void *d_workspace, void *stream);
/* Descriptor mode: d_desc is a device array of nblocks descriptors; src/dst buffers are
 * src_len/dst_len bytes.  A descriptor that is out of bounds, misaligned or has len outside
 * 1..65536 is skipped on the device (nothing written; d_ok[i] = 0 when opening), so a bad
 * descriptor can never fault the GPU. */
int xs_seal_batch_dev(const uint8_t key[32], const xs_block_desc *d_desc, uint64_t nblocks,
                      const void *d_src, uint64_t src_len, void *d_dst, uint64_t dst_len,
                      void *d_workspace, void *stream);
int xs_open_batch_dev(const uint8_t key[32], const xs_block_desc *d_desc, uint64_t nblocks,
                      const void *d_src, uint64_t src_len, void *d_dst, uint64_t dst_len, uint8_t *d_ok,
                      void *d_workspace, void *stream);
/* The two halves of xs_seal_object_dev / xs_open_object_dev, for callers that pipeline or
 * time the kernels separately: xs_keygen_object_dev writes the per-block key schedule
 * (nonce, HSalsa20 subkey, Poly1305 key and power tables) into d_workspace for the object
 * range (len = plaintext bytes when seal != 0, wire-body bytes otherwise); xs_crypt_dev then
 * runs the block kernel over nblocks blocks of that schedule. */
int xs_keygen_object_dev(int seal, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         uint64_t len, void *d_workspace, void *stream);
int xs_crypt_dev(int seal, const void *d_workspace, uint64_t nblocks, const void *d_src, void *d_dst,
                 uint8_t *d_ok, void *stream);
/* Key-schedule half of xs_seal_batch_dev / xs_open_batch_dev (descriptor mode). */
int xs_keygen_batch_dev(int seal, const uint8_t key[32], const xs_block_desc *d_desc, uint64_t nblocks,
                        const void *d_src, uint64_t src_len, const void *d_dst, uint64_t dst_len,
                        void *d_workspace, void *stream);
/* Fill d with the SplitMix64 stream (word k = mix(seed + (k+1)*0x9E3779B97F4A7C15)). */
int xs_fill_random_dev(void *d, uint64_t nbytes, uint64_t seed, void *stream);
/* Fill nblocks 64 KiB blocks: local block b = global block first_block + b*block_stride of the
 * same stream (a rank's round-robin share of a synthetic object set, BASELINE configs[3]). */
int xs_fill_blocks_dev(void *d, uint64_t nblocks, uint64_t first_block, uint64_t block_stride, uint64_t seed,
                       void *stream);
/* Check nblocks 64 KiB blocks at d against the stream xs_fill_blocks_dev(.., first_block,
 * block_stride, seed) writes: the number of differing 64-bit words is added to *d_mismatch (device
 * memory, 8-byte aligned).  The object-set benchmark's round-trip check. */
int xs_verify_blocks_dev(const void *d, uint64_t nblocks, uint64_t first_block, uint64_t block_stride, uint64_t seed,
                         uint64_t *d_mismatch, void *stream);

/* Shader-clock probe (benchmarking): one wave on `stream` records s_memtime against the 100 MHz
 * s_memrealtime until *d_stop (device memory, 0 at launch) becomes non-zero or max_seconds pass;
 * d_out[0..4] = start shader ticks, start 100 MHz ticks, end shader ticks, end 100 MHz ticks,
 * samples.  Clock (GHz) = (d_out[2]-d_out[0]) / (d_out[3]-d_out[1]) / 10. */
int xs_clock_probe_dev(const uint32_t *d_stop, uint64_t *d_out, double max_seconds, void *stream);

/* MD5 of n streams in HBM, one lane per stream (crypt.go:516-533 put's ciphertext hash,
 * :784-806 computeHashWithNonce): d_digest[16*i] = MD5(prefix_i || src[off_i : off_i+len_i]).
 * An invalid descriptor (bounds, alignment, prefix_len) gets d_ok[i] = 0 (d_ok may be NULL)
 * and an unspecified digest. */
int xs_md5_batch_dev(const xs_md5_desc *d_desc, uint64_t n, const void *d_src, uint64_t src_len,
                     uint8_t *d_digest, uint8_t *d_ok, void *stream);

/* Host-memory engine: pinned staging, per-slot streams, H2D/kernel/D2H overlapped. */
typedef struct xs_engine xs_engine;
xs_engine *xs_engine_create(int device, uint32_t batch_blocks, int nslots);
void xs_engine_destroy(xs_engine *e);
int xs_engine_seal(xs_engine *e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void *plain, uint64_t plain_len, void *body);
/* xs_engine_open: ok[i] as d_ok above.  With pinned (zero-copy) buffers the kernels write the
 * plaintext straight into `plain`, so a failed block's bytes transit the caller's buffer before
 * its zero-fill; the call returns only after both, and `plain` must not be read by another
 * thread while the call runs. */
int xs_engine_open(xs_engine *e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void *body, uint64_t body_len, void *plain, uint8_t *ok);
/* xs_engine_open for a caller that will read only plaintext bytes [range_lo, range_hi) of
 * `plain` (offsets within this call's plaintext): the decrypter after RangeSeek with a limit
 * (cipher.go:972-1034), whose reads stop at offset + limit.  Every block's tag is verified over the
 * whole block and ok[] is as for xs_engine_open, but bytes of `plain` outside the range may be
 * left unwritten: a ranged 4 KiB read then decrypts one or two 4 KiB groups of its block instead
 * of all sixteen.  A failed block is zero-filled whole, as before. */
int xs_engine_open_range(xs_engine *e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         const void *body, uint64_t body_len, void *plain, uint8_t *ok, uint64_t range_lo,
                         uint64_t range_hi);
/* Seal many host objects and MD5 their crypt files on the GPU -- the hash Fs.put tees off the
 * ciphertext (crypt.go:516-533) and cryptcheck's computeHashWithNonce (crypt.go:784-806),
 * batched across objects: object i = plain[offs[i] : offs[i]+lens[i]] (offs 16-byte aligned),
 * block j sealed with nonces[24i..] + j; md5[16i..] = MD5("RCLONE\0\0" || nonce_i || wire
 * blocks).  Only the digests come back over PCIe.  MD5 runs one GPU lane per object, so this
 * pays off for many objects per call (hundreds+), not for one large stream. */
int xs_engine_seal_md5(xs_engine *e, const uint8_t key[32], uint64_t nobj, const uint8_t *nonces,
                       const uint64_t *offs, const uint64_t *lens, const void *plain, uint8_t *md5);
/* Fs.put of many whole objects at once (rclone sync/copy of a tree into crypt; replaces, per
 * object, encryptData + the ciphertext MD5 tee of crypt.go:507-536 feeding the wrapped put):
 * the same
 * seal + ciphertext MD5 as xs_engine_seal_md5, and the wire bodies come back too, packed into
 * `body`: object i's body (rc_encrypted_size(len) - 32 bytes: tag||ct per block, no header)
 * starts at the sum over k < i of round16(body bytes of object k).  One D2H per group.
 * xs_put_body_bytes gives the total packed size for the `body` buffer (pinned for speed). */
int xs_engine_put_batch(xs_engine *e, const uint8_t key[32], uint64_t nobj, const uint8_t *nonces,
                        const uint64_t *offs, const uint64_t *lens, const void *plain, void *body,
                        uint8_t *md5);
uint64_t xs_put_body_bytes(uint64_t nobj, const uint64_t *lens);
/* Cross-caller coalescing (default on; env XS_ENGINE_COALESCE=0 or this call turns it off):
 * concurrent xs_engine_seal/xs_engine_open callers whose request fits one engine batch are
 * packed into one combined GPU batch (group commit: the first caller in leads, the others
 * wait).  Results, errors and per-caller buffers are exactly those of separate calls. */
void xs_engine_set_coalesce(xs_engine *e, int on);
/* Cumulative coalescing counters: out[0] combined batches, out[1] requests, out[2] blocks. */
void xs_engine_stats(xs_engine *e, uint64_t out[3]);
/* Objects routed off the GPU MD5 lanes by xs_engine_seal_md5 / xs_engine_put_batch: the
 * longest objects of a group are hashed on host cores over the GPU-sealed wire body when that
 * shortens the group (one GPU lane does ~70 MB/s, one core ~10x that).  threads = host MD5
 * workers (0 = every object on the GPU; default XS_MD5_HOST_THREADS or half the cores, <= 8).
 * out[0] = objects hashed on the host so far, out[1] = their wire bytes, out[2] = all objects
 * sealed + hashed by this engine. */
void xs_engine_set_host_md5(xs_engine *e, int threads);
void xs_engine_md5_stats(xs_engine *e, uint64_t out[3]);

/* Multi-device engine pool: one process spreads its objects over several GPUs (or several
 * engines per GPU).  devices = HIP device ids, repeats allowed ("0,0,0,0" = four engines on
 * device 0); NULL / ndevices <= 0 -> env RCLONE_AMD_DEVICES (comma list), else RCLONE_AMD_DEVICE,
 * else every visible device.  xs_pool_next hands out engines round-robin (one per object
 * stream, fs/sync/sync.go:544 --transfers); xs_pool_seal_md5 / xs_pool_put_batch split their
 * objects into contiguous byte-balanced ranges run concurrently, one engine each, with results
 * identical to one engine's. */
typedef struct xs_pool xs_pool;
xs_pool *xs_pool_create(const int *devices, int ndevices, uint32_t batch_blocks, int nslots);
void xs_pool_destroy(xs_pool *p);
int xs_pool_size(const xs_pool *p);
xs_engine *xs_pool_engine(xs_pool *p, int i);
xs_engine *xs_pool_next(xs_pool *p);
int xs_pool_seal_md5(xs_pool *p, const uint8_t key[32], uint64_t nobj, const uint8_t *nonces,
                     const uint64_t *offs, const uint64_t *lens, const void *plain, uint8_t *md5);
int xs_pool_put_batch(xs_pool *p, const uint8_t key[32], uint64_t nobj, const uint8_t *nonces,
                      const uint64_t *offs, const uint64_t *lens, const void *plain, void *body, uint8_t *md5);

/* Pinned (page-locked) host memory. */
void *xs_host_alloc(size_t bytes);
/* ... placed on NUMA node `node` (preferred-node policy during the allocation; node < 0: no
 * preference).  Free with xs_host_free. */
void *xs_host_alloc_node(size_t bytes, int node);
void xs_host_free(void *p);

/* Node topology (one process over a multi-socket 8-GPU node): each engine's
 * pinned staging, its handles' staging and the host threads the library starts for it (host MD5,
 * batched-call ranges) are placed on the NUMA node of the engine's GPU.  The sysfs root is
 * RCLONE_AMD_SYSFS_ROOT (default /sys); RCLONE_AMD_NUMA=0 turns placement off. */
int xs_device_numa_node(int device);          /* NUMA node of a HIP device's PCI function, or -1 */
int xs_engine_numa_node(const xs_engine *e);  /* the node the engine's host resources use, or -1 */
int xs_engine_device(const xs_engine *e);     /* the HIP device the engine runs on, or -1 */
int xs_pci_numa_node(const char *pci_bus_id); /* <root>/bus/pci/devices/<id>/numa_node, or -1 */
/* CPUs of a node (<root>/devices/system/node/node<N>/cpulist): writes up to cap, returns the count
 * (0 when unknown). */
int xs_numa_node_cpus(int node, int *cpus, int cap);
/* Parse a device list as RCLONE_AMD_DEVICES ("0,1,1,2": repeats allowed); returns the count. */
int xs_parse_device_list(const char *list, int *out, int cap);
/* CPUs this process may use: its affinity mask capped by the cgroup CPU quota (cpu.max under the
 * sysfs root; RCLONE_AMD_CPUS overrides).  The host MD5 tiers size themselves by it. */
int xs_effective_cpus(void);

/* ------------------------------------------------------------------------------------
 * rc_*: backend/crypt/cipher.go data API.
 * Error values (int32): RC_NIL, RC_EOF (io.EOF), RC_UNEXPECTED_EOF (io.ErrUnexpectedEOF),
 * the crypt sentinels below (cipher.go:44-58), or any value >= RC_USER_BASE produced by a
 * caller's reader / opener, which is passed through unchanged exactly where the
 * reference passes the underlying error through.
 * ---------------------------------------------------------------------------------- */
#define RC_NIL 0
#define RC_EOF 1
#define RC_UNEXPECTED_EOF 2
#define RC_USER_BASE 16
#define RC_ERR_FILE_TOO_SHORT (-101) /* ErrorEncryptedFileTooShort */
#define RC_ERR_FILE_BAD_HEADER (-102) /* ErrorEncryptedFileBadHeader */
#define RC_ERR_BAD_MAGIC (-103)       /* ErrorEncryptedBadMagic */
#define RC_ERR_BAD_BLOCK (-104)       /* ErrorEncryptedBadBlock */
#define RC_ERR_FILE_CLOSED (-105)     /* ErrorFileClosed */
#define RC_ERR_BAD_SEEK (-106)        /* ErrorBadSeek */
#define RC_ERR_SHORT_NONCE (-107)     /* "short read of nonce: %w" (cipher.go:633) */
#define RC_ERR_SEEK_NOT_INIT (-108)   /* "can't seek - not initialised with newDecrypterSeek" */
#define RC_ERR_SEEK_WHENCE (-109)     /* "can only seek from the start" */
#define RC_ERR_REOPEN (-110)          /* "couldn't reopen file with offset and limit: %w" */
#define RC_ERR_GPU (-120)             /* device failure (xs_last_error has the reason) */
#define RC_ERR_INVALID (-121)

/* io.Reader: read up to n bytes into p, return the count (>= 0) and set *err. */
typedef int64_t (*rc_read_fn)(void *user, uint8_t *p, int64_t n, int32_t *err);
/* io.Closer */
typedef int32_t (*rc_close_fn)(void *user);
/* optional fs.RangeSeeker (fs/types.go, used at cipher.go:997) */
typedef int32_t (*rc_range_seek_fn)(void *user, int64_t offset, int32_t whence, int64_t limit);
typedef struct rc_reader {
  rc_read_fn read;
  rc_close_fn close;           /* may be NULL (io.NopCloser) */
  rc_range_seek_fn range_seek; /* may be NULL */
  /* Opaque: never dereferenced, only passed back to the callbacks.  A cgo binding stores a
   * cgo.Handle here as (void *)(uintptr_t)h from C code and gets it back as uintptr_t
   *  -- Go code never converts the integer to unsafe.Pointer. */
  void *user;
} rc_reader;
/* OpenRangeSeek (cipher.go:77): open the underlying object at (offset, limit). */
typedef int32_t (*rc_open_fn)(void *user, int64_t offset, int64_t limit, rc_reader *out);

typedef struct rc_cipher rc_cipher;
typedef struct rc_encrypter rc_encrypter;
typedef struct rc_decrypter rc_decrypter;

/* newCipher + Key (cipher.go:187, :231): scrypt(N=16384,r=8,p=1) key derivation; empty
 * password -> all-zero keys; empty salt -> built-in defaultSalt. */
rc_cipher *rc_cipher_new(const char *password, const char *salt, int32_t *err);
int32_t rc_cipher_key(rc_cipher *c, const char *password, const char *salt);
void rc_cipher_keys(const rc_cipher *c, uint8_t data_key[32], uint8_t name_key[32], uint8_t name_tweak[16]);
/* Install keys derived elsewhere (a Go binding that already ran Cipher.Key, cipher.go:231). */
void rc_cipher_set_keys(rc_cipher *c, const uint8_t data_key[32], const uint8_t name_key[32],
                        const uint8_t name_tweak[16]);
void rc_cipher_set_pass_bad_blocks(rc_cipher *c, int32_t pass); /* setPassBadBlocks :217 */
void rc_cipher_set_rand(rc_cipher *c, rc_reader rand);           /* c.cryptoRand */
/* Read-ahead of encrypters/decrypters.  The first refill of a stream, and the first after a
 * seek, reads first_blocks blocks (default 1: exactly what encrypter.Read / fillBuffer read,
 * cipher.go:726-741, :862-898); later refills grow up to batch_blocks per GPU submission
 * (default 64 = 4 MiB): by `factor` each refill, or with factor 0 (default) by doubling while
 * the source is slow and straight to batch_blocks once a refill read faster than 2 GB/s.
 * first_blocks = 0: every refill reads batch_blocks. */
void rc_cipher_set_batch_blocks(rc_cipher *c, uint32_t blocks);
void rc_cipher_set_readahead(rc_cipher *c, uint32_t first_blocks);
void rc_cipher_set_readahead_growth(rc_cipher *c, uint32_t factor);
/* GPU engines used by this cipher's handles and batches (NULL: the process-wide pool over
 * RCLONE_AMD_DEVICES / RCLONE_AMD_DEVICE / every device).  The pool must outlive the cipher. */
void rc_cipher_set_pool(rc_cipher *c, xs_pool *pool);
/* The process-wide pool (created on first use; NULL with xs_last_error when no device). */
xs_pool *rc_default_pool(void);
void rc_cipher_free(rc_cipher *c);

int64_t rc_encrypted_size(int64_t size);               /* EncryptedSize :1121 */
int64_t rc_decrypted_size(int64_t size, int32_t *err); /* DecryptedSize :1131 */
void rc_calculate_underlying(int64_t offset, int64_t limit, int64_t out[4]); /* :935 */
void rc_nonce_increment(uint8_t nonce[24]);            /* :660 */
void rc_nonce_add(uint8_t nonce[24], uint64_t x);      /* :665 */

/* newEncrypter (cipher.go:694) / EncryptData (:771).  nonce NULL -> read 24 bytes from the
 * cipher's random source.  On error returns NULL and sets *err. */
rc_encrypter *rc_encrypt_data(rc_cipher *c, rc_reader in, const uint8_t *nonce, int32_t *err);
int64_t rc_encrypter_read(rc_encrypter *e, uint8_t *p, int64_t n, int32_t *err); /* :719 */
void rc_encrypter_nonce(const rc_encrypter *e, uint8_t out[24]);
/* crypt.put's ciphertext hash (crypt.go:516-533: io.TeeReader(wrappedIn, MD5 hasher)) taken by the
 * encrypter itself, so the Go side drops the TeeReader: call rc_encrypter_set_md5(e, 1) before the
 * first read (RC_ERR_INVALID after it).  A host worker hashes each sealed batch while the consumer
 * reads it.  rc_encrypter_md5 returns the MD5 of exactly the bytes returned by rc_encrypter_read so
 * far -- what hasher.Sums() gives after the wrapped Put -- or RC_ERR_INVALID if the option is off. */
int32_t rc_encrypter_set_md5(rc_encrypter *e, int32_t on);
int32_t rc_encrypter_md5(rc_encrypter *e, uint8_t out[16]);
void rc_encrypter_free(rc_encrypter *e);

/* newDecrypter / DecryptData (:793, :1099) */
rc_decrypter *rc_decrypt_data(rc_cipher *c, rc_reader rc, int32_t *err);
/* DecryptDataSeek (:1112) */
rc_decrypter *rc_decrypt_data_seek(rc_cipher *c, rc_open_fn open, void *open_user, int64_t offset,
                                   int64_t limit, int32_t *err);
/* DecryptDataSeek with the wrapped error: when *err is RC_ERR_REOPEN (or RC_ERR_SHORT_NONCE) the
 * handle is gone, and *wrapped receives the opener's own error -- the %w operand of "couldn't
 * reopen file with offset and limit: %w" (cipher.go:1011) -- so the binding can wrap the real
 * cause (errors.Is on context.Canceled, fs.ErrorObjectNotFound, ...).  wrapped may be NULL. */
rc_decrypter *rc_decrypt_data_seek_ex(rc_cipher *c, rc_open_fn open, void *open_user, int64_t offset,
                                      int64_t limit, int32_t *err, int32_t *wrapped);
int64_t rc_decrypter_read(rc_decrypter *d, uint8_t *p, int64_t n, int32_t *err); /* :901 */
int64_t rc_decrypter_range_seek(rc_decrypter *d, int64_t offset, int32_t whence, int64_t limit,
                                int32_t *err);                                   /* :972 */
int32_t rc_decrypter_close(rc_decrypter *d);                                     /* :1069 */
void rc_decrypter_nonce(const rc_decrypter *d, uint8_t out[24]);
/* error wrapped by RC_ERR_REOPEN / RC_ERR_SHORT_NONCE (the %w operand) */
int32_t rc_decrypter_wrapped_error(const rc_decrypter *d);
void rc_decrypter_free(rc_decrypter *d);

/* Fs.computeHashWithNonce (crypt.go:784-806) for MD5, batched over n source objects -- the
 * cryptcheck / bisync check path (cmd/cryptcheck/cryptcheck.go:67-117): reads srcs[i] to EOF
 * in 64 KiB ReadFills (as newEncrypter would), closes it if it has a close function
 * (fs.CheckClose), seals it with nonces[24i..] and MD5s the crypt file, all on the GPU
 * (xs_engine_seal_md5).  errs[i] = RC_NIL with md5[16i..] set, or the reader's / closer's
 * error (the reference returns it wrapped as "failed to hash data: %w").  Returns RC_NIL, or
 * RC_ERR_GPU if the engine failed (no digest valid). */
int32_t rc_hash_batch_with_nonce(rc_cipher *c, uint64_t n, const rc_reader *srcs, const uint8_t *nonces,
                                 uint8_t *md5, int32_t *errs);
/* Fs.computeHashWithNonce (crypt.go:784-806) for MD5, one object: the call crypt.go's own
 * computeHashWithNonce makes, per object, from unchanged cryptcheck / bisync checkers
 * (cmd/cryptcheck/cryptcheck.go:91-114; concurrency = --checkers).  Reads src to EOF (ReadFill of
 * one block at a time, as newEncrypter would), seals it on the GPU (concurrent callers' seals are
 * group-committed into shared launches), MD5s "RCLONE\0\0" || nonce || wire blocks on host cores
 * (one core hashes a stream ~10x faster than one GPU lane), overlapping batch k's hash with batch
 * k+1's read and seal, then closes src if it has a close function (defer fs.CheckClose(in, &err)).
 * Returns RC_NIL with md5 set; the reader's non-EOF error (io.Copy's, which the reference wraps as
 * "failed to hash data: %w"); the closer's error when every read succeeded -- md5 is then set too,
 * as the reference returns hashStr alongside CheckClose's error; or RC_ERR_GPU. */
int32_t rc_compute_hash_with_nonce(rc_cipher *c, rc_reader src, const uint8_t nonce[24], uint8_t md5[16]);

/* ------------------------------------------------------------------------------------
 * File-name cipher (cipher.go:120-618): NameEncryptionMode, fileNameEncoding, encryptSegment /
 * decryptSegment (EME-AES-256 over pkcs7-padded names, github.com/rfjakob/eme v1.2.0, run on
 * the GPU by xs_eme_batch_dev), obfuscateSegment / deobfuscateSegment, Encrypt/DecryptFileName,
 * Encrypt/DecryptDirName, with lib/version handling and the encrypted suffix of mode "off".
 * ---------------------------------------------------------------------------------- */
#define RC_NAME_OFF 0        /* NameEncryptionOff (cipher.go:87) */
#define RC_NAME_STANDARD 1   /* NameEncryptionStandard */
#define RC_NAME_OBFUSCATE 2  /* NameEncryptionObfuscated */
#define RC_ENC_BASE32 0      /* caseInsensitiveBase32Encoding (cipher.go:127-152) */
#define RC_ENC_BASE64 1      /* base64.RawURLEncoding */
#define RC_ENC_BASE32768 2   /* base32768.SafeEncoding (github.com/Max-Sum/base32768) */

#define RC_ERR_NOT_A_MULTIPLE_OF_BLOCKSIZE (-130) /* ErrorNotAMultipleOfBlocksize */
#define RC_ERR_TOO_SHORT_AFTER_DECODE (-131)      /* ErrorTooShortAfterDecode */
#define RC_ERR_TOO_LONG_AFTER_DECODE (-132)       /* ErrorTooLongAfterDecode */
#define RC_ERR_BAD_BASE32_ENCODING (-133)         /* ErrorBadBase32Encoding */
#define RC_ERR_NOT_AN_ENCRYPTED_FILE (-134)       /* ErrorNotAnEncryptedFile */
#define RC_ERR_PKCS7_NOT_FOUND (-140)             /* pkcs7.ErrorPaddingNotFound (pkcs7.go:10) */
#define RC_ERR_PKCS7_NOT_A_MULTIPLE (-141)        /* pkcs7.ErrorPaddingNotAMultiple */
#define RC_ERR_PKCS7_TOO_LONG (-142)              /* pkcs7.ErrorPaddingTooLong */
#define RC_ERR_PKCS7_TOO_SHORT (-143)             /* pkcs7.ErrorPaddingTooShort */
#define RC_ERR_PKCS7_NOT_ALL_THE_SAME (-144)      /* pkcs7.ErrorPaddingNotAllTheSame */
#define RC_ERR_BASE32_CORRUPT (-150)    /* base32.CorruptInputError(arg) */
#define RC_ERR_BASE64_CORRUPT (-151)    /* base64.CorruptInputError(arg) */
#define RC_ERR_BASE32768_CORRUPT (-152) /* base32768.CorruptInputError(arg) */
#define RC_ERR_UNKNOWN_MODE (-153)      /* "unknown file name encryption mode %q" (cipher.go:101) */
#define RC_ERR_UNKNOWN_ENCODING (-154)  /* "unknown file name encoding mode %q" (cipher.go:166) */
#define RC_ERR_NAME_TOO_LONG (-155)     /* padded name > 2048 bytes: eme.Transform panics there */

/* One name for xs_eme_batch_dev: nblk 16-byte blocks (1..128) at byte offset off (16-aligned). */
typedef struct xs_name_desc {
  uint64_t off;
  uint32_t nblk;
  uint32_t reserved;
} xs_name_desc;

/* eme.Transform(aes.NewCipher(name_key), tweak, names, direction) for every descriptor, on the
 * GPU: encrypt != 0 -> DirectionEncrypt.  d_src and d_dst are device buffers of buf_len bytes
 * (they may be the same buffer: in place); each name is read at d_src+off and written at
 * d_dst+off.  A descriptor out of range is skipped (its output is unspecified). */
int xs_eme_batch_dev(int encrypt, const uint8_t name_key[32], const uint8_t tweak[16], const xs_name_desc *d_desc,
                     uint64_t n, const void *d_src, void *d_dst, uint64_t buf_len, void *stream);

/* NewNameEncryptionMode / NewNameEncoding (cipher.go:92, :155): parse a config string. */
int32_t rc_new_name_encryption_mode(const char *s, int32_t *mode);
int32_t rc_new_name_encoding(const char *s, int32_t *enc);
/* newCipher's name arguments (cipher.go:187): mode, dirNameEncrypt, enc; setEncryptedSuffix :207. */
void rc_cipher_set_name_encryption(rc_cipher *c, int32_t mode, int32_t dir_name_encrypt, int32_t enc);
void rc_cipher_set_encrypted_suffix(rc_cipher *c, const char *suffix);

/* fileNameEncoding.EncodeToString / DecodeString for one encoding.  Encode writes at most
 * cap bytes and returns the full encoded length; decode returns RC_NIL or an RC_ERR_* value
 * with *err_arg = the CorruptInputError offset. */
int64_t rc_name_encode(int32_t enc, const uint8_t *src, uint64_t n, char *out, uint64_t cap);
int32_t rc_name_decode(int32_t enc, const char *s, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                       int64_t *err_arg);

/* Batched name operations: one GPU EME launch for every segment of every name in the batch.
 * op: which cipher.go function is applied to each input string. */
#define RC_OP_ENCRYPT_FILE_NAME 0 /* EncryptFileName :542 */
#define RC_OP_DECRYPT_FILE_NAME 1 /* DecryptFileName :600 */
#define RC_OP_ENCRYPT_DIR_NAME 2  /* EncryptDirName :550 */
#define RC_OP_DECRYPT_DIR_NAME 3  /* DecryptDirName :613 */
#define RC_OP_ENCRYPT_SEGMENT 4   /* encryptSegment :280 (standard mode) */
#define RC_OP_DECRYPT_SEGMENT 5   /* decryptSegment :293 (standard mode) */
#define RC_OP_OBFUSCATE_SEGMENT 6 /* obfuscateSegment :315 */
#define RC_OP_DEOBFUSCATE_SEGMENT 7 /* deobfuscateSegment :402 */
typedef struct rc_names rc_names;
/* Runs op over n strings (in[i], in_len[i] bytes).  Returns RC_NIL and *out, or RC_ERR_GPU /
 * RC_ERR_INVALID (no result).  Per-name errors are in the result, as the reference returns them. */
int32_t rc_names_run(rc_cipher *c, int32_t op, uint64_t n, const char *const *in, const uint64_t *in_len,
                     rc_names **out);
/* Result i: string (not NUL-terminated), its length, error value and error argument. */
void rc_names_get(const rc_names *r, uint64_t i, const char **s, uint64_t *len, int32_t *err, int64_t *err_arg);
/* Device time of the batch's EME kernel (ms, HIP events), 0 when no segment went to the GPU. */
double rc_names_kernel_ms(const rc_names *r);
void rc_names_free(rc_names *r);

/* Message of an rc_* error value (the reference's error string). */
const char *rc_error_string(int32_t err);

#ifdef __cplusplus
}
#endif
#endif
