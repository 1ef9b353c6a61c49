// cipher.cpp -- host mirror of the data half of rclone's backend/crypt/cipher.go (v1.76.0)
// behind the rc_* C ABI (include/rclone_crypt_gpu.h).
//
// Same names, argument meaning, error values and error precedence as the reference:
//   Cipher/newCipher/Key          cipher.go:172-252   (rc_cipher_new, rc_cipher_key)
//   nonce carry/increment/add     cipher.go:621-678   (rc_nonce_*)
//   encrypter / newEncrypter / Read / finish / EncryptData   cipher.go:681-774
//   decrypter / newDecrypter / newDecrypterSeek / fillBuffer / Read / RangeSeek / Seek /
//   finish / unFinish / Close / finishAndClose / DecryptData / DecryptDataSeek
//                                 cipher.go:776-1118
//   calculateUnderlying           cipher.go:935-965
//   EncryptedSize / DecryptedSize cipher.go:1121-1146
//
// What differs is only *when* blocks are sealed/opened: instead of one secretbox call per
// 64 KiB block (cipher.go:737, :880) a handle ReadFills up to batch_blocks blocks from the
// underlying reader in the reference's exact call sequence (a short or failed ReadFill ends
// the batch, so the reader sees the same Read calls, just earlier) and seals/opens them in
// one GPU submission through the xs_engine.  Bytes returned, errors returned, the position
// at which each error surfaces and the nonce after EOF are those of the reference.
#include <sys/random.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rclone_crypt_gpu.h"
#include "md5_workers.h"
#include "rc_internal.h"

namespace rc {
bool scrypt(const uint8_t* pw, size_t pwlen, const uint8_t* salt, size_t slen, uint64_t N, int r, int p,
            uint8_t* out, size_t olen);
}

namespace {

constexpr int64_t kBlockData = XS_BLOCK_DATA;
constexpr int64_t kBlockHdr = XS_BLOCK_HDR;
constexpr int64_t kBlockSize = XS_BLOCK_SIZE;
constexpr int64_t kFileHdr = XS_FILE_HDR;
const uint8_t kMagic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};
// defaultSalt cipher.go:59
const uint8_t kDefaultSalt[16] = {0xA8, 0x0D, 0xF4, 0x3A, 0x8F, 0xBD, 0x03, 0x08,
                                  0xA7, 0xCA, 0xB8, 0x3E, 0x58, 0x1F, 0x86, 0xB1};

bool is_pending(int32_t e) { return e != RC_NIL && e != RC_EOF; }  // "err != nil && err != io.EOF"

// readers.ReadFill (lib/readers/readfill.go:11)
int64_t read_fill(const rc_reader& r, uint8_t* buf, int64_t len, int32_t* err) {
  int64_t n = 0;
  int32_t e = RC_NIL;
  while (n < len && e == RC_NIL) {
    int64_t nn = r.read(r.user, buf + n, len - n, &e);
    if (nn < 0) nn = 0;
    n += nn;
  }
  *err = e;
  return n;
}

// ---------------------------------------------------------------- GPU engines (process-wide)
// One pool of engines for the process, over every device in RCLONE_AMD_DEVICES (or
// RCLONE_AMD_DEVICE, or all visible devices): each encrypter / decrypter takes an engine
// round-robin when it first needs the GPU, so the transfers of one rclone process spread over the
// node's GPUs (fs/sync/sync.go:544 startTransfers); a cipher may be bound to its own pool
// (rc_cipher_set_pool).
std::mutex g_pool_create_mu;
std::atomic<xs_pool*> g_xs_pool{nullptr};  // read without the lock once created (every refill asks)
bool g_xs_pool_failed = false;

xs_pool* process_pool() {
  if (xs_pool* p = g_xs_pool.load(std::memory_order_acquire)) return p;
  std::lock_guard<std::mutex> g(g_pool_create_mu);
  if (g_xs_pool.load() || g_xs_pool_failed) return g_xs_pool.load();
  uint32_t batch = 256;
  if (const char* s = getenv("RCLONE_AMD_ENGINE_BLOCKS")) batch = (uint32_t)atoi(s);
  int slots = 3;  // combined batches in flight per engine
  if (const char* s = getenv("RCLONE_AMD_ENGINE_SLOTS")) slots = std::max(1, std::min(16, atoi(s)));
  xs_pool* p = xs_pool_create(nullptr, 0, batch, slots);
  if (!p) g_xs_pool_failed = true;
  g_xs_pool.store(p, std::memory_order_release);
  return p;
}

xs_pool* cipher_pool(const rc_cipher* c) { return c->pool ? c->pool : process_pool(); }

}  // namespace

extern "C" xs_pool* rc_default_pool(void) { return process_pool(); }

namespace {

// Pinned staging pool -- the counterpart of the reference's Cipher.buffers sync.Pool
// (cipher.go:179, :255-262): handles come and go per object, and hipHostMalloc/hipHostFree
// cost milliseconds and synchronise the device, so buffers are recycled (best fit by size, per
// NUMA node: a handle's staging sits on the node of its engine's GPU), keeping at most
// kPoolBytes cached.
constexpr size_t kPoolBytes = (size_t)1 << 30;
std::mutex g_pool_mu;
// process-lifetime cache, deliberately never destroyed: buffers stay reachable (no exit-time
// hipHostFree after the HIP runtime may already be torn down)
std::map<int, std::multimap<size_t, uint8_t*>>& g_pool = *new std::map<int, std::multimap<size_t, uint8_t*>>();
size_t g_pool_cached = 0;

// A buffer may serve a request of `bytes` when it is at least that large and not wastefully larger.
inline bool fits(size_t cap, size_t bytes) { return cap >= bytes && cap <= 2 * bytes + (1u << 20); }

// Per-thread front of the pool, as sync.Pool keeps a per-P private slot before its shared list: a
// handle's buffers released on a thread are usually asked for again by the next handle on that
// thread (a reader opening one ranged read after another), and with many threads the shared
// pool's mutex was the point where 8 or 16 concurrent ranged readers stopped scaling (round 6,
// DESIGN.md section 3e).  Bounded per thread (a handle's two or three buffers) and over all
// threads (a cgo caller may call in from many OS threads, and pinned memory is scarce); returned
// to the shared pool when the thread exits.
constexpr int kTlsEntries = 4;
constexpr size_t kTlsBytes = (size_t)16 << 20;
constexpr size_t kTlsTotalBytes = (size_t)512 << 20;
std::atomic<size_t> g_tls_cached{0};
struct TlsPool {
  struct E {
    uint8_t* p;
    size_t cap;
    int node;
  } e[kTlsEntries];
  int n = 0;
  size_t bytes = 0;
  ~TlsPool();
};
thread_local TlsPool t_pool;

// Page-locked when possible.  If pinning fails (no device, pinned-memory limit) the buffer is plain
// heap memory: a source that fails before its first block never needs the GPU, and the engine
// stages pageable buffers through its own copies.
uint8_t* pool_get(size_t bytes, size_t* cap, int node, bool* heap) {
  *heap = false;
  {  // this thread's own cache first: no lock
    TlsPool& t = t_pool;
    int best = -1;
    for (int i = 0; i < t.n; i++)
      if (t.e[i].node == node && fits(t.e[i].cap, bytes) && (best < 0 || t.e[i].cap < t.e[best].cap)) best = i;
    if (best >= 0) {
      uint8_t* p = t.e[best].p;
      *cap = t.e[best].cap;
      t.bytes -= *cap;
      g_tls_cached.fetch_sub(*cap, std::memory_order_relaxed);
      t.e[best] = t.e[--t.n];
      return p;
    }
  }
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    auto& m = g_pool[node];
    auto it = m.lower_bound(bytes);
    if (it != m.end() && fits(it->first, bytes)) {
      *cap = it->first;
      uint8_t* p = it->second;
      g_pool_cached -= it->first;
      m.erase(it);
      return p;
    }
  }
  uint8_t* p = (uint8_t*)xs_host_alloc_node(bytes, node);
  if (!p) {
    p = (uint8_t*)aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    *heap = p != nullptr;
  }
  *cap = p ? bytes : 0;
  return p;
}

void pool_put(uint8_t* p, size_t cap, int node, bool heap) {
  if (!p) return;
  if (heap) {
    free(p);
    return;
  }
  {
    TlsPool& t = t_pool;
    if (t.n < kTlsEntries && t.bytes + cap <= kTlsBytes &&
        g_tls_cached.fetch_add(cap, std::memory_order_relaxed) + cap <= kTlsTotalBytes) {
      t.e[t.n++] = {p, cap, node};
      t.bytes += cap;
      return;
    }
    if (t.n < kTlsEntries && t.bytes + cap <= kTlsBytes) g_tls_cached.fetch_sub(cap, std::memory_order_relaxed);
  }
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (g_pool_cached + cap <= kPoolBytes) {
      g_pool[node].emplace(cap, p);
      g_pool_cached += cap;
      return;
    }
  }
  xs_host_free(p);
}

// a thread's cached buffers go back to the shared pool when it exits; cached there whatever the
// cap (never freed here: at process exit the HIP runtime may be going away)
TlsPool::~TlsPool() {
  g_tls_cached.fetch_sub(bytes, std::memory_order_relaxed);
  std::lock_guard<std::mutex> g(g_pool_mu);
  for (int i = 0; i < n; i++) {
    g_pool[e[i].node].emplace(e[i].cap, e[i].p);
    g_pool_cached += e[i].cap;
  }
  n = 0;
  bytes = 0;
}

struct PinnedBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  int node = -1;      // NUMA node of p (the owner's engine's)
  bool heap = false;  // pinning failed: plain heap memory
  // at least `bytes` on node `want_node` (contents dropped)
  bool ensure(size_t bytes, int want_node = -1) {
    if (n >= bytes && node == want_node) return true;
    pool_put(p, n, node, heap);
    node = want_node;
    p = pool_get(bytes, &n, node, &heap);
    return p != nullptr;
  }
  // grow keeping the contents (doubling)
  bool ensure_keep(size_t bytes) {
    if (n >= bytes) return true;
    size_t want = n ? n : (1u << 20);
    while (want < bytes) want *= 2;
    size_t cap = 0;
    bool qheap = false;
    uint8_t* q = pool_get(want, &cap, node, &qheap);
    if (!q) return false;
    if (p) memcpy(q, p, n);
    pool_put(p, n, node, heap);
    p = q;
    n = cap;
    heap = qheap;
    return true;
  }
  void release() {
    pool_put(p, n, node, heap);
    p = nullptr;
    n = 0;
    heap = false;
  }
  ~PinnedBuf() { release(); }
};

}  // namespace

// ---------------------------------------------------------------- Cipher (struct in rc_internal.h)
extern "C" int32_t rc_cipher_key(rc_cipher* c, const char* password, const char* salt) {
  if (!c) return RC_ERR_INVALID;
  uint8_t key[80] = {0};
  if (password && password[0]) {
    const uint8_t* s = kDefaultSalt;
    size_t sl = sizeof kDefaultSalt;
    if (salt && salt[0]) {
      s = (const uint8_t*)salt;
      sl = strlen(salt);
    }
    if (!rc::scrypt((const uint8_t*)password, strlen(password), s, sl, 16384, 8, 1, key, sizeof key))
      return RC_ERR_INVALID;
  }
  memcpy(c->data_key, key, 32);
  memcpy(c->name_key, key + 32, 32);
  memcpy(c->name_tweak, key + 64, 16);
  xs::aes::expand_key(c->name_key, c->name_tweak, &c->eme);  // aes.NewCipher(c.nameKey[:]) :249
  return RC_NIL;
}

extern "C" rc_cipher* rc_cipher_new(const char* password, const char* salt, int32_t* err) {
  rc_cipher* c = new rc_cipher();
  int32_t e = rc_cipher_key(c, password, salt);
  if (err) *err = e;
  if (e != RC_NIL) {
    delete c;
    return nullptr;
  }
  return c;
}

extern "C" void rc_cipher_set_keys(rc_cipher* c, const uint8_t data_key[32], const uint8_t name_key[32],
                                   const uint8_t name_tweak[16]) {
  memcpy(c->data_key, data_key, 32);
  memcpy(c->name_key, name_key, 32);
  memcpy(c->name_tweak, name_tweak, 16);
  xs::aes::expand_key(c->name_key, c->name_tweak, &c->eme);
}

extern "C" void rc_cipher_keys(const rc_cipher* c, uint8_t data_key[32], uint8_t name_key[32], uint8_t name_tweak[16]) {
  if (data_key) memcpy(data_key, c->data_key, 32);
  if (name_key) memcpy(name_key, c->name_key, 32);
  if (name_tweak) memcpy(name_tweak, c->name_tweak, 16);
}

extern "C" void rc_cipher_set_pass_bad_blocks(rc_cipher* c, int32_t pass) { c->pass_bad_blocks = pass != 0; }
extern "C" void rc_cipher_set_rand(rc_cipher* c, rc_reader rand) { c->rand = rand; }
extern "C" void rc_cipher_set_batch_blocks(rc_cipher* c, uint32_t blocks) { c->batch_blocks = blocks ? blocks : 1; }
extern "C" void rc_cipher_set_readahead(rc_cipher* c, uint32_t first_blocks) { c->first_blocks = first_blocks; }
extern "C" void rc_cipher_set_readahead_growth(rc_cipher* c, uint32_t factor) { c->growth = factor == 1 ? 2 : factor; }
extern "C" void rc_cipher_set_pool(rc_cipher* c, xs_pool* pool) { c->pool = pool; }
extern "C" void rc_cipher_free(rc_cipher* c) { delete c; }

// ---------------------------------------------------------------- sizes, nonce arithmetic
extern "C" int64_t rc_encrypted_size(int64_t size) {
  int64_t blocks = size / kBlockData, residue = size % kBlockData;
  int64_t e = kFileHdr + blocks * kBlockSize;
  if (residue != 0) e += kBlockHdr + residue;
  return e;
}

extern "C" int64_t rc_decrypted_size(int64_t size, int32_t* err) {
  if (err) *err = RC_NIL;
  size -= kFileHdr;
  if (size < 0) {
    if (err) *err = RC_ERR_FILE_TOO_SHORT;
    return 0;
  }
  int64_t blocks = size / kBlockSize, residue = size % kBlockSize;
  int64_t d = blocks * kBlockData;
  if (residue != 0) {
    residue -= kBlockHdr;
    if (residue <= 0) {
      if (err) *err = RC_ERR_FILE_BAD_HEADER;
      return 0;
    }
  }
  return d + residue;
}

extern "C" void rc_calculate_underlying(int64_t offset, int64_t limit, int64_t out[4]) {
  int64_t blocks = offset / kBlockData, discard = offset % kBlockData;
  int64_t uoff = kFileHdr + blocks * kBlockSize;
  int64_t ulim = -1;
  if (limit >= 0) {
    int64_t bytes_to_read = limit - (kBlockData - discard);
    int64_t blocks_to_read = 1;
    if (bytes_to_read > 0) {
      int64_t extra = bytes_to_read / kBlockData, end = bytes_to_read % kBlockData;
      if (end != 0) extra++;
      blocks_to_read += extra;
    }
    ulim = blocks_to_read * kBlockSize;
  }
  out[0] = uoff;
  out[1] = ulim;
  out[2] = discard;
  out[3] = blocks;
}

static void nonce_carry(uint8_t n[24], int i) {
  for (; i < 24; i++) {
    uint8_t digit = n[i];
    uint8_t nd = (uint8_t)(digit + 1);
    n[i] = nd;
    if (nd >= digit) break;
  }
}
extern "C" void rc_nonce_increment(uint8_t n[24]) { nonce_carry(n, 0); }
extern "C" void rc_nonce_add(uint8_t n[24], uint64_t x) {
  uint16_t carry = 0;
  for (int i = 0; i < 8; i++) {
    uint8_t digit = n[i];
    uint8_t xd = (uint8_t)x;
    x >>= 8;
    carry = (uint16_t)(carry + digit + xd);
    n[i] = (uint8_t)carry;
    carry >>= 8;
  }
  if (carry != 0) nonce_carry(n, 8);
}

extern "C" const char* rc_error_string(int32_t e) {
  switch (e) {
    case RC_NIL: return "";
    case RC_EOF: return "EOF";
    case RC_UNEXPECTED_EOF: return "unexpected EOF";
    case RC_ERR_FILE_TOO_SHORT: return "file is too short to be encrypted";
    case RC_ERR_FILE_BAD_HEADER: return "file has truncated block header";
    case RC_ERR_BAD_MAGIC: return "not an encrypted file - bad magic string";
    case RC_ERR_BAD_BLOCK: return "failed to authenticate decrypted block - bad password?";
    case RC_ERR_FILE_CLOSED: return "file already closed";
    case RC_ERR_BAD_SEEK: return "Seek beyond end of file";
    case RC_ERR_SHORT_NONCE: return "short read of nonce";
    case RC_ERR_SEEK_NOT_INIT: return "can't seek - not initialised with newDecrypterSeek";
    case RC_ERR_SEEK_WHENCE: return "can only seek from the start";
    case RC_ERR_REOPEN: return "couldn't reopen file with offset and limit";
    case RC_ERR_GPU: return "GPU crypt engine failure";
    case RC_ERR_INVALID: return "invalid argument";
    case RC_ERR_NOT_A_MULTIPLE_OF_BLOCKSIZE: return "not a multiple of blocksize";
    case RC_ERR_TOO_SHORT_AFTER_DECODE: return "too short after base32 decode";
    case RC_ERR_TOO_LONG_AFTER_DECODE: return "too long after base32 decode";
    case RC_ERR_BAD_BASE32_ENCODING: return "bad base32 filename encoding";
    case RC_ERR_NOT_AN_ENCRYPTED_FILE: return "not an encrypted file - does not match suffix";
    case RC_ERR_PKCS7_NOT_FOUND: return "bad PKCS#7 padding - not padded";
    case RC_ERR_PKCS7_NOT_A_MULTIPLE: return "bad PKCS#7 padding - not a multiple of blocksize";
    case RC_ERR_PKCS7_TOO_LONG: return "bad PKCS#7 padding - too long";
    case RC_ERR_PKCS7_TOO_SHORT: return "bad PKCS#7 padding - too short";
    case RC_ERR_PKCS7_NOT_ALL_THE_SAME: return "bad PKCS#7 padding - not all the same";
    case RC_ERR_BASE32_CORRUPT: return "illegal base32 data at input byte";
    case RC_ERR_BASE64_CORRUPT: return "illegal base64 data at input byte";
    case RC_ERR_BASE32768_CORRUPT: return "illegal base32768 data at input byte";
    case RC_ERR_UNKNOWN_MODE: return "unknown file name encryption mode";
    case RC_ERR_UNKNOWN_ENCODING: return "unknown file name encoding mode";
    case RC_ERR_NAME_TOO_LONG: return "EME operates on 1 to 128 block-cipher blocks";
    default: return "reader error";
  }
}

// ---------------------------------------------------------------- phase times (diagnostic)
// RCLONE_AMD_PHASES=1: where the streaming refills and per-object hashes spend their time,
// summed over threads and printed to stderr at exit (source reads, GPU seals, MD5 waits / inline
// MD5, consumer-side copies are the rest).  Off: one predictable branch per refill.
namespace {
enum Phase { kEncRead, kEncSeal, kEncWait, kEncInline, kEncRefills, kHashRead, kHashSeal, kHashWait, kHashInline,
             kHashCalls, kHashFinal, kNPhase };
std::atomic<uint64_t> g_phase[kNPhase];
bool phases_on() {
  static const bool on = [] {
    const char* v = getenv("RCLONE_AMD_PHASES");
    if (!v || atoi(v) == 0) return false;
    atexit([] {
      static const char* names[kNPhase] = {"enc_read", "enc_seal", "enc_md5_wait", "enc_md5_inline", "enc_refills",
                                           "hash_read", "hash_seal", "hash_md5_wait", "hash_md5_inline", "hash_calls",
                                           "hash_final_wait"};
      fprintf(stderr, "{\"rclone_amd_phases\": {");
      for (int i = 0; i < kNPhase; i++) {
        const bool count = i == kEncRefills || i == kHashCalls;
        fprintf(stderr, "%s\"%s%s\": %.4f", i ? ", " : "", names[i], count ? "" : "_s",
                count ? (double)g_phase[i].load() : g_phase[i].load() * 1e-9);
      }
      auto& t = xs::md5_tier_stats();
      const double ws = t.worker_ns.load() * 1e-9;
      fprintf(stderr,
              ", \"md5_jobs_worker\": %llu, \"md5_jobs_inline\": %llu, \"md5_jobs_lanes\": %llu, "
              "\"md5_worker_s\": %.4f, \"md5_worker_GB_s\": %.3f}}\n",
              (unsigned long long)t.worker.load(), (unsigned long long)t.inline_.load(),
              (unsigned long long)t.lanes.load(), ws, ws > 0 ? t.worker_bytes.load() / ws * 1e-9 : 0.0);
    });
    return true;
  }();
  return on;
}
struct PhaseClock {  // adds the time since the last mark to a phase
  bool on = phases_on();
  std::chrono::steady_clock::time_point t = on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  void mark(Phase p) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    g_phase[p].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count(),
                         std::memory_order_relaxed);
    t = n;
  }
  void count(Phase p) {
    if (on) g_phase[p].fetch_add(1, std::memory_order_relaxed);
  }
};
}  // namespace

// ---------------------------------------------------------------- encrypter
// Read-ahead: the first refill of a stream (and the first after a seek) reads exactly one block,
// as encrypter.Read / fillBuffer do (cipher.go:726-741, :862-898), so a slow or streaming source
// sees the reference's first-byte behaviour.  Later refills grow up to the cipher's batch_blocks:
// by the cipher's growth factor, or (growth 0, the default) by doubling while the source is slow
// and straight to full batches once a refill shows a fast source (memory, page cache: > 2 GB/s),
// where every extra GPU round trip would only cost throughput.
constexpr double kFastSourceBps = 2e9;

static uint32_t next_batch(const rc_cipher* c, uint32_t grow) {
  const uint32_t cap = c->batch_blocks;
  if (grow == 0) grow = c->first_blocks ? c->first_blocks : cap;  // first_blocks 0: full batches at once
  return std::min(grow, cap);
}

static uint32_t grow_batch(const rc_cipher* c, uint32_t used, int64_t bytes, std::chrono::steady_clock::duration t) {
  const uint64_t cap = c->batch_blocks;
  uint64_t next = (uint64_t)used * (c->growth ? c->growth : 2);
  if (c->growth == 0 && bytes > 0 && std::chrono::duration<double>(t).count() * kFastSourceBps < (double)bytes)
    next = cap;
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(next, 1), cap);
}

struct rc_encrypter {
  std::mutex mu;
  rc_reader in{};
  rc_cipher* c = nullptr;
  xs_engine* eng = nullptr;  // taken from the cipher's pool at the first refill
  uint8_t nonce[24] = {0};  // fh.nonce: initial nonce + blocks sealed
  uint8_t hdr[kFileHdr];    // magic || initial nonce, served before the first block
  bool in_hdr = true;
  PinnedBuf plain, wire;    // staging (fh.readBuf / fh.buf), allocated at the first refill
  uint32_t grow = 0;        // read-ahead blocks of the next refill (next_batch)
  int64_t buf_index = 0, buf_size = 0;
  int32_t err = RC_NIL;
  bool finished = false;
  // crypt.put's tee hash (crypt.go:516-533) taken by the encrypter itself (rc_encrypter_set_md5):
  // a worker hashes batch k while the consumer reads it and the next refill seals batch k+1 into
  // the other wire buffer.  md5 covers every byte produced once `job` is done; md5_cur is the
  // state before the batch being served (for a consumer that stops inside a batch).
  bool md5_on = false;
  bool md5_counted = false;  // in g_md5_streams
  bool wsel = false;  // md5_on: the batch being served is in wire2 (else wire)
  PinnedBuf wire2;
  xs::HostMd5 md5, md5_cur;
  xs::Md5Job job;
};

// the bytes the encrypter is serving now: the header, then the current wire batch
static const uint8_t* enc_cur(const rc_encrypter* fh) {
  return fh->in_hdr ? fh->hdr : (fh->md5_on && fh->wsel ? fh->wire2.p : fh->wire.p);
}

// Per-object hashing (the tee and computeHashWithNonce) hashes batch k on a worker while the stream
// reads and seals batch k+1.  MD5 is the slowest stage (one chain, ~1 GB/s against several GB/s of
// reads and seals), so what a stream loses is the time before its chain starts and any gap in it.
// With the ramp a stream's seals double from one block -- the chain starts after one block's read
// and seal, not a whole batch's, and each next batch is read and sealed while the previous, half
// as large, is hashed -- and every batch from one full block up goes to a worker.  The ramp costs
// more GPU calls and hand-offs, which pay only while each stream has a core to spare for its
// worker: it is on while the per-object streams hashing now are at most half the process's CPU
// budget (the reference defaults, --transfers 4 / --checkers 8, on 16 cores), else a stream uses
// full batches and a 256 KiB inline threshold as before.  RCLONE_AMD_MD5_RAMP=0 turns it off.
static std::atomic<int> g_md5_streams{0};  // tee encrypters until they finish + hash calls running

static bool md5_ramp_now() {
  static const bool on = [] {
    const char* e = getenv("RCLONE_AMD_MD5_RAMP");
    return !e || atoi(e) != 0;
  }();
  static const int cpus = std::max(1, xs::effective_cpus());
  return on && 2 * g_md5_streams.load(std::memory_order_relaxed) <= cpus;
}

// Batches below this are hashed on the stream's own thread (a worker hand-off costs ~10 us).
static int64_t inline_md5_below(bool ramping) {
  static const int64_t env = [] {
    const char* e = getenv("RCLONE_AMD_MD5_INLINE");
    return e ? (int64_t)std::max(0, atoi(e)) : (int64_t)-1;
  }();
  if (env >= 0) return env;
  return ramping ? (int64_t)kBlockData : (int64_t)(256 << 10);
}

static void md5_stream_count(bool& counted, bool on) {
  if (on == counted) return;
  counted = on;
  g_md5_streams.fetch_add(on ? 1 : -1, std::memory_order_relaxed);
}

// finish (cipher.go:748-758)
static int64_t enc_finish(rc_encrypter* fh, int32_t err, int32_t* out_err) {
  if (fh->finished) {
    *out_err = fh->err;
    return 0;
  }
  fh->finished = true;
  fh->err = err;
  md5_stream_count(fh->md5_counted, false);
  xs::md5_wait(&fh->job);  // the worker may still be reading a wire buffer
  fh->plain.release();
  fh->wire.release();
  fh->wire2.release();
  *out_err = err;
  return 0;
}

extern "C" rc_encrypter* rc_encrypt_data(rc_cipher* c, rc_reader in, const uint8_t* nonce, int32_t* err) {
  if (err) *err = RC_NIL;
  if (!c || !in.read) {
    if (err) *err = RC_ERR_INVALID;
    return nullptr;
  }
  rc_encrypter* fh = new rc_encrypter();
  fh->in = in;
  fh->c = c;
  if (nonce) {
    memcpy(fh->nonce, nonce, 24);
  } else {
    // nonce.fromReader(c.cryptoRand) (cipher.go:630-636)
    int32_t e = RC_NIL;
    int64_t got = 0;
    if (c->rand.read) {
      std::lock_guard<std::mutex> g(c->rand_mu);
      got = read_fill(c->rand, fh->nonce, 24, &e);
    } else {
      got = getrandom(fh->nonce, 24, 0);
      e = got == 24 ? RC_NIL : RC_UNEXPECTED_EOF;
    }
    if (got != 24) {
      if (err) *err = RC_ERR_SHORT_NONCE;
      delete fh;
      return nullptr;
    }
  }
  memcpy(fh->hdr, kMagic, 8);
  memcpy(fh->hdr + 8, fh->nonce, 24);
  fh->buf_size = kFileHdr;
  return fh;
}

extern "C" int64_t rc_encrypter_read(rc_encrypter* fh, uint8_t* p, int64_t n, int32_t* err) {
  std::lock_guard<std::mutex> g(fh->mu);
  *err = RC_NIL;
  if (fh->finished) {
    *err = fh->err;
    return 0;
  }
  if (fh->buf_index >= fh->buf_size) {
    // refill: ReadFill block by block exactly as encrypter.Read would, up to next_batch blocks
    fh->in_hdr = false;
    const uint32_t batch = next_batch(fh->c, fh->grow);
    if (!fh->eng) fh->eng = xs_pool_next(cipher_pool(fh->c));  // staging goes on its GPU's node
    if (!fh->eng) return enc_finish(fh, RC_ERR_GPU, err);
    const int node = xs_engine_numa_node(fh->eng);
    if (!fh->plain.ensure((size_t)fh->c->batch_blocks * kBlockData, node) ||
        !fh->wire.ensure((size_t)fh->c->batch_blocks * kBlockSize, node) ||
        (fh->md5_on && !fh->wire2.ensure((size_t)fh->c->batch_blocks * kBlockSize, node)))
      return enc_finish(fh, RC_ERR_GPU, err);
    const auto t0 = std::chrono::steady_clock::now();
    PhaseClock pc;
    pc.count(kEncRefills);
    int64_t total = 0;
    uint32_t nb = 0;
    int32_t first_err = RC_NIL;
    for (; nb < batch; nb++) {
      int32_t e = RC_NIL;
      int64_t got = read_fill(fh->in, fh->plain.p + (int64_t)nb * kBlockData, kBlockData, &e);
      if (got == 0) {
        if (nb == 0) first_err = e;
        break;
      }
      total += got;
      if (got < kBlockData || e != RC_NIL) {  // the next ReadFill must be a fresh call
        nb++;
        break;
      }
    }
    if (nb == 0) return enc_finish(fh, first_err, err);
    fh->grow = grow_batch(fh->c, batch, total, std::chrono::steady_clock::now() - t0);
    const bool ramp = fh->md5_on && md5_ramp_now();
    if (ramp && fh->c->growth == 0)  // keep the tee's chain fed: double, no jump to full batches
      fh->grow = std::min<uint32_t>(2 * batch, fh->c->batch_blocks);
    // with the tee hash on, seal into the wire buffer that is neither served nor being hashed
    const bool into2 = fh->md5_on && !fh->wsel;
    uint8_t* out = into2 ? fh->wire2.p : fh->wire.p;
    pc.mark(kEncRead);
    if (xs_engine_seal(fh->eng, fh->c->data_key, fh->nonce, 0, fh->plain.p, (uint64_t)total, out) != XS_OK)
      return enc_finish(fh, RC_ERR_GPU, err);
    pc.mark(kEncSeal);
    fh->buf_index = 0;
    fh->buf_size = total + (int64_t)nb * kBlockHdr;
    rc_nonce_add(fh->nonce, nb);  // nonce.increment() once per sealed block
    if (fh->md5_on) {
      auto& w = xs::md5_workers(node);
      w.wait(&fh->job);  // the previous batch is hashed: md5 covers everything served so far
      pc.mark(kEncWait);
      fh->md5_cur = fh->md5;
      fh->wsel = into2;
      fh->job.st = &fh->md5;
      fh->job.p = out;
      fh->job.n = (size_t)fh->buf_size;
      if (fh->buf_size < inline_md5_below(ramp)) fh->md5.update(out, (size_t)fh->buf_size);
      else w.submit(&fh->job);
      pc.mark(kEncInline);
    }
  }
  int64_t m = fh->buf_size - fh->buf_index;
  if (m > n) m = n;
  memcpy(p, enc_cur(fh) + fh->buf_index, (size_t)m);
  fh->buf_index += m;
  return m;
}

extern "C" void rc_encrypter_nonce(const rc_encrypter* fh, uint8_t out[24]) { memcpy(out, fh->nonce, 24); }

extern "C" int32_t rc_encrypter_set_md5(rc_encrypter* fh, int32_t on) {
  if (!fh) return RC_ERR_INVALID;
  std::lock_guard<std::mutex> g(fh->mu);
  if (!fh->in_hdr || fh->buf_index != 0 || fh->finished) return RC_ERR_INVALID;  // before the first Read only
  fh->md5_on = on != 0;
  md5_stream_count(fh->md5_counted, fh->md5_on);
  fh->md5 = xs::HostMd5();
  fh->md5_cur = fh->md5;
  if (fh->md5_on) fh->md5.update(fh->hdr, kFileHdr);  // the header is the first "batch" served
  return RC_NIL;
}

extern "C" int32_t rc_encrypter_md5(rc_encrypter* fh, uint8_t out[16]) {
  if (!fh || !out) return RC_ERR_INVALID;
  std::lock_guard<std::mutex> g(fh->mu);
  if (!fh->md5_on) return RC_ERR_INVALID;
  xs::md5_wait(&fh->job);
  // MD5 of exactly the bytes returned so far, like the TeeReader: all produced bytes when the
  // current batch is used up (always so after EOF), else the state before it plus its served part
  xs::HostMd5 h = fh->md5;
  if (fh->buf_index < fh->buf_size && !fh->finished) {
    h = fh->md5_cur;
    h.update(enc_cur(fh), (size_t)fh->buf_index);
  }
  h.final(out);
  return RC_NIL;
}

extern "C" void rc_encrypter_free(rc_encrypter* fh) {
  if (!fh) return;
  md5_stream_count(fh->md5_counted, false);
  xs::md5_wait(&fh->job);
  delete fh;
}

// ---------------------------------------------------------------- decrypter
struct rc_decrypter {
  std::mutex mu;
  rc_reader rc{};
  bool have_rc = false;
  uint8_t nonce[24] = {0};
  uint8_t initial_nonce[24] = {0};
  rc_cipher* c = nullptr;
  xs_engine* eng = nullptr;  // taken from the cipher's pool at the first refill
  uint32_t grow = 0;         // read-ahead blocks of the next refill (next_batch); 0 after open/seek
  PinnedBuf wire, plain, okb;
  // decoded batch: blocks [cur, nblk) still to serve; block i has payload length blen[i]
  std::vector<int64_t> blen;
  std::vector<int32_t> berr;  // error returned by the ReadFill that produced block i
  size_t cur = 0, nblk = 0;
  int32_t tail_err = RC_NIL;  // what fillBuffer returns after the decoded blocks (RC_NIL = read more)
  bool have_tail = false;
  int64_t buf_index = 0, buf_size = 0;  // within the current block
  int64_t cur_off = 0;                  // plaintext offset of the current block in plain
  int32_t err = RC_NIL;
  bool finished = false;
  int64_t limit = -1;
  // plaintext offset, from the next batch's start, of the first byte a Read can reach: the
  // discard of the RangeSeek that fills that batch (bytes before it are never served)
  int64_t win_lo = 0;
  rc_open_fn open = nullptr;
  void* open_user = nullptr;
  int32_t wrapped = RC_NIL;
};

// staging for the `blocks` blocks this refill reads (a limited handle -- a ranged read -- needs one
// or two, not a whole read-ahead batch; grown when a later refill reads more), allocated when the
// first block is read (not at open: a header error or a failing source never needs it)
static bool dec_alloc(rc_decrypter* fh, uint32_t blocks) {
  if (!fh->eng) fh->eng = xs_pool_next(cipher_pool(fh->c));  // staging goes on its GPU's node
  if (!fh->eng) return false;
  const int node = xs_engine_numa_node(fh->eng);
  return fh->wire.ensure((size_t)blocks * kBlockSize, node) && fh->plain.ensure((size_t)blocks * kBlockData, node) &&
         fh->okb.ensure(blocks, node);
}

// finish (cipher.go:1042-1052): sets the sticky error and returns it
static int32_t dec_finish(rc_decrypter* fh, int32_t err) {
  if (fh->finished) return fh->err;
  fh->finished = true;
  fh->err = err;
  fh->wire.release();
  fh->plain.release();
  fh->okb.release();
  fh->nblk = fh->cur = 0;
  fh->have_tail = false;
  return err;
}

// unFinish (cipher.go:1054-1066)
static void dec_unfinish(rc_decrypter* fh) {
  fh->finished = false;
  fh->err = RC_NIL;
  fh->buf_index = fh->buf_size = 0;
  fh->nblk = fh->cur = 0;
  fh->have_tail = false;
}

static int32_t dec_close_locked(rc_decrypter* fh) {
  if (fh->finished && fh->err == RC_ERR_FILE_CLOSED) return RC_ERR_FILE_CLOSED;
  if (!fh->finished) dec_finish(fh, RC_EOF);
  fh->err = RC_ERR_FILE_CLOSED;
  if (!fh->have_rc) return RC_NIL;
  return fh->rc.close ? fh->rc.close(fh->rc.user) : RC_NIL;
}

// Read up to `want` blocks with the reference's per-block ReadFill sequence and open them on
// the GPU.  Errors are not returned here; they are queued at the block position where
// fillBuffer (cipher.go:862-898) would return them.
static int32_t dec_read_batch(rc_decrypter* fh, uint32_t want) {
  const uint32_t ra = next_batch(fh->c, fh->grow);
  if (want == 0 || want > ra) want = ra;
  if (!dec_alloc(fh, want)) return RC_ERR_GPU;
  const auto t0 = std::chrono::steady_clock::now();
  fh->blen.assign(want, 0);
  fh->berr.assign(want, RC_NIL);
  fh->nblk = fh->cur = 0;
  fh->have_tail = false;
  int64_t total = 0;
  uint32_t nb = 0;
  for (; nb < want; nb++) {
    int32_t e = RC_NIL;
    int64_t got = read_fill(fh->rc, fh->wire.p + (int64_t)nb * kBlockSize, kBlockSize, &e);
    if (got == 0) {
      fh->have_tail = true;
      fh->tail_err = e;
      break;
    }
    if (got <= kBlockHdr) {  // "Check header + 1 byte exists"
      fh->have_tail = true;
      fh->tail_err = is_pending(e) ? e : RC_ERR_FILE_BAD_HEADER;
      break;
    }
    fh->blen[nb] = got - kBlockHdr;
    fh->berr[nb] = e;
    total += got;
    if (got < kBlockSize || e != RC_NIL) {
      nb++;
      break;
    }
  }
  fh->nblk = nb;
  if (nb == 0) return RC_NIL;
  fh->grow = grow_batch(fh->c, ra, total, std::chrono::steady_clock::now() - t0);
  // Reads reach plaintext bytes [win_lo, limit) of this batch at most (limit counts from the batch
  // start here, see range_seek_locked): the GPU may skip decrypting the rest of a block, every tag
  // is still verified whole (a ranged 4 KiB read decrypts one or two 4 KiB groups of its block)
  const uint64_t lo = (uint64_t)fh->win_lo, hi = fh->limit >= 0 ? (uint64_t)fh->limit : UINT64_MAX;
  fh->win_lo = 0;
  if (xs_engine_open_range(fh->eng, fh->c->data_key, fh->nonce, 0, fh->wire.p, (uint64_t)total, fh->plain.p,
                           fh->okb.p, lo, hi) != XS_OK) {
    fh->nblk = 0;
    return RC_ERR_GPU;
  }
  return RC_NIL;
}

// fillBuffer (cipher.go:862-898): make the next block current.  Returns RC_NIL or the error
// the reference returns at this position.
static int32_t dec_fill(rc_decrypter* fh) {
  if (fh->cur >= fh->nblk) {
    if (fh->have_tail) {
      fh->have_tail = false;
      return fh->tail_err;
    }
    uint32_t want = 0;
    if (fh->limit >= 0) want = (uint32_t)((fh->limit + kBlockData - 1) / kBlockData);
    int32_t e = dec_read_batch(fh, want);  // want == 0: a full batch
    if (e != RC_NIL) return e;
    if (fh->nblk == 0) {
      fh->have_tail = false;
      return fh->tail_err;
    }
  }
  const size_t i = fh->cur;
  if (!fh->okb.p[i]) {
    if (is_pending(fh->berr[i])) return fh->berr[i];  // pending error is likely more accurate
    if (!fh->c->pass_bad_blocks) return RC_ERR_BAD_BLOCK;
    // pass_bad_blocks: the kernel already zero-filled the block ("crypt: ignoring: ...")
  }
  fh->cur_off = (int64_t)i * kBlockData;
  fh->buf_index = 0;
  fh->buf_size = fh->blen[i];
  fh->cur++;
  rc_nonce_increment(fh->nonce);
  return RC_NIL;
}

static rc_decrypter* new_decrypter(rc_cipher* c, rc_reader rc, int32_t* err) {
  rc_decrypter* fh = new rc_decrypter();
  fh->rc = rc;
  fh->have_rc = true;
  fh->c = c;
  uint8_t hdr[kFileHdr];
  int32_t e = RC_NIL;
  int64_t n = read_fill(fh->rc, hdr, kFileHdr, &e);
  int32_t fail = RC_NIL;
  if (n < kFileHdr && e == RC_EOF) fail = RC_ERR_FILE_TOO_SHORT;
  else if (e != RC_EOF && e != RC_NIL) fail = e;
  else if (memcmp(hdr, kMagic, 8) != 0) fail = RC_ERR_BAD_MAGIC;
  if (fail != RC_NIL) {
    // finishAndClose (cipher.go:1089-1095)
    dec_finish(fh, fail);
    dec_close_locked(fh);
    delete fh;
    *err = fail;
    return nullptr;
  }
  memcpy(fh->nonce, hdr + 8, 24);
  memcpy(fh->initial_nonce, hdr + 8, 24);
  *err = RC_NIL;
  return fh;
}

extern "C" rc_decrypter* rc_decrypt_data(rc_cipher* c, rc_reader rc, int32_t* err) {
  int32_t e = RC_NIL;
  if (!c || !rc.read) {
    if (err) *err = RC_ERR_INVALID;
    return nullptr;
  }
  rc_decrypter* fh = new_decrypter(c, rc, &e);
  if (err) *err = e;
  return fh;
}

static int64_t range_seek_locked(rc_decrypter* fh, int64_t offset, int32_t whence, int64_t limit, int32_t* err);

extern "C" rc_decrypter* rc_decrypt_data_seek(rc_cipher* c, rc_open_fn open, void* open_user, int64_t offset,
                                              int64_t limit, int32_t* err) {
  return rc_decrypt_data_seek_ex(c, open, open_user, offset, limit, err, nullptr);
}

extern "C" rc_decrypter* rc_decrypt_data_seek_ex(rc_cipher* c, rc_open_fn open, void* open_user, int64_t offset,
                                                 int64_t limit, int32_t* err, int32_t* wrapped) {
  if (wrapped) *wrapped = RC_NIL;
  if (!c || !open) {
    if (err) *err = RC_ERR_INVALID;
    return nullptr;
  }
  rc_reader rc{};
  bool do_range_seek = false, set_limit = false;
  int32_t e;
  if (offset == 0 && limit < 0) {
    e = open(open_user, 0, -1, &rc);
  } else if (offset == 0) {
    int64_t u[4];
    rc_calculate_underlying(offset, limit, u);
    e = open(open_user, 0, kFileHdr + u[1], &rc);
    set_limit = true;
  } else {
    e = open(open_user, 0, kFileHdr, &rc);
    do_range_seek = true;
  }
  if (e != RC_NIL) {
    if (err) *err = e;
    return nullptr;
  }
  rc_decrypter* fh = new_decrypter(c, rc, &e);
  if (!fh) {
    if (err) *err = e;
    return nullptr;
  }
  fh->open = open;
  fh->open_user = open_user;
  if (do_range_seek) {  // the handle is not shared yet: no lock needed
    int32_t se = RC_NIL;
    range_seek_locked(fh, offset, 0, limit, &se);
    if (se != RC_NIL) {
      // the %w operand of "couldn't reopen file with offset and limit: %w" (cipher.go:1011)
      if (wrapped && (se == RC_ERR_REOPEN || se == RC_ERR_SHORT_NONCE)) *wrapped = fh->wrapped;
      dec_close_locked(fh);  // fh.Close()
      delete fh;
      if (err) *err = se;
      return nullptr;
    }
  }
  if (set_limit) fh->limit = limit;
  if (err) *err = RC_NIL;
  return fh;
}

extern "C" int64_t rc_decrypter_read(rc_decrypter* fh, uint8_t* p, int64_t n, int32_t* err) {
  std::lock_guard<std::mutex> g(fh->mu);
  *err = RC_NIL;
  if (fh->finished) {
    *err = fh->err;
    return 0;
  }
  if (fh->buf_index >= fh->buf_size) {
    int32_t e = dec_fill(fh);
    if (e != RC_NIL) {
      *err = dec_finish(fh, e);
      return 0;
    }
  }
  int64_t to_copy = fh->buf_size - fh->buf_index;
  if (fh->limit >= 0 && fh->limit < to_copy) to_copy = fh->limit;
  if (to_copy > n) to_copy = n;
  memcpy(p, fh->plain.p + fh->cur_off + fh->buf_index, (size_t)to_copy);
  fh->buf_index += to_copy;
  if (fh->limit >= 0) {
    fh->limit -= to_copy;
    if (fh->limit == 0) {
      *err = dec_finish(fh, RC_EOF);
      return to_copy;
    }
  }
  return to_copy;
}

// RangeSeek (cipher.go:972-1034)
static int64_t range_seek_locked(rc_decrypter* fh, int64_t offset, int32_t whence, int64_t limit, int32_t* err) {
  *err = RC_NIL;
  if (!fh->open) {
    *err = dec_finish(fh, RC_ERR_SEEK_NOT_INIT);
    return 0;
  }
  if (whence != 0) {
    *err = dec_finish(fh, RC_ERR_SEEK_WHENCE);
    return 0;
  }
  if (fh->finished && fh->err == RC_EOF) {
    dec_unfinish(fh);
  } else if (fh->finished) {
    *err = fh->err;
    return 0;
  }
  int64_t u[4];
  rc_calculate_underlying(offset, limit, u);
  const int64_t uoff = u[0], ulim = u[1], discard = u[2], blocks = u[3];
  memcpy(fh->nonce, fh->initial_nonce, 24);
  rc_nonce_add(fh->nonce, (uint64_t)blocks);
  // drop read-ahead; the first refill after the seek reads one block again
  fh->nblk = fh->cur = 0;
  fh->have_tail = false;
  fh->buf_index = fh->buf_size = 0;
  fh->grow = 0;
  if (fh->have_rc && fh->rc.range_seek) {
    int32_t e = fh->rc.range_seek(fh->rc.user, uoff, 0, ulim);
    if (e != RC_NIL) {
      *err = dec_finish(fh, e);
      return 0;
    }
  } else {
    if (fh->have_rc && fh->rc.close) (void)fh->rc.close(fh->rc.user);
    fh->have_rc = false;
    rc_reader nrc{};
    int32_t e = fh->open(fh->open_user, uoff, ulim, &nrc);
    if (e != RC_NIL) {
      fh->wrapped = e;
      *err = dec_finish(fh, RC_ERR_REOPEN);
      return 0;
    }
    fh->rc = nrc;
    fh->have_rc = true;
  }
  // fillBuffer for the first block; read ahead only what (discard + limit) needs, and decrypt only
  // what Reads from discard on can reach
  fh->limit = (limit >= 0) ? discard + limit : -1;
  fh->win_lo = discard;
  int32_t e = dec_fill(fh);
  fh->win_lo = 0;
  if (e != RC_NIL) {
    *err = dec_finish(fh, e);
    return 0;
  }
  if (discard > fh->buf_size) {
    *err = dec_finish(fh, RC_ERR_BAD_SEEK);
    return 0;
  }
  fh->buf_index = discard;
  fh->limit = limit;
  return offset;
}

extern "C" int64_t rc_decrypter_range_seek(rc_decrypter* fh, int64_t offset, int32_t whence, int64_t limit,
                                           int32_t* err) {
  std::lock_guard<std::mutex> g(fh->mu);
  return range_seek_locked(fh, offset, whence, limit, err);
}

extern "C" int32_t rc_decrypter_close(rc_decrypter* fh) {
  std::lock_guard<std::mutex> g(fh->mu);
  return dec_close_locked(fh);
}

extern "C" void rc_decrypter_nonce(const rc_decrypter* fh, uint8_t out[24]) { memcpy(out, fh->nonce, 24); }
extern "C" int32_t rc_decrypter_wrapped_error(const rc_decrypter* fh) { return fh->wrapped; }
extern "C" void rc_decrypter_free(rc_decrypter* fh) { delete fh; }

// ---------------------------------------------------------------- computeHashWithNonce, batched
extern "C" int32_t rc_hash_batch_with_nonce(rc_cipher* c, uint64_t n, const rc_reader* srcs, const uint8_t* nonces,
                                            uint8_t* md5, int32_t* errs) {
  if (n == 0) return RC_NIL;
  if (!c || !srcs || !nonces || !md5 || !errs) return RC_ERR_INVALID;
  PinnedBuf buf;
  uint64_t pos = 0;
  std::vector<uint64_t> offs, lens;
  std::vector<uint8_t> ns;
  std::vector<uint64_t> idx;  // objects that read cleanly
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t start = (pos + 15) & ~15ull;
    pos = start;
    int32_t err = RC_NIL;
    for (;;) {
      if (!buf.ensure_keep(pos + kBlockData)) return RC_ERR_GPU;
      int64_t got = read_fill(srcs[i], buf.p + pos, kBlockData, &err);
      pos += (uint64_t)got;
      if (err != RC_NIL) break;
    }
    if (err == RC_EOF) err = RC_NIL;  // io.Copy: EOF is success
    if (srcs[i].close) {              // defer fs.CheckClose(in, &err)
      int32_t ce = srcs[i].close(srcs[i].user);
      if (err == RC_NIL && ce != RC_NIL) err = ce;
    }
    errs[i] = err;
    if (err != RC_NIL) {
      pos = start;  // drop the partial object
      continue;
    }
    offs.push_back(start);
    lens.push_back(pos - start);
    ns.insert(ns.end(), nonces + 24 * i, nonces + 24 * i + 24);
    idx.push_back(i);
  }
  if (idx.empty()) return RC_NIL;  // every source failed: nothing for the GPU
  xs_pool* pool = cipher_pool(c);
  if (!pool) return RC_ERR_GPU;
  std::vector<uint8_t> dig(16 * idx.size());
  if (xs_pool_seal_md5(pool, c->data_key, idx.size(), ns.data(), offs.data(), lens.data(), buf.p, dig.data()) != XS_OK)
    return RC_ERR_GPU;
  for (size_t k = 0; k < idx.size(); k++) memcpy(md5 + 16 * idx[k], dig.data() + 16 * k, 16);
  return RC_NIL;
}

// ---------------------------------------------------------------- computeHashWithNonce, one object
// computeHashWithNonce (crypt.go:784-806) as an unchanged caller runs it: one object per call, from
// cryptcheck's --checkers goroutines (cmd/cryptcheck/cryptcheck.go:91-114) or bisync's check.  The
// object is read in ReadFills of one block, as newEncrypter would, up to hash_batch_blocks() blocks
// per GPU seal, ramping 1, 2, 4, ... from the first (md5_ramp_now; concurrent callers' seals are
// group-committed by the engine).  The MD5 of
// "RCLONE\0\0" || nonce || wire blocks runs on a host core: with a handful of objects in flight a
// core is ~10x a GPU lane (one dependency chain per stream).  A worker hashes
// batch k while this thread reads and seals batch k+1 into the other wire buffer.
static uint32_t hash_batch_blocks() {
  static const uint32_t v = [] {
    const char* e = getenv("RCLONE_AMD_HASH_BLOCKS");
    const int k = e ? atoi(e) : 16;
    return (uint32_t)std::max(1, std::min(256, k));
  }();
  return v;
}

extern "C" int32_t rc_compute_hash_with_nonce(rc_cipher* c, rc_reader src, const uint8_t nonce[24], uint8_t md5[16]) {
  if (!c || !src.read || !nonce || !md5) return RC_ERR_INVALID;
  const uint32_t batch = hash_batch_blocks();
  xs_engine* eng = xs_pool_next(cipher_pool(c));
  const int node = eng ? xs_engine_numa_node(eng) : -1;
  auto& w = xs::md5_workers(node);
  xs::HostMd5 m;
  m.update(kMagic, 8);
  m.update(nonce, 24);
  uint8_t n[24];
  memcpy(n, nonce, 24);
  PinnedBuf plain, wire[2];
  xs::Md5Job job;
  job.st = &m;
  int32_t err = RC_NIL;
  PhaseClock pc;
  pc.count(kHashCalls);
  bool counted = false;
  md5_stream_count(counted, true);
  bool ramp = md5_ramp_now();
  uint32_t cur = ramp ? 1u : batch;  // blocks in this seal: 1, 2, 4, ... batch while ramping
  for (int k = 0;; k ^= 1, ramp = md5_ramp_now(), cur = ramp ? std::min(2 * cur, batch) : batch) {
    if (!plain.ensure((size_t)batch * kBlockData, node) || !wire[k].ensure((size_t)batch * kBlockSize, node)) {
      err = RC_ERR_GPU;
      break;
    }
    int64_t total = 0;
    uint32_t nb = 0;
    bool end = false, short_read = false;
    int32_t e = RC_NIL;
    for (; nb < cur; nb++) {
      const int64_t got = read_fill(src, plain.p + (int64_t)nb * kBlockData, kBlockData, &e);
      if (got == 0) {  // encrypter.Read: n == 0 -> finish(err); io.Copy ends (EOF = success)
        end = true;
        break;
      }
      total += got;
      if (got < kBlockData || e != RC_NIL) {  // the next ReadFill must be a fresh call
        nb++;
        short_read = true;
        break;
      }
    }
    pc.mark(kHashRead);
    if (nb > 0) {
      if (!eng || xs_engine_seal(eng, c->data_key, n, 0, plain.p, (uint64_t)total, wire[k].p) != XS_OK) {
        err = RC_ERR_GPU;
        break;
      }
      pc.mark(kHashSeal);
      rc_nonce_add(n, nb);
      w.wait(&job);  // batch k-1 hashed (its buffer is the one sealed into next)
      pc.mark(kHashWait);
      job.p = wire[k].p;
      job.n = (size_t)(total + (int64_t)nb * kBlockHdr);
      // the stream's (probably) last batch: nothing is left to overlap it with, so no hand-off to
      // a scalar worker -- this thread, or an engine lane once the cores are all hashing
      if ((int64_t)job.n < inline_md5_below(ramp)) m.update(job.p, job.n);
      else w.submit(&job, !(end || short_read));
      pc.mark(kHashInline);
    }
    if (end) {
      err = e == RC_EOF ? RC_NIL : e;
      break;
    }
  }
  w.wait(&job);
  pc.mark(kHashFinal);
  md5_stream_count(counted, false);
  // the reference returns hashStr with CheckClose's error: the digest is set whenever the reads
  // succeeded, also when the close then fails
  if (err == RC_NIL) m.final(md5);
  if (src.close) {  // defer fs.CheckClose(in, &err)
    const int32_t ce = src.close(src.user);
    if (err == RC_NIL && ce != RC_NIL) err = ce;
  }
  return err;
}
