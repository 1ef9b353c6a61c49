// TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never linked into librclone_crypt.so.
//
// The GPU engine's C ABI (include/rclone_crypt_gpu.h: xs_engine_*, xs_pool_*, the name engine)
// implemented on host cores with the vectorised CPU oracle (oracle/xsalsa_simd.c: AVX-512 Salsa20,
// radix-2^44 Poly1305; the scalar AES of oracle/eme_oracle.c for names), so the same harnesses and
// the same host C++ run with every crypt byte on the CPU:
//   * tools/e2e_sync.cpp  -> tests/native/build/e2e_sync_cpu   (BASELINE configs[4]'s CPU baseline:
//     the reference's shape, crypt on the transfer's own thread, crypt.go:497-563);
//   * tools/seek_latency.cpp -> tests/native/build/seek_latency_cpu (a ranged 4 KiB read on one
//     core: cipher.go:972-1034 RangeSeek + Read).
// Like bench.py's cpu_baseline leg, this measures the CPU restatement beside the GPU path; it is
// never the product.  Semantics follow xs_api.cpp: failed blocks zero-filled with ok = 0, block j
// of a call sealed with nonce0 + first_block + j, ranged opens verify every tag over the whole
// block but write only the plaintext bytes [range_lo, range_hi).
//
// Threads: a per-object call (seal / open of one stream's batch) runs on the calling thread, as Go
// runs secretbox on the transfer's goroutine.  A many-object call (put_batch / seal_md5, the batch
// shapes) spreads its objects over effective_cpus() / (calls in flight) threads.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rclone_crypt_gpu.h"
#include "../../rclone_amd/csrc/rc_internal.h"
#include "../../rclone_amd/csrc/xs_host_md5.h"

extern "C" {
void orc_simd_secretbox_seal(uint8_t* out, const uint8_t* msg, size_t n, const uint8_t nonce[24],
                             const uint8_t key[32]);
int orc_simd_secretbox_open(uint8_t* out, const uint8_t* box, size_t boxlen, const uint8_t nonce[24],
                            const uint8_t key[32]);
int orc_simd_open_window(uint8_t* out, const uint8_t* box, size_t boxlen, const uint8_t nonce[24],
                         const uint8_t key[32], size_t lo, size_t hi);
int orc_simd_level(void);
void orc_nonce_add(uint8_t n[24], uint64_t x);
int orc_eme_transform(const uint8_t key[32], const uint8_t tweak[16], const uint8_t* in, uint8_t* out, int m,
                      int direction);
}

namespace xs {
static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}
std::vector<int> default_devices() { return {0}; }
}  // namespace xs

struct xs_engine {
  std::atomic<uint64_t> calls{0}, objects{0};
};
struct xs_pool {
  xs_engine e[1];
};

static std::atomic<int> g_active{0};  // many-object calls in flight (they share the cores)

static void parallel_objects(uint64_t n, const std::function<void(uint64_t)>& f) {
  const int active = ++g_active;
  const int cpus = std::max(1, xs::effective_cpus());
  const int threads = (int)std::min<uint64_t>(n, (uint64_t)std::max(1, cpus / std::max(1, active)));
  std::atomic<uint64_t> next{0};
  auto run = [&] {
    for (uint64_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; t++) th.emplace_back(run);
  run();
  for (auto& t : th) t.join();
  --g_active;
}

static uint64_t body_bytes(uint64_t len) { return len + ((len + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA) * XS_BLOCK_HDR; }

static void seal_blocks(const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block, const uint8_t* in,
                        uint64_t len, uint8_t* out) {
  for (uint64_t j = 0; j * XS_BLOCK_DATA < len; j++) {
    uint8_t n[24];
    memcpy(n, nonce0, 24);
    orc_nonce_add(n, first_block + j);
    const uint64_t m = std::min<uint64_t>(XS_BLOCK_DATA, len - j * XS_BLOCK_DATA);
    orc_simd_secretbox_seal(out + j * XS_BLOCK_SIZE, in + j * XS_BLOCK_DATA, m, n, key);
  }
}

// seal one object and MD5 its crypt file ("RCLONE\0\0" || nonce || wire blocks), block by block
// from a 64 KiB scratch when body == nullptr
static void seal_md5_one(const uint8_t key[32], const uint8_t nonce[24], const uint8_t* in, uint64_t len,
                         uint8_t* body, uint8_t md5[16]) {
  static const uint8_t magic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};
  xs::HostMd5 m;
  m.update(magic, 8);
  m.update(nonce, 24);
  std::vector<uint8_t> scratch(body ? 0 : XS_BLOCK_SIZE);
  for (uint64_t j = 0; j * XS_BLOCK_DATA < len; j++) {
    uint8_t n[24];
    memcpy(n, nonce, 24);
    orc_nonce_add(n, j);
    const uint64_t k = std::min<uint64_t>(XS_BLOCK_DATA, len - j * XS_BLOCK_DATA);
    uint8_t* w = body ? body + j * XS_BLOCK_SIZE : scratch.data();
    orc_simd_secretbox_seal(w, in + j * XS_BLOCK_DATA, k, n, key);
    m.update(w, k + XS_BLOCK_HDR);
  }
  m.final(md5);
}

extern "C" {
const char* xs_last_error(void) { return xs::g_err.c_str(); }
void* xs_host_alloc(size_t bytes) { return aligned_alloc(64, ((bytes ? bytes : 1) + 63) & ~(size_t)63); }
void* xs_host_alloc_node(size_t bytes, int) { return xs_host_alloc(bytes); }
void xs_host_free(void* p) { free(p); }
int xs_engine_numa_node(const xs_engine*) { return -1; }

xs_pool* xs_pool_create(const int*, int, uint32_t, int) {
  if (orc_simd_level() == 0) {
    xs::set_error("cpu engine: the CPU has no AVX2");
    return nullptr;
  }
  return new xs_pool();
}
void xs_pool_destroy(xs_pool* p) { delete p; }
xs_engine* xs_pool_next(xs_pool* p) { return p ? &p->e[0] : nullptr; }
xs_engine* xs_pool_engine(xs_pool* p, int i) { return p && i == 0 ? &p->e[0] : nullptr; }
void xs_engine_stats(xs_engine* e, uint64_t out[3]) {  // one "batch" per call: no cross-caller combining
  if (!e || !out) return;
  out[0] = out[1] = e->calls.load();
  out[2] = 0;
}
xs_engine* xs_engine_create(int, uint32_t, int) { return orc_simd_level() ? new xs_engine() : nullptr; }
void xs_engine_destroy(xs_engine* e) { delete e; }

int xs_engine_seal(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void* plain, uint64_t plain_len, void* body) {
  e->calls++;
  seal_blocks(key, nonce0, first_block, (const uint8_t*)plain, plain_len, (uint8_t*)body);
  return XS_OK;
}

int xs_engine_open_range(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         const void* body, uint64_t body_len, void* plain, uint8_t* ok, uint64_t range_lo,
                         uint64_t range_hi) {
  e->calls++;
  const uint8_t* in = (const uint8_t*)body;
  uint8_t* out = (uint8_t*)plain;
  for (uint64_t j = 0; j * XS_BLOCK_SIZE < body_len; j++) {
    uint8_t n[24];
    memcpy(n, nonce0, 24);
    orc_nonce_add(n, first_block + j);
    const uint64_t blen = std::min<uint64_t>(XS_BLOCK_SIZE, body_len - j * XS_BLOCK_SIZE);
    if (blen <= XS_BLOCK_HDR) {
      xs::set_error("cpu engine: truncated block");
      return XS_ERR_INVALID;
    }
    const uint64_t b0 = j * XS_BLOCK_DATA, len = blen - XS_BLOCK_HDR;
    // this block's share of [range_lo, range_hi), in block offsets
    const uint64_t lo = range_lo > b0 ? std::min(range_lo - b0, len) : 0;
    const uint64_t hi = range_hi > b0 ? std::min(range_hi - b0, len) : 0;
    const bool whole = lo == 0 && hi == len;
    ok[j] = (whole ? orc_simd_secretbox_open(out + b0, in + j * XS_BLOCK_SIZE, blen, n, key)
                   : orc_simd_open_window(out + b0, in + j * XS_BLOCK_SIZE, blen, n, key, lo, hi)) == 0;
    if (!ok[j]) memset(out + b0, 0, len);
  }
  return XS_OK;
}

int xs_engine_open(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void* body, uint64_t body_len, void* plain, uint8_t* ok) {
  return xs_engine_open_range(e, key, nonce0, first_block, body, body_len, plain, ok, 0, UINT64_MAX);
}

int xs_engine_seal_md5(xs_engine* e, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces, const uint64_t* offs,
                       const uint64_t* lens, const void* plain, uint8_t* md5) {
  e->calls++;
  e->objects += nobj;
  parallel_objects(nobj, [&](uint64_t i) {
    seal_md5_one(key, nonces + 24 * i, (const uint8_t*)plain + offs[i], lens[i], nullptr, md5 + 16 * i);
  });
  return XS_OK;
}

uint64_t xs_put_body_bytes(uint64_t nobj, const uint64_t* lens) {
  uint64_t t = 0;
  for (uint64_t i = 0; i < nobj; i++) t += (body_bytes(lens[i]) + 15) & ~15ull;
  return t;
}

int xs_engine_put_batch(xs_engine* e, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                        const uint64_t* offs, const uint64_t* lens, const void* plain, void* body, uint8_t* md5) {
  e->calls++;
  e->objects += nobj;
  std::vector<uint64_t> boff(nobj);
  for (uint64_t i = 0, pos = 0; i < nobj; i++) {
    boff[i] = pos;
    pos += (body_bytes(lens[i]) + 15) & ~15ull;
  }
  parallel_objects(nobj, [&](uint64_t i) {
    seal_md5_one(key, nonces + 24 * i, (const uint8_t*)plain + offs[i], lens[i], (uint8_t*)body + boff[i],
                 md5 + 16 * i);
  });
  return XS_OK;
}

int xs_pool_seal_md5(xs_pool* p, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces, const uint64_t* offs,
                     const uint64_t* lens, const void* plain, uint8_t* md5) {
  return xs_engine_seal_md5(&p->e[0], key, nobj, nonces, offs, lens, plain, md5);
}
}  // extern "C"

// name engine: EME on host cores (the oracle's AES) over the staged names, one lock per process
namespace rcn {
struct EmeDev {
  std::mutex mu;
  std::vector<uint8_t> h;
};
static EmeDev g_dev;

EmeDev* eme_acquire(size_t bytes, uint8_t** host) {
  g_dev.mu.lock();
  if (g_dev.h.size() < bytes) g_dev.h.resize(bytes);
  *host = g_dev.h.data();
  return &g_dev;
}

int32_t eme_run(EmeDev* dev, bool encrypt, const rc_cipher* c, size_t desc_off, size_t ndesc, size_t data_bytes,
                size_t total, double* ms) {
  const xs_name_desc* d = (const xs_name_desc*)(dev->h.data() + desc_off);
  if (total < desc_off) return RC_ERR_INVALID;
  std::vector<uint8_t> out;
  for (size_t i = 0; i < ndesc; i++) {
    if (d[i].off + 16ull * d[i].nblk > data_bytes || d[i].nblk < 1 || d[i].nblk > 128) return RC_ERR_INVALID;
    uint8_t* p = dev->h.data() + d[i].off;
    out.resize(16 * d[i].nblk);
    if (orc_eme_transform(c->name_key, c->name_tweak, p, out.data(), (int)d[i].nblk, encrypt ? 0 : 1) != 0)
      return RC_ERR_INVALID;
    memcpy(p, out.data(), out.size());
  }
  *ms = 0;
  return RC_NIL;
}

void eme_release(EmeDev* dev) { dev->mu.unlock(); }
}  // namespace rcn
