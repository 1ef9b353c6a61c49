// TEST INFRASTRUCTURE ONLY -- never linked into librclone_crypt.so.
//
// Host stand-in for the GPU side of librclone_crypt.so, so that the host C++ of the drop-in
// (rclone_amd/csrc/cipher.cpp, names.cpp, scrypt.cpp: the cipher.go mirror and the name cipher's
// host stages) can be built with AddressSanitizer / UBSan / ThreadSanitizer on a machine without a
// GPU (VERDICT r01 "What's missing" 5).  The engine entry points the host code calls are
// implemented here with the CPU oracle (oracle/xsalsa_oracle.c, oracle/eme_oracle.c), which is the
// checker the rest of the test suite uses; the device contract is kept: failed blocks are
// zero-filled with ok = 0, descriptor order and nonces as in xs_api.cpp.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rclone_crypt_gpu.h"
#include "../../rclone_amd/csrc/rc_internal.h"
#include "../../rclone_amd/csrc/xs_host_md5.h"

extern "C" {
void orc_secretbox_seal(uint8_t* out, const uint8_t* msg, size_t n, const uint8_t nonce[24], const uint8_t key[32]);
int orc_secretbox_open(uint8_t* out, const uint8_t* box, size_t boxlen, const uint8_t nonce[24],
                       const uint8_t key[32]);  // 0: authentic
void orc_nonce_add(uint8_t n[24], uint64_t x);
int orc_eme_transform(const uint8_t key[32], const uint8_t tweak[16], const uint8_t* in, uint8_t* out, int m,
                      int direction);  // direction != 0: decrypt
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

// Failure injection (tests): every engine submission (seal, open, ranged open -- one GPU batch each
// in the real library) takes a number from one process-wide counter; submissions numbered
// [g_fail_from, g_fail_from + g_fail_count) fail as a HIP error would (XS_ERR_HIP, last error set),
// writing nothing.  stub_engine_fail(-1, 0) turns it off.
static std::atomic<long> g_submits{0}, g_fail_from{-1}, g_fail_count{0}, g_failed{0};
static bool inject_failure() {
  const long k = g_submits.fetch_add(1);
  const long f = g_fail_from.load();
  if (f < 0 || k < f || k >= f + g_fail_count.load()) return false;
  g_failed++;
  xs::set_error("stub engine: injected failure of submission %ld", k);
  return true;
}

struct xs_engine {
  std::mutex mu;
  uint64_t calls = 0;
  uint64_t ranged = 0;
};
struct xs_pool {
  xs_engine e[2];
  std::mutex mu;
  unsigned rr = 0;
};

extern "C" {
long stub_engine_submissions(void) { return g_submits.load(); }
long stub_engine_failed(void) { return g_failed.load(); }
void stub_engine_fail(long from, long count) {
  g_fail_count = count;
  g_fail_from = from;
}
const char* xs_last_error(void) { return xs::g_err.c_str(); }
void* xs_host_alloc(size_t bytes) { return malloc(bytes ? bytes : 1); }
void* xs_host_alloc_node(size_t bytes, int) { return malloc(bytes ? bytes : 1); }
int xs_engine_numa_node(const xs_engine*) { return -1; }
void xs_host_free(void* p) { free(p); }

xs_pool* xs_pool_create(const int*, int, uint32_t, int) { return new xs_pool(); }
void xs_pool_destroy(xs_pool* p) { delete p; }
xs_engine* xs_pool_next(xs_pool* p) {
  std::lock_guard<std::mutex> g(p->mu);
  return &p->e[p->rr++ % 2];
}

int xs_engine_seal(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void* plain, uint64_t plain_len, void* body) {
  std::lock_guard<std::mutex> g(e->mu);
  e->calls++;
  if (inject_failure()) return XS_ERR_HIP;
  const uint8_t* in = (const uint8_t*)plain;
  uint8_t* out = (uint8_t*)body;
  for (uint64_t j = 0; j * XS_BLOCK_DATA < plain_len; j++) {
    uint8_t n[24];
    memcpy(n, nonce0, 24);
    orc_nonce_add(n, first_block + j);
    const uint64_t len = plain_len - j * XS_BLOCK_DATA < XS_BLOCK_DATA ? plain_len - j * XS_BLOCK_DATA : XS_BLOCK_DATA;
    orc_secretbox_seal(out + j * XS_BLOCK_SIZE, in + j * XS_BLOCK_DATA, len, n, key);
  }
  return XS_OK;
}

int xs_engine_open(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                   const void* body, uint64_t body_len, void* plain, uint8_t* ok) {
  std::lock_guard<std::mutex> g(e->mu);
  e->calls++;
  if (inject_failure()) return XS_ERR_HIP;
  if (getenv("STUB_TRACE"))
    fprintf(stderr, "open fb=%llu len=%llu in%%16=%u out%%16=%u\n", (unsigned long long)first_block,
            (unsigned long long)body_len, (unsigned)((uintptr_t)body & 15u), (unsigned)((uintptr_t)plain & 15u));
  const uint8_t* in = (const uint8_t*)body;
  uint8_t* out = (uint8_t*)plain;
  for (uint64_t j = 0; j * XS_BLOCK_SIZE < body_len; j++) {
    uint8_t n[24];
    memcpy(n, nonce0, 24);
    orc_nonce_add(n, first_block + j);
    const uint64_t blen = body_len - j * XS_BLOCK_SIZE < XS_BLOCK_SIZE ? body_len - j * XS_BLOCK_SIZE : XS_BLOCK_SIZE;
    if (blen <= XS_BLOCK_HDR) {
      xs::set_error("stub open: truncated block");
      return XS_ERR_INVALID;
    }
    ok[j] = orc_secretbox_open(out + j * XS_BLOCK_DATA, in + j * XS_BLOCK_SIZE, blen, n, key) == 0;
    if (!ok[j]) memset(out + j * XS_BLOCK_DATA, 0, blen - XS_BLOCK_HDR);
  }
  return XS_OK;
}

// Ranged open: the bytes outside [range_lo, range_hi) of a verified block are poisoned (0xA5), so a
// decrypter that serves bytes outside the range it asked for fails the harness's content checks.
int xs_engine_open_range(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         const void* body, uint64_t body_len, void* plain, uint8_t* ok, uint64_t range_lo,
                         uint64_t range_hi) {
  const int rc = xs_engine_open(e, key, nonce0, first_block, body, body_len, plain, ok);
  if (rc != XS_OK) return rc;
  std::lock_guard<std::mutex> g(e->mu);
  e->ranged++;
  uint8_t* out = (uint8_t*)plain;
  for (uint64_t j = 0; j * XS_BLOCK_SIZE < body_len; j++) {
    if (!ok[j]) continue;  // a failed block stays zero-filled whole
    const uint64_t blen = body_len - j * XS_BLOCK_SIZE < XS_BLOCK_SIZE ? body_len - j * XS_BLOCK_SIZE : XS_BLOCK_SIZE;
    for (uint64_t b = 0; b < blen - XS_BLOCK_HDR; b++) {
      const uint64_t pos = j * XS_BLOCK_DATA + b;
      if (pos < range_lo || pos >= range_hi) out[pos] = 0xA5;
    }
  }
  return XS_OK;
}

int xs_pool_seal_md5(xs_pool*, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces, const uint64_t* offs,
                     const uint64_t* lens, const void* plain, uint8_t* md5) {
  for (uint64_t i = 0; i < nobj; i++) {
    const uint64_t nb = (lens[i] + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
    std::vector<uint8_t> body(lens[i] + nb * XS_BLOCK_HDR + 1);
    xs_engine e;
    if (xs_engine_seal(&e, key, nonces + 24 * i, 0, (const uint8_t*)plain + offs[i], lens[i], body.data()) != XS_OK)
      return XS_ERR_HIP;
    xs::HostMd5 m;
    static const uint8_t magic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};
    m.update(magic, 8);
    m.update(nonces + 24 * i, 24);
    m.update(body.data(), body.size() - 1);
    m.final(md5 + 16 * i);
  }
  return XS_OK;
}
}  // extern "C"

// name engine: EME on the host (the oracle) over the staged names
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
  for (size_t i = 0; i < ndesc; i++) {
    if (d[i].off + 16ull * d[i].nblk > data_bytes || d[i].nblk < 1 || d[i].nblk > 128 || total < desc_off) abort();
    uint8_t* p = dev->h.data() + d[i].off;
    std::vector<uint8_t> out(16 * d[i].nblk);
    if (orc_eme_transform(c->name_key, c->name_tweak, p, out.data(), (int)d[i].nblk, encrypt ? 0 : 1) != 0) abort();
    memcpy(p, out.data(), out.size());
  }
  *ms = 0;
  return RC_NIL;
}

void eme_release(EmeDev* dev) { dev->mu.unlock(); }
}  // namespace rcn
