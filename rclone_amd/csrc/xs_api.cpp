// xs_api.cpp -- C ABI of the device primitives (include/rclone_crypt_gpu.h, xs_* part).
//
// Replaces the per-block secretbox.Seal / secretbox.Open calls of backend/crypt
// (cipher.go:737, :880) with batched launches: xs_keygen (per-block key schedule) then
// xs_seal/xs_open (one 64 KiB block per wave64).  The engine keeps per-slot device buffers and
// streams so host->device copies, kernels and device->host copies of consecutive batches
// overlap (the host-path number in DESIGN.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "xs_host_md5.h"
#include "xs_internal.h"
#include "xs_topo.h"

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
}  // namespace xs

// Pinned allocations made by xs_host_alloc (portable: mapped for every device): base -> (size,
// device address).  Engine requests on such buffers (every rc_* handle's staging) resolve their
// device address here instead of two HIP pointer queries per buffer per request.
namespace xs {
struct PinRange {
  size_t size;
  uint64_t dev;
};
static std::shared_mutex& pin_mu() {
  static std::shared_mutex* m = new std::shared_mutex();  // leaked: used until process exit
  return *m;
}
static std::map<uintptr_t, PinRange>& pins() {
  static auto* m = new std::map<uintptr_t, PinRange>();
  return *m;
}
void pin_register(void* p, size_t size) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return;  // not resolvable up front: such requests take the HIP query path
  }
  std::unique_lock<std::shared_mutex> g(pin_mu());
  pins()[(uintptr_t)p] = PinRange{size, (uint64_t)(uintptr_t)d};
}
void pin_unregister(void* p) {
  std::unique_lock<std::shared_mutex> g(pin_mu());
  pins().erase((uintptr_t)p);
}
// Device address of p when it lies inside a registered allocation.
static bool pin_lookup(const void* p, uint64_t* dev) {
  std::shared_lock<std::shared_mutex> g(pin_mu());
  auto& m = pins();
  auto it = m.upper_bound((uintptr_t)p);
  if (it == m.begin()) return false;
  --it;
  const uintptr_t off = (uintptr_t)p - it->first;
  if (off >= it->second.size) return false;
  *dev = it->second.dev + off;
  return true;
}
}  // namespace xs

using namespace xs;

static KeyArg key_arg(const uint8_t key[32]) {
  KeyArg k;
  for (int i = 0; i < 8; i++) {
    k.k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
             ((uint32_t)key[4 * i + 3] << 24);
  }
  return k;
}

static NonceArg nonce_arg(const uint8_t n[24]) {
  NonceArg a;
  for (int i = 0; i < 6; i++) {
    a.n[i] = (uint32_t)n[4 * i] | ((uint32_t)n[4 * i + 1] << 8) | ((uint32_t)n[4 * i + 2] << 16) |
             ((uint32_t)n[4 * i + 3] << 24);
  }
  return a;
}

static int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return XS_ERR_HIP;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

extern "C" {

const char* xs_version(void) { return "rclone_amd crypt 0.1 (gfx950)"; }

// sha256 of the sources and build flags this library was compiled from (rclone_amd/build.py
// passes it in); the tagged copy lets the loader read it from the file without loading it
#ifndef XS_BUILD_ID
#define XS_BUILD_ID "unstamped"
#endif
__attribute__((used)) static const char kBuildIdTag[] = "xs-build-id:" XS_BUILD_ID;
const char* xs_build_id(void) { return kBuildIdTag + 12; }
// the compiler that built it (rclone_amd/build.py compiler_id: the first 16 hex digits of a sha256
// over the resolved hipcc and clang paths, the clang binary's size and the ROCm .info release
// files -- file-system facts, hipcc is never run): the loader rebuilds a library whose compiler
// differs from the one installed next to the tree
#ifndef XS_BUILD_COMPILER
#define XS_BUILD_COMPILER "unstamped"
#endif
__attribute__((used)) static const char kBuildCompilerTag[] = "xs-build-compiler:" XS_BUILD_COMPILER;

const char* xs_last_error(void) { return g_err.c_str(); }

int xs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

size_t xs_workspace_bytes(uint64_t nblocks) { return (size_t)nblocks * sizeof(BlockKey); }

int xs_seal_object_dev(const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block, const void* d_plain,
                       uint64_t plain_len, void* d_body, void* d_workspace, void* stream) {
  if (!key || !nonce0 || !d_plain || !d_body || !d_workspace) {
    set_error("xs_seal_object_dev: null argument");
    return XS_ERR_INVALID;
  }
  if (plain_len == 0) return XS_OK;
  if (!aligned16(d_plain) || !aligned16(d_body) || !aligned16(d_workspace)) {
    set_error("xs_seal_object_dev: device buffers must be 16-byte aligned");
    return XS_ERR_INVALID;
  }
  const uint64_t nblocks = (plain_len + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
  hipStream_t s = (hipStream_t)stream;
  BlockKey* keys = (BlockKey*)d_workspace;
  hipError_t e = launch_keygen(0, key_arg(key), nonce_arg(nonce0), first_block, plain_len, nblocks, nullptr, keys, s);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  e = launch_crypt(true, keys, nblocks, (const uint8_t*)d_plain, (uint8_t*)d_body, nullptr, s);
  if (e != hipSuccess) return hip_fail(e, "seal launch");
  return XS_OK;
}

int xs_open_object_dev(const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block, const void* d_body,
                       uint64_t body_len, void* d_plain, uint8_t* d_ok, void* d_workspace, void* stream) {
  if (!key || !nonce0 || !d_body || !d_plain || !d_ok || !d_workspace) {
    set_error("xs_open_object_dev: null argument");
    return XS_ERR_INVALID;
  }
  if (body_len == 0) return XS_OK;
  if (!aligned16(d_plain) || !aligned16(d_body) || !aligned16(d_workspace)) {
    set_error("xs_open_object_dev: device buffers must be 16-byte aligned");
    return XS_ERR_INVALID;
  }
  const uint64_t nblocks = (body_len + XS_BLOCK_SIZE - 1) / XS_BLOCK_SIZE;
  const uint64_t last = body_len - (nblocks - 1) * XS_BLOCK_SIZE;
  if (last <= XS_BLOCK_HDR) {
    set_error("xs_open_object_dev: truncated block header (last block %llu bytes)", (unsigned long long)last);
    return XS_ERR_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  BlockKey* keys = (BlockKey*)d_workspace;
  hipError_t e = launch_keygen(1, key_arg(key), nonce_arg(nonce0), first_block, body_len, nblocks, nullptr, keys, s);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  e = launch_crypt(false, keys, nblocks, (const uint8_t*)d_body, (uint8_t*)d_plain, d_ok, s);
  if (e != hipSuccess) return hip_fail(e, "open launch");
  return XS_OK;
}

int xs_seal_batch_dev(const uint8_t key[32], const xs_block_desc* d_desc, uint64_t nblocks, const void* d_src,
                      uint64_t src_len, void* d_dst, uint64_t dst_len, void* d_workspace, void* stream) {
  if (!key || !d_desc || !d_src || !d_dst || !d_workspace) {
    set_error("xs_seal_batch_dev: null argument");
    return XS_ERR_INVALID;
  }
  if (nblocks == 0) return XS_OK;
  NonceArg bounds{};
  bounds.n[0] = (uint32_t)src_len; bounds.n[1] = (uint32_t)(src_len >> 32);
  bounds.n[2] = (uint32_t)dst_len; bounds.n[3] = (uint32_t)(dst_len >> 32);
  bounds.n[4] = (uint32_t)((uintptr_t)d_src & 15u); bounds.n[5] = (uint32_t)((uintptr_t)d_dst & 15u);
  hipStream_t s = (hipStream_t)stream;
  BlockKey* keys = (BlockKey*)d_workspace;
  hipError_t e = launch_keygen(2, key_arg(key), bounds, 0, 0, nblocks, d_desc, keys, s);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  e = launch_crypt(true, keys, nblocks, (const uint8_t*)d_src, (uint8_t*)d_dst, nullptr, s);
  if (e != hipSuccess) return hip_fail(e, "seal launch");
  return XS_OK;
}

int xs_open_batch_dev(const uint8_t key[32], const xs_block_desc* d_desc, uint64_t nblocks, const void* d_src,
                      uint64_t src_len, void* d_dst, uint64_t dst_len, uint8_t* d_ok, void* d_workspace,
                      void* stream) {
  if (!key || !d_desc || !d_src || !d_dst || !d_ok || !d_workspace) {
    set_error("xs_open_batch_dev: null argument");
    return XS_ERR_INVALID;
  }
  if (nblocks == 0) return XS_OK;
  NonceArg bounds{};
  bounds.n[0] = (uint32_t)src_len; bounds.n[1] = (uint32_t)(src_len >> 32);
  bounds.n[2] = (uint32_t)dst_len; bounds.n[3] = (uint32_t)(dst_len >> 32);
  bounds.n[4] = (uint32_t)((uintptr_t)d_src & 15u); bounds.n[5] = (uint32_t)((uintptr_t)d_dst & 15u);
  hipStream_t s = (hipStream_t)stream;
  BlockKey* keys = (BlockKey*)d_workspace;
  hipError_t e = launch_keygen(3, key_arg(key), bounds, 0, 0, nblocks, d_desc, keys, s);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  e = launch_crypt(false, keys, nblocks, (const uint8_t*)d_src, (uint8_t*)d_dst, d_ok, s);
  if (e != hipSuccess) return hip_fail(e, "open launch");
  return XS_OK;
}

int xs_keygen_object_dev(int seal, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         uint64_t len, void* d_workspace, void* stream) {
  if (!key || !nonce0 || !d_workspace || !aligned16(d_workspace)) {
    set_error("xs_keygen_object_dev: bad argument");
    return XS_ERR_INVALID;
  }
  if (len == 0) return XS_OK;
  const uint64_t unit = seal ? XS_BLOCK_DATA : XS_BLOCK_SIZE;
  const uint64_t nblocks = (len + unit - 1) / unit;
  if (!seal && len - (nblocks - 1) * XS_BLOCK_SIZE <= XS_BLOCK_HDR) {
    set_error("xs_keygen_object_dev: truncated block header");
    return XS_ERR_INVALID;
  }
  hipError_t e = launch_keygen(seal ? 0 : 1, key_arg(key), nonce_arg(nonce0), first_block, len, nblocks, nullptr,
                               (BlockKey*)d_workspace, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  return XS_OK;
}

int xs_crypt_dev(int seal, const void* d_workspace, uint64_t nblocks, const void* d_src, void* d_dst, uint8_t* d_ok,
                 void* stream) {
  if (!d_workspace || !d_src || !d_dst || (!seal && !d_ok)) {
    set_error("xs_crypt_dev: null argument");
    return XS_ERR_INVALID;
  }
  hipError_t e = launch_crypt(seal != 0, (const BlockKey*)d_workspace, nblocks, (const uint8_t*)d_src,
                              (uint8_t*)d_dst, d_ok, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "crypt launch");
  return XS_OK;
}

int xs_keygen_batch_dev(int seal, const uint8_t key[32], const xs_block_desc* d_desc, uint64_t nblocks,
                        const void* d_src, uint64_t src_len, const void* d_dst, uint64_t dst_len, void* d_workspace,
                        void* stream) {
  if (!key || !d_desc || !d_src || !d_dst || !d_workspace || !aligned16(d_workspace)) {
    set_error("xs_keygen_batch_dev: bad argument");
    return XS_ERR_INVALID;
  }
  if (nblocks == 0) return XS_OK;
  NonceArg bounds{};
  bounds.n[0] = (uint32_t)src_len; bounds.n[1] = (uint32_t)(src_len >> 32);
  bounds.n[2] = (uint32_t)dst_len; bounds.n[3] = (uint32_t)(dst_len >> 32);
  bounds.n[4] = (uint32_t)((uintptr_t)d_src & 15u); bounds.n[5] = (uint32_t)((uintptr_t)d_dst & 15u);
  hipError_t e = launch_keygen(seal ? 2 : 3, key_arg(key), bounds, 0, 0, nblocks, d_desc, (BlockKey*)d_workspace,
                               (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "keygen launch");
  return XS_OK;
}

int xs_fill_random_dev(void* d, uint64_t nbytes, uint64_t seed, void* stream) {
  if (!d || (nbytes & 7u) || !aligned16(d)) {
    set_error("xs_fill_random_dev: need a 16-byte aligned buffer and a multiple of 8 bytes");
    return XS_ERR_INVALID;
  }
  hipError_t e = launch_fill((uint64_t*)d, nbytes / 8, seed, 0, 1, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "fill launch");
  return XS_OK;
}

int xs_md5_batch_dev(const xs_md5_desc* d_desc, uint64_t n, const void* d_src, uint64_t src_len, uint8_t* d_digest,
                     uint8_t* d_ok, void* stream) {
  if (n == 0) return XS_OK;
  if (!d_desc || !d_digest || (!d_src && src_len)) {
    set_error("xs_md5_batch_dev: null argument");
    return XS_ERR_INVALID;
  }
  hipError_t e = launch_md5(d_desc, n, (const uint8_t*)d_src, src_len, d_digest, d_ok, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "md5 launch");
  return XS_OK;
}

int xs_fill_blocks_dev(void* d, uint64_t nblocks, uint64_t first_block, uint64_t block_stride, uint64_t seed,
                       void* stream) {
  if (!d || !aligned16(d) || block_stride == 0) {
    set_error("xs_fill_blocks_dev: need a 16-byte aligned buffer and block_stride >= 1");
    return XS_ERR_INVALID;
  }
  hipError_t e = launch_fill((uint64_t*)d, nblocks * 8192u, seed, first_block, block_stride, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "fill launch");
  return XS_OK;
}

void* xs_host_alloc_node(size_t bytes, int node) {
  void* p = nullptr;
  hipError_t e = hipErrorUnknown;
  if (node >= 0 && numa_enabled()) {
    // the pages follow the calling thread's policy (hipHostMallocNumaUser), preferred = node
    xs::ScopedMemPolicy pol(node);
    e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable | hipHostMallocNumaUser);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess) e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable);
  if (e != hipSuccess) {
    set_error("hipHostMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  xs::pin_register(p, bytes ? bytes : 1);
  return p;
}

void* xs_host_alloc(size_t bytes) { return xs_host_alloc_node(bytes, -1); }

// NUMA node of a device's PCI function (sysfs), cached per device
int xs_device_numa_node(int device) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  char bus[64] = {0};
  int node = -1;
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) == hipSuccess) node = xs::pci_numa_node(bus);
  else (void)hipGetLastError();
  cache[device] = node;
  return node;
}

void xs_host_free(void* p) {
  if (!p) return;
  xs::pin_unregister(p);
  (void)hipHostFree(p);
}

}  // extern "C"

// ---------------------------------------------------------------- engine
struct xs_engine {
  int device = 0;
  int numa = -1;  // NUMA node of the device: the engine's pinned staging and host threads go there
  uint32_t batch = 0;
  std::mutex mu;
  struct Slot {
    hipStream_t s = nullptr;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    BlockKey* d_keys = nullptr;
    uint8_t* d_ok = nullptr;
    uint8_t* zc_keys = nullptr;  // key schedules of a zero-copy chunk (kZcChunk blocks)
    uint8_t* zc_ok = nullptr;
    size_t zc_keys_cap = 0, zc_ok_cap = 0;
  };
  std::vector<Slot> slots;
  // ---- cross-caller coalescing (group commit, see engine_submit)
  struct Req {
    bool seal;
    uint8_t key[32];
    uint8_t nonce0[24];
    uint64_t first_block, nblocks, in_len, out_len;
    const uint8_t* in;
    uint8_t* out;
    uint8_t* ok;
    int rc;
    bool done;
    // zero-copy: in/out are pinned host memory the kernels can address directly (d_in/d_out)
    bool zc;
    uint64_t d_in, d_out;
    uint64_t blk0;  // first block within its combined batch
    // OPEN: the plaintext bytes [range_lo, range_hi) of out the caller will read (xs_engine_open_range);
    // the fused kernel leaves the rest of a full block's 4 KiB groups undecrypted
    uint64_t range_lo, range_hi;
    // woken (under qmu) when the request is done or when it heads the queue and the lead is free:
    // one waiter at a time, not every caller on each completion
    std::condition_variable cv;
  };
  bool coalesce = true;
  int host_md5_threads = -1;  // -1: the default (XS_MD5_HOST_THREADS or half the cores, <= 8); 0: GPU only
  bool zero_copy = true;  // pinned caller buffers go to the kernels directly (no staging copies)
  std::mutex qmu;
  std::vector<Req*> queue;
  std::atomic<size_t> qcount{0};  // queue.size(), readable without qmu (the leader's issue-while-waiting poll)
  bool overlap = false;           // XS_ENGINE_OVERLAP=1: the leader issues newly queued requests while it
                                  // waits (lower latency at low load, less coalescing: off by default)
  bool wake_all = false;          // XS_ENGINE_WAKE_ALL=1: one shared condition, every waiter woken (A/B)
  bool one_run = true;            // a combined batch holds one (direction, key) run (XS_BATCH_ONE_RUN=0: mixed)
  std::condition_variable qcv;    // the shared condition of wake_all
  bool leader = false;
  struct CSlot {  // one combined batch in flight
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    uint8_t *in = nullptr, *out = nullptr, *ok = nullptr, *desc = nullptr;
    BlockKey* keys = nullptr;
    xs_block_desc* h_desc = nullptr;  // pinned
    uint8_t* h_ok = nullptr;          // pinned: verdicts of a zero-copy batch
    uint64_t d_h_desc = 0, d_h_ok = 0;  // their device addresses
    uint32_t* h_flag = nullptr;  // pinned completion word of a fused batch (the kernel stores seq)
    uint64_t d_h_flag = 0;
    uint32_t* d_ctr = nullptr;   // workgroups finished (the last one resets it and stores the word)
    uint32_t seq = 0;
    bool spin = false;           // wait by polling h_flag instead of the event
    bool zc = false;
    std::vector<Req*> batch;
    uint64_t blocks = 0;
    int rc = XS_OK;
  };
  std::vector<CSlot> cslots;  // [0, ncslots): the leader's ring; then the express lanes
  size_t ncslots = 0, nexpress = 2;
  uint64_t express_max = 4;  // requests of at most this many blocks may take an express lane
  std::atomic<uint32_t> express_busy{0};  // bit i: express lane i in use
  std::atomic<uint64_t> st_express{0};
  uint64_t c_cap_blocks = 0, c_cap_bytes = 0;
  uint64_t st_batches = 0, st_reqs = 0, st_blocks = 0;
  std::atomic<uint64_t> st_host_md5_objs{0}, st_host_md5_bytes{0}, st_md5_objs{0};
  // grow-only buffers of xs_engine_seal_md5 (whole objects per group)
  struct HashBufs {
    uint8_t* d_plain = nullptr;
    uint8_t* d_body = nullptr;
    uint8_t* d_desc = nullptr;
    uint8_t* d_mdesc = nullptr;
    uint8_t* d_digest = nullptr;
    BlockKey* d_keys = nullptr;
    size_t plain_cap = 0, body_cap = 0, desc_cap = 0, mdesc_cap = 0, digest_cap = 0, keys_cap = 0;
    uint8_t* route[2] = {nullptr, nullptr};  // pinned: host-routed bodies of seal_md5 groups
    size_t route_cap[2] = {0, 0};
    hipStream_t aux = nullptr;        // wire-body D2H, overlapped with the MD5 lanes
    hipEvent_t ev_sealed = nullptr;   // the group's seal is done (aux may copy the bodies)
  } hb;
};

// Device address of pinned (page-locked, device-mapped) host memory, or false for anything else
// (pageable memory, device memory): only such buffers are handed to the kernels directly.
static bool host_dev_ptr(const void* p, uint64_t* dev, int device) {
  if (!p) return false;
  if (pin_lookup(p, dev)) return true;  // xs_host_alloc memory: portable, mapped for every device
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory reports an error; clear it
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  // mapped for this engine's device: allocated portable, or while that device was current
  if (!(a.allocationFlags & hipHostMallocPortable) && a.device != device) return false;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return false;
  }
  *dev = (uint64_t)(uintptr_t)d;
  return true;
}

constexpr uint64_t kZcChunk = 4096;  // blocks per zero-copy launch of a large pinned request

static bool grow(uint8_t** p, size_t* cap, size_t need) {
  if (*cap >= need) return true;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, need ? need : 16) != hipSuccess) return false;
  *cap = need;
  return true;
}

static bool grow_pinned(uint8_t** p, size_t* cap, size_t need, int node) {  // grow-only (x1.5), contents dropped
  if (*cap >= need) return true;
  xs_host_free(*p);
  *p = nullptr;
  *cap = 0;
  const size_t want = std::max(need, need / 2 * 3);
  *p = (uint8_t*)xs_host_alloc_node(want ? want : 16, node);
  if (!*p) return false;
  *cap = want;
  return true;
}

static void engine_free(xs_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  for (auto& sl : e->slots) {
    if (sl.s) (void)hipStreamSynchronize(sl.s);
    (void)hipFree(sl.d_in);
    (void)hipFree(sl.d_out);
    (void)hipFree(sl.d_keys);
    (void)hipFree(sl.d_ok);
    (void)hipFree(sl.zc_keys);
    (void)hipFree(sl.zc_ok);
    if (sl.s) (void)hipStreamDestroy(sl.s);
  }
  for (auto& c : e->cslots) {
    if (c.s) (void)hipStreamSynchronize(c.s);
    (void)hipFree(c.in);
    (void)hipFree(c.out);
    (void)hipFree(c.ok);
    (void)hipFree(c.desc);
    (void)hipFree(c.keys);
    (void)hipHostFree(c.h_desc);
    (void)hipHostFree(c.h_ok);
    (void)hipHostFree(c.h_flag);
    (void)hipFree(c.d_ctr);
    if (c.done) (void)hipEventDestroy(c.done);
    if (c.s) (void)hipStreamDestroy(c.s);
  }
  (void)hipFree(e->hb.d_plain);
  (void)hipFree(e->hb.d_body);
  (void)hipFree(e->hb.d_desc);
  (void)hipFree(e->hb.d_mdesc);
  (void)hipFree(e->hb.d_digest);
  (void)hipFree(e->hb.d_keys);
  if (e->hb.aux) {
    (void)hipStreamSynchronize(e->hb.aux);
    (void)hipStreamDestroy(e->hb.aux);
  }
  if (e->hb.ev_sealed) (void)hipEventDestroy(e->hb.ev_sealed);
  for (auto* r : e->hb.route) xs_host_free(r);
  delete e;
}

extern "C" xs_engine* xs_engine_create(int device, uint32_t batch_blocks, int nslots) {
  if (batch_blocks == 0) batch_blocks = 256;
  if (nslots <= 0) nslots = 3;
  if (device < 0 || device >= xs_device_count()) {
    set_error("xs_engine_create: no HIP device %d", device);
    return nullptr;
  }
  xs_engine* e = new xs_engine();
  e->device = device;
  e->numa = numa_enabled() ? xs_device_numa_node(device) : -1;
  e->batch = batch_blocks;
  if (hipSetDevice(device) != hipSuccess) {
    set_error("hipSetDevice(%d) failed", device);
    delete e;
    return nullptr;
  }
  e->slots.resize(nslots);
  for (auto& sl : e->slots) {
    const size_t io = (size_t)batch_blocks * XS_BLOCK_SIZE;
    if (hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&sl.d_in, io) != hipSuccess || hipMalloc(&sl.d_out, io) != hipSuccess ||
        hipMalloc(&sl.d_keys, (size_t)batch_blocks * sizeof(BlockKey)) != hipSuccess ||
        hipMalloc(&sl.d_ok, batch_blocks) != hipSuccess) {
      set_error("xs_engine_create: device allocation failed");
      engine_free(e);
      return nullptr;
    }
  }
  // coalescing buffers: one combined batch of up to batch_blocks blocks from many callers
  // (+16 bytes of alignment slack per block for the per-request 16-byte alignment)
  e->c_cap_blocks = batch_blocks;
  e->c_cap_bytes = (uint64_t)batch_blocks * (XS_BLOCK_SIZE + 16);
  e->ncslots = (size_t)nslots;
  if (const char* v = getenv("XS_EXPRESS_LANES")) e->nexpress = std::min<size_t>(strtoull(v, nullptr, 10), 8);
  e->cslots.resize(e->ncslots + e->nexpress);
  int prio_least = 0, prio_greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
  for (auto& c : e->cslots) {
    const bool express = &c >= &e->cslots[e->ncslots];
    if ((express ? hipStreamCreateWithPriority(&c.s, hipStreamNonBlocking, prio_greatest)
                 : hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking)) != hipSuccess ||
        hipEventCreateWithFlags(&c.done, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c.in, e->c_cap_bytes) != hipSuccess || hipMalloc(&c.out, e->c_cap_bytes) != hipSuccess ||
        hipMalloc(&c.ok, batch_blocks) != hipSuccess ||
        hipMalloc(&c.desc, (size_t)batch_blocks * sizeof(xs_block_desc)) != hipSuccess ||
        hipMalloc(&c.keys, (size_t)batch_blocks * sizeof(BlockKey)) != hipSuccess ||
        hipHostMalloc(&c.h_desc, (size_t)batch_blocks * sizeof(xs_block_desc), hipHostMallocPortable) != hipSuccess ||
        hipHostMalloc(&c.h_ok, batch_blocks, hipHostMallocPortable) != hipSuccess ||
        !host_dev_ptr(c.h_desc, &c.d_h_desc, device) || !host_dev_ptr(c.h_ok, &c.d_h_ok, device) ||
        hipHostMalloc(&c.h_flag, 64, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        !host_dev_ptr(c.h_flag, &c.d_h_flag, device) || hipMalloc(&c.d_ctr, 4) != hipSuccess ||
        hipMemset(c.d_ctr, 0, 4) != hipSuccess) {
      set_error("xs_engine_create: device allocation failed");
      engine_free(e);
      return nullptr;
    }
    // hipHostMalloc does not promise zeroed memory: a stale word equal to the first sequence
    // number would end the first spin wait before the kernel ran
    memset(c.h_flag, 0, 64);
    c.seq = 0;
  }
  if (hipStreamCreateWithFlags(&e->hb.aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->hb.ev_sealed, hipEventDisableTiming) != hipSuccess) {
    set_error("xs_engine_create: stream/event creation failed");
    engine_free(e);
    return nullptr;
  }
  if (const char* v = getenv("XS_ENGINE_COALESCE")) e->coalesce = atoi(v) != 0;
  if (const char* v = getenv("XS_ENGINE_ZERO_COPY")) e->zero_copy = atoi(v) != 0;
  if (const char* v = getenv("XS_EXPRESS_MAX")) e->express_max = strtoull(v, nullptr, 10);
  if (const char* v = getenv("XS_ENGINE_OVERLAP")) e->overlap = atoi(v) != 0;
  if (const char* v = getenv("XS_ENGINE_WAKE_ALL")) e->wake_all = atoi(v) != 0;
  if (const char* v = getenv("XS_BATCH_ONE_RUN")) e->one_run = atoi(v) != 0;
  return e;
}

extern "C" void xs_engine_set_coalesce(xs_engine* e, int on) {
  if (e) e->coalesce = on != 0;
}

extern "C" void xs_engine_stats(xs_engine* e, uint64_t out[3]) {
  if (!e || !out) return;
  std::lock_guard<std::mutex> g(e->qmu);
  out[0] = e->st_batches;
  out[1] = e->st_reqs;
  out[2] = e->st_blocks;
}

extern "C" void xs_engine_destroy(xs_engine* e) { engine_free(e); }

extern "C" int xs_engine_numa_node(const xs_engine* e) { return e ? e->numa : -1; }
extern "C" int xs_engine_device(const xs_engine* e) { return e ? e->device : -1; }

static int engine_sync(xs_engine* e) {
  int rc = XS_OK;
  for (auto& sl : e->slots) {
    hipError_t err = hipStreamSynchronize(sl.s);
    if (err != hipSuccess && rc == XS_OK) rc = hip_fail(err, "engine stream");
  }
  return rc;
}

static int engine_submit(xs_engine* e, bool seal, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         const void* in, uint64_t in_len, void* out, uint8_t* ok, uint64_t nblocks, uint64_t range_lo = 0,
                         uint64_t range_hi = UINT64_MAX);

static int engine_seal_direct(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* plain, uint64_t plain_len, void* body);
static int engine_open_direct(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* body, uint64_t body_len, void* plain, uint8_t* ok);

extern "C" int xs_engine_seal(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* plain, uint64_t plain_len, void* body) {
  if (!e || !key || !nonce0 || (plain_len && (!plain || !body))) {
    set_error("xs_engine_seal: null argument");
    return XS_ERR_INVALID;
  }
  if (plain_len == 0) return XS_OK;
  const uint64_t nblocks = (plain_len + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
  if (e->coalesce && nblocks <= e->c_cap_blocks)
    return engine_submit(e, true, key, nonce0, first_block, plain, plain_len, body, nullptr, nblocks);
  return engine_seal_direct(e, key, nonce0, first_block, plain, plain_len, body);
}

static int engine_seal_direct(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* plain, uint64_t plain_len, void* body) {
  std::lock_guard<std::mutex> g(e->mu);
  if (hipSetDevice(e->device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
  const KeyArg k = key_arg(key);
  const NonceArg n = nonce_arg(nonce0);
  const uint64_t nblocks = (plain_len + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
  uint64_t dp = 0, db = 0;
  if (e->zero_copy && host_dev_ptr(plain, &dp, e->device) && host_dev_ptr(body, &db, e->device) && !(dp & 15u) && !(db & 15u)) {
    // pinned caller buffers: the kernels read and write them over PCIe in large chunks (the
    // link, not the launches, is then the limit), no staging copies
    for (uint64_t b0 = 0, chunk = 0; b0 < nblocks; b0 += kZcChunk, chunk++) {
      auto& sl = e->slots[chunk % e->slots.size()];
      const uint64_t nb = std::min<uint64_t>(nblocks - b0, kZcChunk);
      const uint64_t in_off = b0 * XS_BLOCK_DATA;
      if (!grow(&sl.zc_keys, &sl.zc_keys_cap, kZcChunk * sizeof(BlockKey))) return hip_fail(hipErrorOutOfMemory, "keys");
      hipError_t err = launch_keygen(0, k, n, first_block + b0, plain_len - in_off, nb, nullptr, (BlockKey*)sl.zc_keys, sl.s);
      if (err != hipSuccess) return hip_fail(err, "keygen");
      err = launch_crypt(true, (BlockKey*)sl.zc_keys, nb, (const uint8_t*)(uintptr_t)(dp + in_off),
                         (uint8_t*)(uintptr_t)(db + b0 * XS_BLOCK_SIZE), nullptr, sl.s);
      if (err != hipSuccess) return hip_fail(err, "seal");
    }
    return engine_sync(e);
  }
  for (uint64_t b0 = 0, chunk = 0; b0 < nblocks; b0 += e->batch, chunk++) {
    auto& sl = e->slots[chunk % e->slots.size()];
    const uint64_t nb = (nblocks - b0) < e->batch ? (nblocks - b0) : e->batch;
    const uint64_t in_off = b0 * XS_BLOCK_DATA;
    const uint64_t in_bytes = (plain_len - in_off) < nb * XS_BLOCK_DATA ? (plain_len - in_off) : nb * XS_BLOCK_DATA;
    const uint64_t out_bytes = in_bytes + nb * XS_BLOCK_HDR;
    hipError_t err = hipMemcpyAsync(sl.d_in, (const uint8_t*)plain + in_off, in_bytes, hipMemcpyHostToDevice, sl.s);
    if (err != hipSuccess) return hip_fail(err, "H2D");
    err = launch_keygen(0, k, n, first_block + b0, in_bytes, nb, nullptr, sl.d_keys, sl.s);
    if (err != hipSuccess) return hip_fail(err, "keygen");
    err = launch_crypt(true, sl.d_keys, nb, sl.d_in, sl.d_out, nullptr, sl.s);
    if (err != hipSuccess) return hip_fail(err, "seal");
    err = hipMemcpyAsync((uint8_t*)body + b0 * XS_BLOCK_SIZE, sl.d_out, out_bytes, hipMemcpyDeviceToHost, sl.s);
    if (err != hipSuccess) return hip_fail(err, "D2H");
  }
  return engine_sync(e);
}

// The descriptor's group window for block j of an OPEN request whose caller reads only plaintext
// bytes [lo, hi): 0 = the whole block, else XS_DESC_WINDOW | one bit per 4 KiB group to decrypt.
// Group g is keystream blocks 64g..64g+63, i.e. plaintext bytes [4096g - 32, 4096g + 4064) of the
// block (keystream block 0's first 32 bytes are the Poly1305 key); the last 32 bytes (keystream
// block 1024) are always written.
static uint32_t open_window(uint64_t lo, uint64_t hi, uint64_t j) {
  const uint64_t b0 = j * XS_BLOCK_DATA, b1 = b0 + XS_BLOCK_DATA;
  if (lo <= b0 && hi >= b1) return 0u;
  uint32_t mask = 0;
  if (lo < b1 && hi > b0 && hi > lo) {
    const uint64_t a = std::max(lo, b0) - b0, z = std::min(hi, b1) - b0;  // [a, z) within the block
    const uint64_t g0 = (a + 32) / XS_WINDOW_GROUP, g1 = std::min<uint64_t>((z - 1 + 32) / XS_WINDOW_GROUP, 15);
    for (uint64_t g = g0; g <= g1; g++) mask |= 1u << g;
  }
  return XS_DESC_WINDOW | mask;
}

extern "C" int xs_engine_open_range(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                                    const void* body, uint64_t body_len, void* plain, uint8_t* ok, uint64_t range_lo,
                                    uint64_t range_hi) {
  if (!e || !key || !nonce0 || (body_len && (!body || !plain || !ok))) {
    set_error("xs_engine_open_range: null argument");
    return XS_ERR_INVALID;
  }
  if (body_len == 0) return XS_OK;
  const uint64_t nblocks = (body_len + XS_BLOCK_SIZE - 1) / XS_BLOCK_SIZE;
  if (body_len - (nblocks - 1) * XS_BLOCK_SIZE <= XS_BLOCK_HDR) {
    set_error("xs_engine_open_range: truncated block header");
    return XS_ERR_INVALID;
  }
  if (e->coalesce && nblocks <= e->c_cap_blocks)
    return engine_submit(e, false, key, nonce0, first_block, body, body_len, plain, ok, nblocks, range_lo, range_hi);
  return engine_open_direct(e, key, nonce0, first_block, body, body_len, plain, ok);  // writes every byte
}

extern "C" int xs_engine_open(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* body, uint64_t body_len, void* plain, uint8_t* ok) {
  if (!e || !key || !nonce0 || (body_len && (!body || !plain || !ok))) {
    set_error("xs_engine_open: null argument");
    return XS_ERR_INVALID;
  }
  if (body_len == 0) return XS_OK;
  const uint64_t nblocks = (body_len + XS_BLOCK_SIZE - 1) / XS_BLOCK_SIZE;
  if (body_len - (nblocks - 1) * XS_BLOCK_SIZE <= XS_BLOCK_HDR) {
    set_error("xs_engine_open: truncated block header");
    return XS_ERR_INVALID;
  }
  if (e->coalesce && nblocks <= e->c_cap_blocks)
    return engine_submit(e, false, key, nonce0, first_block, body, body_len, plain, ok, nblocks);
  return engine_open_direct(e, key, nonce0, first_block, body, body_len, plain, ok);
}

static int engine_open_direct(xs_engine* e, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                              const void* body, uint64_t body_len, void* plain, uint8_t* ok) {
  const uint64_t nblocks = (body_len + XS_BLOCK_SIZE - 1) / XS_BLOCK_SIZE;
  std::lock_guard<std::mutex> g(e->mu);
  if (hipSetDevice(e->device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
  const KeyArg k = key_arg(key);
  const NonceArg n = nonce_arg(nonce0);
  uint64_t dbody = 0, dplain = 0;
  if (e->zero_copy && host_dev_ptr(body, &dbody, e->device) && host_dev_ptr(plain, &dplain, e->device) && !(dbody & 15u) && !(dplain & 15u)) {
    // pinned caller buffers: no data copies, only the verdicts come back
    for (uint64_t b0 = 0, chunk = 0; b0 < nblocks; b0 += kZcChunk, chunk++) {
      auto& sl = e->slots[chunk % e->slots.size()];
      const uint64_t nb = std::min<uint64_t>(nblocks - b0, kZcChunk);
      const uint64_t in_off = b0 * XS_BLOCK_SIZE;
      if (!grow(&sl.zc_keys, &sl.zc_keys_cap, kZcChunk * sizeof(BlockKey)) || !grow(&sl.zc_ok, &sl.zc_ok_cap, kZcChunk))
        return hip_fail(hipErrorOutOfMemory, "keys");
      hipError_t err = launch_keygen(1, k, n, first_block + b0, body_len - in_off, nb, nullptr, (BlockKey*)sl.zc_keys, sl.s);
      if (err != hipSuccess) return hip_fail(err, "keygen");
      err = launch_crypt(false, (BlockKey*)sl.zc_keys, nb, (const uint8_t*)(uintptr_t)(dbody + in_off),
                         (uint8_t*)(uintptr_t)(dplain + b0 * XS_BLOCK_DATA), sl.zc_ok, sl.s);
      if (err != hipSuccess) return hip_fail(err, "open");
      err = hipMemcpyAsync(ok + b0, sl.zc_ok, nb, hipMemcpyDeviceToHost, sl.s);
      if (err != hipSuccess) return hip_fail(err, "D2H ok");
    }
    return engine_sync(e);
  }
  for (uint64_t b0 = 0, chunk = 0; b0 < nblocks; b0 += e->batch, chunk++) {
    auto& sl = e->slots[chunk % e->slots.size()];
    const uint64_t nb = (nblocks - b0) < e->batch ? (nblocks - b0) : e->batch;
    const uint64_t in_off = b0 * XS_BLOCK_SIZE;
    const uint64_t in_bytes = (body_len - in_off) < nb * XS_BLOCK_SIZE ? (body_len - in_off) : nb * XS_BLOCK_SIZE;
    const uint64_t out_bytes = in_bytes - nb * XS_BLOCK_HDR;
    hipError_t err = hipMemcpyAsync(sl.d_in, (const uint8_t*)body + in_off, in_bytes, hipMemcpyHostToDevice, sl.s);
    if (err != hipSuccess) return hip_fail(err, "H2D");
    err = launch_keygen(1, k, n, first_block + b0, in_bytes, nb, nullptr, sl.d_keys, sl.s);
    if (err != hipSuccess) return hip_fail(err, "keygen");
    err = launch_crypt(false, sl.d_keys, nb, sl.d_in, sl.d_out, sl.d_ok, sl.s);
    if (err != hipSuccess) return hip_fail(err, "open");
    err = hipMemcpyAsync((uint8_t*)plain + b0 * XS_BLOCK_DATA, sl.d_out, out_bytes, hipMemcpyDeviceToHost, sl.s);
    if (err != hipSuccess) return hip_fail(err, "D2H");
    err = hipMemcpyAsync(ok + b0, sl.d_ok, nb, hipMemcpyDeviceToHost, sl.s);
    if (err != hipSuccess) return hip_fail(err, "D2H ok");
  }
  return engine_sync(e);
}

// ---------------------------------------------------------------- cross-caller coalescing
// rclone runs many transfers/checkers at once (--transfers, --checkers), each handle sealing
// or opening a few blocks at a time (cipher.go:719-745, :862-898).  Instead of one GPU round
// trip per handle, callers queue their requests and the first one in becomes the leader: it
// packs every queued request (up to the engine's batch capacity) into ONE descriptor batch --
// per-request H2D straight from the caller's buffer, one keygen per (direction, key), one crypt
// launch per direction, per-request D2H -- and wakes the owners.  Leadership passes on once
// the leader's own request is done, so a lone caller sees no queueing delay.
static void nonce_plus(uint8_t out[24], const uint8_t n0[24], uint64_t x) {
  memcpy(out, n0, 24);
  uint64_t carry = 0;
  for (int i = 0; i < 8; i++) {
    const uint64_t sum = (uint64_t)out[i] + (uint8_t)(x >> (8 * i)) + carry;
    out[i] = (uint8_t)sum;
    carry = sum >> 8;
  }
  for (int i = 8; i < 24 && carry; i++) {
    const uint64_t sum = (uint64_t)out[i] + carry;
    out[i] = (uint8_t)sum;
    carry = sum >> 8;
  }
}

static NonceArg bounds_arg(uint64_t src_len, uint64_t dst_len);

// Wait for fused batches by polling their completion word (XS_ENGINE_SPIN=0: the event only),
// for at most kSpinNs before falling back to a blocking event wait.
constexpr int64_t kSpinNs = 200000;
// Pure spinning only for about one fused batch's round trip; past it the poll yields the core
// between checks, so that waiters do not starve the callers' own threads when there are more
// runnable threads than cores (16 concurrent readers on a 16-core share).
static int64_t spin_pure_ns() {
  static const int64_t ns = [] {
    const char* v = getenv("XS_SPIN_PURE_US");
    return (v ? atoll(v) : 30) * 1000;
  }();
  return ns;
}
static bool spin_wait() {
  static const bool on = [] {
    const char* v = getenv("XS_ENGINE_SPIN");
    return v ? atoi(v) != 0 : true;
  }();
  return on;
}

// Zero-copy form of a combined batch (descriptors already in the pinned h_desc, offsets from
// the lowest caller input / output address): keygen reads the descriptors from host memory,
// the crypt kernels read the callers' inputs and write their outputs over PCIe, verdicts land
// in the pinned h_ok.  Two launches per direction run and one event -- no staging copies.
static int engine_issue_zero_copy(xs_engine::CSlot& c, const std::vector<uint64_t>& blk0, uint64_t nblk) {
  auto& batch = c.batch;
  hipStream_t st = c.s;
  uint64_t sbase = UINT64_MAX, dbase = UINT64_MAX, send = 0, dend = 0;
  for (const auto* q : batch) {
    sbase = std::min(sbase, q->d_in);
    dbase = std::min(dbase, q->d_out);
    send = std::max(send, q->d_in + q->in_len);
    dend = std::max(dend, q->d_out + q->out_len);
  }
  NonceArg bounds = bounds_arg(send - sbase, dend - dbase);
  bounds.n[4] = (uint32_t)(sbase & 15u);
  bounds.n[5] = (uint32_t)(dbase & 15u);
  const xs_block_desc* dd = (const xs_block_desc*)(uintptr_t)c.d_h_desc;
  uint64_t nseal = 0;
  hipError_t err = hipSuccess;
  bool one_run = true;  // every request of the batch has the same direction and key
  for (const auto* q : batch) one_run = one_run && q->seal == batch[0]->seal && !memcmp(q->key, batch[0]->key, 32);
  c.spin = false;
  if (one_run && nblk <= fused_max_blocks()) {  // tiny batch (a ranged read): one launch
    const bool seal = batch[0]->seal;
    c.seq++;
    err = launch_crypt_fused(seal, key_arg(batch[0]->key), bounds, dd, c.h_desc, nblk, (const uint8_t*)(uintptr_t)sbase,
                             (uint8_t*)(uintptr_t)dbase, seal ? nullptr : (uint8_t*)(uintptr_t)c.d_h_ok,
                             spin_wait() ? c.d_ctr : nullptr, (uint32_t*)(uintptr_t)c.d_h_flag, c.seq, st);
    c.spin = spin_wait();
    if (err != hipSuccess) return hip_fail(err, "zero-copy fused");
    return XS_OK;
  }
  for (size_t r = 0; r < batch.size();) {  // one keygen per run of (direction, key)
    size_t r1 = r + 1;
    while (r1 < batch.size() && batch[r1]->seal == batch[r]->seal && !memcmp(batch[r1]->key, batch[r]->key, 32)) r1++;
    const uint64_t b0 = blk0[r], b1 = r1 < batch.size() ? blk0[r1] : nblk;
    err = launch_keygen(batch[r]->seal ? 2 : 3, key_arg(batch[r]->key), bounds, 0, 0, b1 - b0, dd + b0, c.keys + b0, st);
    if (err != hipSuccess) return hip_fail(err, "zero-copy keygen");
    if (batch[r]->seal) nseal = b1;
    r = r1;
  }
  const uint8_t* src = (const uint8_t*)(uintptr_t)sbase;
  uint8_t* dst = (uint8_t*)(uintptr_t)dbase;
  if (nseal) {
    err = launch_crypt(true, c.keys, nseal, src, dst, nullptr, st);
    if (err != hipSuccess) return hip_fail(err, "zero-copy seal");
  }
  if (nblk > nseal) {
    err = launch_crypt(false, c.keys + nseal, nblk - nseal, src, dst, (uint8_t*)(uintptr_t)c.d_h_ok + nseal, st);
    if (err != hipSuccess) return hip_fail(err, "zero-copy open");
  }
  return XS_OK;
}

#ifdef XS_TEST_HOOKS
// TEST-ONLY failure injection (compiled into librclone_crypt_testhooks.so alone, rclone_amd/build.py):
// the first combined batch of at least g_fail_min requests issued after xs_test_fail_batch(min)
// fails before any launch, as a HIP error would; every request it carried must get XS_ERR_HIP.
static std::atomic<int> g_fail_min{0}, g_failed_reqs{0};
extern "C" void xs_test_fail_batch(int min_reqs) {
  g_failed_reqs = 0;
  g_fail_min = min_reqs;
}
extern "C" int xs_test_failed_requests(void) { return g_failed_reqs.load(); }
#endif

// Issue one combined batch on coalescing slot c (asynchronously).  The slot's stream carries only
// this batch, so the stream's completion is the batch's: no event is recorded (one runtime call
// less per batch; concurrent callers' launches serialise inside the runtime).
static int engine_issue_batch(xs_engine* e, xs_engine::CSlot& c) {
  auto& batch = c.batch;
#ifdef XS_TEST_HOOKS
  int want = g_fail_min.load();
  if (want > 0 && (int)batch.size() >= want && g_fail_min.compare_exchange_strong(want, 0)) {
    g_failed_reqs = (int)batch.size();
    set_error("test hook: injected failure of a combined batch of %zu requests", batch.size());
    return XS_ERR_HIP;
  }
#endif
  c.spin = false;  // only a fused zero-copy launch sets it
  if (hipSetDevice(e->device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
  // seal requests first, then open; inside a direction, requests with equal keys adjacent
  std::stable_sort(batch.begin(), batch.end(), [](const xs_engine::Req* a, const xs_engine::Req* b) {
    if (a->seal != b->seal) return a->seal;
    return memcmp(a->key, b->key, 32) < 0;
  });
  hipStream_t st = c.s;
  std::vector<uint64_t> blk0(batch.size()), inoff(batch.size()), outoff(batch.size());
  uint64_t nblk = 0, in_pos = 0, out_pos = 0;
  // zero-copy batch: every request's buffers are pinned; descriptors then hold offsets of the
  // caller buffers themselves from the lowest input / output address
  c.zc = true;
  uint64_t sbase = UINT64_MAX, dbase = UINT64_MAX;
  for (const auto* q : batch) {
    c.zc = c.zc && q->zc;
    sbase = std::min(sbase, q->d_in);
    dbase = std::min(dbase, q->d_out);
  }
  for (size_t r = 0; r < batch.size(); r++) {
    auto* q = batch[r];
    blk0[r] = nblk;
    q->blk0 = nblk;
    if (c.zc) {
      in_pos = q->d_in - sbase;
      out_pos = q->d_out - dbase;
    }
    inoff[r] = in_pos;
    outoff[r] = out_pos;
    for (uint64_t j = 0; j < q->nblocks; j++) {
      xs_block_desc& d = c.h_desc[nblk + j];
      d.reserved = q->seal ? 0u : open_window(q->range_lo, q->range_hi, j);
      nonce_plus(d.nonce, q->nonce0, q->first_block + j);
      if (q->seal) {
        d.src_off = in_pos + j * XS_BLOCK_DATA;
        d.dst_off = out_pos + j * XS_BLOCK_SIZE;
        const uint64_t rem = q->in_len - j * XS_BLOCK_DATA;
        d.len = (uint32_t)(rem < (uint64_t)XS_BLOCK_DATA ? rem : XS_BLOCK_DATA);
      } else {
        d.src_off = in_pos + j * XS_BLOCK_SIZE;
        d.dst_off = out_pos + j * XS_BLOCK_DATA;
        const uint64_t rem = q->in_len - j * XS_BLOCK_SIZE;
        d.len = (uint32_t)(rem < (uint64_t)XS_BLOCK_SIZE ? rem : XS_BLOCK_SIZE) - XS_BLOCK_HDR;
      }
    }
    nblk += q->nblocks;
    in_pos = (in_pos + q->in_len + 15) & ~15ull;
    out_pos = (out_pos + q->out_len + 15) & ~15ull;
  }
  if (c.zc) return engine_issue_zero_copy(c, blk0, nblk);
  hipError_t err = hipMemcpyAsync(c.desc, c.h_desc, nblk * sizeof(xs_block_desc), hipMemcpyHostToDevice, st);
  for (size_t r = 0; r < batch.size() && err == hipSuccess; r++)
    err = hipMemcpyAsync(c.in + inoff[r], batch[r]->in, batch[r]->in_len, hipMemcpyHostToDevice, st);
  if (err != hipSuccess) return hip_fail(err, "coalesced H2D");
  const NonceArg bounds = bounds_arg(e->c_cap_bytes, e->c_cap_bytes);
  const xs_block_desc* dd = (const xs_block_desc*)c.desc;
  uint64_t nseal = 0;
  for (size_t r = 0; r < batch.size();) {  // one keygen per run of (direction, key)
    size_t r1 = r + 1;
    while (r1 < batch.size() && batch[r1]->seal == batch[r]->seal && !memcmp(batch[r1]->key, batch[r]->key, 32)) r1++;
    const uint64_t b0 = blk0[r], b1 = r1 < batch.size() ? blk0[r1] : nblk;
    err = launch_keygen(batch[r]->seal ? 2 : 3, key_arg(batch[r]->key), bounds, 0, 0, b1 - b0, dd + b0, c.keys + b0, st);
    if (err != hipSuccess) return hip_fail(err, "coalesced keygen");
    if (batch[r]->seal) nseal = b1;
    r = r1;
  }
  if (nseal) {
    err = launch_crypt(true, c.keys, nseal, c.in, c.out, nullptr, st);
    if (err != hipSuccess) return hip_fail(err, "coalesced seal");
  }
  if (nblk > nseal) {
    err = launch_crypt(false, c.keys + nseal, nblk - nseal, c.in, c.out, c.ok + nseal, st);
    if (err != hipSuccess) return hip_fail(err, "coalesced open");
  }
  for (size_t r = 0; r < batch.size() && err == hipSuccess; r++) {
    err = hipMemcpyAsync(batch[r]->out, c.out + outoff[r], batch[r]->out_len, hipMemcpyDeviceToHost, st);
    if (err == hipSuccess && !batch[r]->seal)
      err = hipMemcpyAsync(batch[r]->ok, c.ok + blk0[r], batch[r]->nblocks, hipMemcpyDeviceToHost, st);
  }
  if (err != hipSuccess) return hip_fail(err, "coalesced D2H");
  return XS_OK;
}

// Wait for the combined batch in flight on c and hand its verdicts to the requests (zero-copy
// batches); c.rc carries the outcome.  A fused batch stores its completion word (after its
// outputs, system scope): poll it, falling back to the event if the stream ends (or fails)
// without it.
static void engine_wait_batch(xs_engine::CSlot& c) {
  if (c.rc == XS_OK) {
    bool seen = false;
    if (c.spin) {
      // bounded: a fused batch takes tens of microseconds; past kSpinNs (a busy GPU) the
      // waiter blocks on the event instead of burning a core
      const auto t0 = std::chrono::steady_clock::now();
      bool yielding = false;
      for (unsigned k = 1;; k++) {
        if (__atomic_load_n(c.h_flag, __ATOMIC_ACQUIRE) == c.seq) {
          seen = true;
          break;
        }
        if (yielding) std::this_thread::yield();
        else __builtin_ia32_pause();
        if ((k & 255u) == 0 || yielding) {
          if ((k & 15u) == 0 && hipStreamQuery(c.s) != hipErrorNotReady) break;
          const auto el = std::chrono::steady_clock::now() - t0;
          if (el > std::chrono::nanoseconds(kSpinNs)) break;
          yielding = el > std::chrono::nanoseconds(spin_pure_ns());
        }
      }
    }
    hipError_t err = seen ? hipSuccess : hipStreamSynchronize(c.s);
    if (err != hipSuccess) c.rc = hip_fail(err, "coalesced stream");
  } else {
    (void)hipStreamSynchronize(c.s);
  }
  if (c.rc == XS_OK && c.zc)
    for (auto* q : c.batch)
      if (!q->seal) memcpy(q->ok, c.h_ok + q->blk0, q->nblocks);
}

static int engine_submit(xs_engine* e, bool seal, const uint8_t key[32], const uint8_t nonce0[24], uint64_t first_block,
                         const void* in, uint64_t in_len, void* out, uint8_t* ok, uint64_t nblocks, uint64_t range_lo,
                         uint64_t range_hi) {
  xs_engine::Req req{};
  req.seal = seal;
  req.range_lo = range_lo;
  req.range_hi = range_hi;
  memcpy(req.key, key, 32);
  memcpy(req.nonce0, nonce0, 24);
  req.first_block = first_block;
  req.nblocks = nblocks;
  req.in = (const uint8_t*)in;
  req.in_len = in_len;
  req.out = (uint8_t*)out;
  req.out_len = seal ? in_len + nblocks * XS_BLOCK_HDR : in_len - nblocks * XS_BLOCK_HDR;
  req.ok = ok;
  req.rc = XS_OK;
  req.done = false;
  req.zc = e->zero_copy && host_dev_ptr(in, &req.d_in, e->device) && host_dev_ptr(out, &req.d_out, e->device) &&
           !(req.d_in & 15u) && !(req.d_out & 15u);
  if (!req.zc) req.d_in = req.d_out = 0;
  // Express lanes (XS_EXPRESS_LANES, default 2; XS_EXPRESS_MAX=0 turns them off): a small
  // request (a stream's first one-block refill, a ranged read) launches at once on a lane of its
  // own with a high-priority stream when one is free, instead of joining -- and waiting for --
  // the combined batches of large requests in the leader's ring.
  for (size_t x = 0; x < e->nexpress && nblocks <= e->express_max; x++) {
    const uint32_t bit = 1u << x;
    if (!(e->express_busy.fetch_or(bit, std::memory_order_acquire) & bit)) {
      auto& c = e->cslots[e->ncslots + x];
      c.batch.assign(1, &req);
      c.blocks = nblocks;
      c.rc = engine_issue_batch(e, c);
      engine_wait_batch(c);
      const int rc = c.rc;
      c.batch.clear();
      e->express_busy.fetch_and(~bit, std::memory_order_release);
      e->st_express.fetch_add(1, std::memory_order_relaxed);
      std::lock_guard<std::mutex> g(e->qmu);
      e->st_batches++;
      e->st_reqs++;
      e->st_blocks += nblocks;
      return rc;
    }
  }
  std::unique_lock<std::mutex> lk(e->qmu);
  e->queue.push_back(&req);
  e->qcount.store(e->queue.size(), std::memory_order_relaxed);
  while (!req.done) {
    if (e->leader) {
      (e->wake_all ? e->qcv : req.cv).wait(lk);
      continue;
    }
    // lead: keep up to nslots combined batches in flight until our own request is done and
    // nothing is in flight, then hand over
    e->leader = true;
    const size_t ns = e->ncslots;
    size_t head = 0, inflight = 0;  // ring of slots: [head, head + inflight) are in flight
    // move the queue's head requests (up to one batch) into the next free slot; qmu held
    auto take_batch = [&]() -> xs_engine::CSlot& {
      auto& c = e->cslots[(head + inflight) % ns];
      c.batch.clear();
      c.blocks = 0;
      if (e->one_run) {
        // one (direction, key) run per batch: a small batch then stays one fused launch instead
        // of keygen + crypt per direction; requests of the other run keep their queue order
        const xs_engine::Req* f = e->queue.front();
        size_t keep = 0;
        for (size_t i = 0; i < e->queue.size(); i++) {
          auto* q = e->queue[i];
          if (q->seal == f->seal && !memcmp(q->key, f->key, 32) && c.blocks + q->nblocks <= e->c_cap_blocks) {
            c.blocks += q->nblocks;
            c.batch.push_back(q);
          } else {
            e->queue[keep++] = q;
          }
        }
        e->queue.resize(keep);
      } else {
        size_t take = 0;
        while (take < e->queue.size() && c.blocks + e->queue[take]->nblocks <= e->c_cap_blocks)
          c.blocks += e->queue[take++]->nblocks;
        c.batch.assign(e->queue.begin(), e->queue.begin() + take);
        e->queue.erase(e->queue.begin(), e->queue.begin() + take);
      }
      e->qcount.store(e->queue.size(), std::memory_order_relaxed);
      return c;
    };
    while (!(req.done && inflight == 0)) {
      if (inflight < ns && !e->queue.empty() && !req.done) {
        auto& c = take_batch();
        lk.unlock();
        c.rc = engine_issue_batch(e, c);
        lk.lock();
        inflight++;
        continue;
      }
      if (inflight == 0) break;  // nothing queued for us (own request already done)
      auto& c = e->cslots[head];
      lk.unlock();
      if (e->overlap) {
        // wait for the head batch, but put requests that arrive meanwhile into free slots at once
        // (they would otherwise wait for the head's whole round trip before being issued)
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned k = 1; c.rc == XS_OK; k++) {
          if (c.spin && __atomic_load_n(c.h_flag, __ATOMIC_ACQUIRE) == c.seq) break;
          if (inflight < ns && !req.done && e->qcount.load(std::memory_order_relaxed) != 0) {
            lk.lock();
            if (!e->queue.empty()) {
              auto& n = take_batch();
              lk.unlock();
              n.rc = engine_issue_batch(e, n);
              inflight++;
            } else {
              lk.unlock();
            }
            continue;
          }
          __builtin_ia32_pause();
          if ((k & 255u) == 0) {
            if (hipStreamQuery(c.s) != hipErrorNotReady) break;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(kSpinNs)) break;
          }
        }
      }
      engine_wait_batch(c);
      lk.lock();
      for (auto* q : c.batch) {
        q->rc = c.rc;
        q->done = true;
        if (!e->wake_all) q->cv.notify_one();  // under qmu: the waiter cannot return (and its request vanish) first
      }
      e->st_batches++;
      e->st_reqs += c.batch.size();
      e->st_blocks += c.blocks;
      c.batch.clear();
      head = (head + 1) % ns;
      inflight--;
      if (e->wake_all) e->qcv.notify_all();
    }
    e->leader = false;
    if (e->wake_all) e->qcv.notify_all();
    else if (!e->queue.empty()) e->queue.front()->cv.notify_one();  // it takes over the lead
  }
  return req.rc;
}

// ---------------------------------------------------------------- seal + MD5 (cryptcheck)
static NonceArg bounds_arg(uint64_t src_len, uint64_t dst_len) {  // descriptor-mode keygen bounds
  NonceArg b{};
  b.n[0] = (uint32_t)src_len; b.n[1] = (uint32_t)(src_len >> 32);
  b.n[2] = (uint32_t)dst_len; b.n[3] = (uint32_t)(dst_len >> 32);
  return b;  // hipMalloc buffers: base alignment bits 0
}

static void nonce_add_host(uint8_t n[24], uint64_t x) {  // nonce.add (cipher.go:665-678)
  uint64_t carry = 0;
  for (int i = 0; i < 8; i++) {
    const uint64_t sum = (uint64_t)n[i] + (uint8_t)(x >> (8 * i)) + carry;
    n[i] = (uint8_t)sum;
    carry = sum >> 8;
  }
  for (int i = 8; i < 24 && carry; i++) {
    const uint64_t sum = (uint64_t)n[i] + carry;
    n[i] = (uint8_t)sum;
    carry = sum >> 8;
  }
}

static uint64_t body_bytes(uint64_t plain_len) {
  const uint64_t nb = (plain_len + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
  return plain_len + nb * XS_BLOCK_HDR;
}

// ---- host MD5 for long objects
// MD5 is one dependency chain per stream, so the GPU kernel runs one lane per object at
// ~70 MB/s; one host core does ~0.5-1 GB/s.  A group of objects lasts as long as
// its longest GPU lane, so the longest objects of a group are hashed on the host instead, over
// the wire body the GPU sealed (crypt.put's tee hash, crypt.go:516-533, is the same bytes), by a
// small worker pool that keeps running while the next group goes through the GPU.
static double lane_md5_bps() {
  static const double v = [] {
    const char* e = getenv("XS_MD5_LANE_BPS");
    return e ? atof(e) : 70e6;
  }();
  return v;
}

// One host core's MD5 rate, measured once (8 MiB, a few ms).
static double host_md5_bps() {
  static const double v = [] {
    if (const char* e = getenv("XS_MD5_HOST_BPS")) return atof(e);
    std::vector<uint8_t> b((size_t)8 << 20, 0x5a);
    uint8_t out[16];
    const auto t0 = std::chrono::steady_clock::now();
    HostMd5 m;
    m.update(b.data(), b.size());
    m.final(out);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return s > 0 ? (double)b.size() / s : 500e6;
  }();
  return v;
}

static int host_md5_threads_default() {
  if (const char* e = getenv("XS_MD5_HOST_THREADS")) return std::max(0, atoi(e));
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(8u, hc ? hc / 2 : 1u));
}

// Below this an object stays on its GPU lane: a 16 MiB lane takes ~0.24 s, longer than a 4 GiB
// group's PCIe copies; shorter objects finish within the group's own copy time, and hashing them on
// host cores only competes with the file reads feeding the next group (configs[4]'s 4 KiB-8 MiB
// tree measured no gain, profiles/r02/e2e_routing_ab.jsonl).
constexpr uint64_t kHostMd5Min = 16ull << 20;

// Which objects of a group go to the host (route[k] = 1): take the longest first while the host
// pool's makespan stays below that object's GPU lane time, i.e. while moving it shortens the
// group (the group's GPU MD5 time is then set by the longest object left on the GPU).
static void route_host_md5(const uint64_t* wire_len, size_t n, int threads, std::vector<uint8_t>& route) {
  route.assign(n, 0);
  if (threads <= 0 || n == 0) return;
  std::vector<size_t> order;
  for (size_t k = 0; k < n; k++)
    if (wire_len[k] >= kHostMd5Min) order.push_back(k);
  if (order.empty()) return;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return wire_len[a] > wire_len[b]; });
  const double hb = host_md5_bps(), lb = lane_md5_bps();
  double sum = 0, mx = 0;
  for (size_t k : order) {
    const double L = (double)wire_len[k];
    const double nsum = sum + L, nmx = std::max(mx, L);
    const double host_t = std::max(nmx, nsum / threads) / hb;
    if (host_t >= L / lb) break;
    route[k] = 1;
    sum = nsum;
    mx = nmx;
  }
}

namespace {
struct HostMd5Pool {
  struct Job {
    uint8_t prefix[32];
    const uint8_t* body;
    uint64_t len;
    uint8_t* out;
    int tag;  // staging buffer the body sits in (-1: the caller's body buffer)
  };
  std::mutex mu;
  std::condition_variable cv, idle;
  std::vector<Job> jobs;
  size_t next = 0;
  bool closing = false;
  std::vector<std::thread> th;
  uint64_t bytes = 0, count = 0;
  int pending[2] = {0, 0};  // unfinished jobs per staging buffer
  int node = -1;            // the engine's NUMA node: workers run on its CPUs

  void push(const Job& j, int max_threads) {
    std::lock_guard<std::mutex> g(mu);
    bytes += j.len;
    count++;
    if (j.tag >= 0) pending[j.tag]++;
    jobs.push_back(j);
    if ((int)th.size() < max_threads && th.size() < jobs.size() - next)
      th.emplace_back([this] {
        pin_thread_to_node(node);
        work();
      });
    cv.notify_one();
  }
  void work() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return next < jobs.size() || closing; });
      if (next >= jobs.size()) return;
      const Job j = jobs[next++];
      lk.unlock();
      HostMd5 m;
      m.update(j.prefix, 32);
      m.update(j.body, j.len);
      m.final(j.out);
      lk.lock();
      if (j.tag >= 0 && --pending[j.tag] == 0) idle.notify_all();
    }
  }
  // every job reading staging buffer `tag` is done (it may be overwritten)
  void wait_tag(int tag) {
    std::unique_lock<std::mutex> lk(mu);
    idle.wait(lk, [&] { return pending[tag] == 0; });
  }
  void finish() {
    {
      std::lock_guard<std::mutex> g(mu);
      closing = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
    th.clear();
  }
  ~HostMd5Pool() { finish(); }
};
}  // namespace

// Seal + MD5 of whole objects in groups of ~budget plaintext bytes; with `body` the wire
// bodies also come back (packed: object i at xs_put_body_offset of i, one D2H per group).
// host_threads > 0 lets the longest objects of a group be hashed on the host (route_host_md5).
static int seal_md5_impl(xs_engine* e, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                         const uint64_t* offs, const uint64_t* lens, const void* plain, uint8_t* md5,
                         uint8_t* body, int host_threads, uint64_t* host_routed) {
  if (host_routed) *host_routed = 0;
  if (nobj == 0) return XS_OK;
  if (!e || !key || !nonces || !offs || !lens || !md5) {
    set_error("xs_engine_seal_md5: null argument");
    return XS_ERR_INVALID;
  }
  for (uint64_t i = 0; i < nobj; i++) {
    if ((offs[i] & 15u) || (lens[i] && !plain)) {
      set_error("xs_engine_seal_md5: object %llu: plaintext offset must be 16-byte aligned",
                (unsigned long long)i);
      return XS_ERR_INVALID;
    }
  }
  static const uint8_t magic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};
  std::lock_guard<std::mutex> g(e->mu);
  if (hipSetDevice(e->device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
  hipStream_t st = e->slots[0].s;
  auto& hb = e->hb;
  HostMd5Pool host;  // joined (every digest written) before this function returns
  host.node = e->numa;
  // groups of whole objects, ~budget plaintext bytes each (MD5 is sequential per object)
  // large groups: the MD5 of a group takes as long as its largest object (one lane each)
  const uint64_t budget = std::max<uint64_t>((uint64_t)e->batch * XS_BLOCK_DATA * 16, 4096ull << 20);
  std::vector<xs_block_desc> desc;
  std::vector<xs_md5_desc> mdesc;
  std::vector<uint64_t> wlen, gpu_obj, host_obj;
  std::vector<uint8_t> route, dig;
  uint64_t o0 = 0, body_pos = 0;
  for (uint64_t group = 0; o0 < nobj; group++) {
    uint64_t o1 = o0, lo = UINT64_MAX, hi = 0, bsum = 0, nblk = 0;
    while (o1 < nobj) {
      const uint64_t nlo = std::min(lo, offs[o1]), nhi = std::max(hi, offs[o1] + lens[o1]);
      if (o1 > o0 && nhi - nlo > budget) break;
      lo = nlo;
      hi = nhi;
      bsum += (body_bytes(lens[o1]) + 15) & ~15ull;
      nblk += (lens[o1] + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
      o1++;
    }
    const uint64_t span = hi > lo ? hi - lo : 0, ng = o1 - o0;
    wlen.resize(ng);
    for (uint64_t i = o0; i < o1; i++) wlen[i - o0] = body_bytes(lens[i]);
    route_host_md5(wlen.data(), ng, host_threads, route);
    desc.clear();
    mdesc.clear();
    gpu_obj.clear();
    host_obj.clear();
    uint64_t w = 0;
    std::vector<uint64_t> wpos(ng);
    for (uint64_t i = o0; i < o1; i++) {
      const uint64_t nb = (lens[i] + XS_BLOCK_DATA - 1) / XS_BLOCK_DATA;
      wpos[i - o0] = w;
      if (route[i - o0]) {
        host_obj.push_back(i);
      } else {
        xs_md5_desc m{};
        m.off = w;
        m.len = wlen[i - o0];
        memcpy(m.prefix, magic, 8);
        memcpy(m.prefix + 8, nonces + 24 * i, 24);
        m.prefix_len = 32;
        mdesc.push_back(m);
        gpu_obj.push_back(i);
      }
      for (uint64_t j = 0; j < nb; j++) {
        xs_block_desc d{};
        d.src_off = offs[i] - lo + j * XS_BLOCK_DATA;
        d.dst_off = w + j * XS_BLOCK_SIZE;
        const uint64_t rem = lens[i] - j * XS_BLOCK_DATA;
        d.len = (uint32_t)(rem < (uint64_t)XS_BLOCK_DATA ? rem : XS_BLOCK_DATA);
        memcpy(d.nonce, nonces + 24 * i, 24);
        nonce_add_host(d.nonce, j);
        desc.push_back(d);
      }
      w += (wlen[i - o0] + 15) & ~15ull;
    }
    const uint64_t ngpu = mdesc.size();
    if (!grow(&hb.d_plain, &hb.plain_cap, span) || !grow(&hb.d_body, &hb.body_cap, bsum) ||
        !grow(&hb.d_desc, &hb.desc_cap, nblk * sizeof(xs_block_desc)) ||
        !grow(&hb.d_mdesc, &hb.mdesc_cap, std::max<uint64_t>(ngpu, 1) * sizeof(xs_md5_desc)) ||
        !grow(&hb.d_digest, &hb.digest_cap, std::max<uint64_t>(ngpu, 1) * 16) ||
        !grow((uint8_t**)&hb.d_keys, &hb.keys_cap, nblk * sizeof(BlockKey))) {
      set_error("xs_engine_seal_md5: device allocation failed");
      return XS_ERR_HIP;
    }
    hipError_t err = hipSuccess;
    if (span) err = hipMemcpyAsync(hb.d_plain, (const uint8_t*)plain + lo, span, hipMemcpyHostToDevice, st);
    if (err == hipSuccess && nblk)
      err = hipMemcpyAsync(hb.d_desc, desc.data(), nblk * sizeof(xs_block_desc), hipMemcpyHostToDevice, st);
    if (err == hipSuccess && ngpu)
      err = hipMemcpyAsync(hb.d_mdesc, mdesc.data(), ngpu * sizeof(xs_md5_desc), hipMemcpyHostToDevice, st);
    if (err != hipSuccess) return hip_fail(err, "H2D");
    if (nblk) {
      err = launch_keygen(2, key_arg(key), bounds_arg(span, bsum), 0, 0, nblk, (const xs_block_desc*)hb.d_desc,
                          hb.d_keys, st);
      if (err != hipSuccess) return hip_fail(err, "keygen");
      err = launch_crypt(true, hb.d_keys, nblk, hb.d_plain, hb.d_body, nullptr, st);
      if (err != hipSuccess) return hip_fail(err, "seal");
    }
    // the wire bodies (all of them for put_batch, the host-routed ones otherwise) leave on the
    // aux stream while the MD5 lanes run on st; the host pool starts as soon as they have landed
    hipStream_t ax = hb.aux;
    if (err == hipSuccess) err = hipEventRecord(hb.ev_sealed, st);
    if (err == hipSuccess) err = hipStreamWaitEvent(ax, hb.ev_sealed, 0);
    // without caller bodies (cryptcheck) the routed bodies land in one of two pinned staging
    // buffers, alternating by group, so the host can still be hashing group g while g+1 lands
    const int tag = (int)(group & 1);
    std::vector<uint64_t> spos(host_obj.size());
    if (!body && !host_obj.empty()) {
      uint64_t need = 0;
      for (size_t k = 0; k < host_obj.size(); k++) {
        spos[k] = need;
        need += wlen[host_obj[k] - o0];
      }
      host.wait_tag(tag);
      if (!grow_pinned(&hb.route[tag], &hb.route_cap[tag], need, e->numa)) {
        set_error("xs_engine_seal_md5: pinned staging of %llu bytes failed", (unsigned long long)need);
        return XS_ERR_NOMEM;
      }
      for (size_t k = 0; k < host_obj.size() && err == hipSuccess; k++) {
        const uint64_t i = host_obj[k], len = wlen[i - o0];
        if (len) err = hipMemcpyAsync(hb.route[tag] + spos[k], hb.d_body + wpos[i - o0], len, hipMemcpyDeviceToHost, ax);
      }
    } else if (body && w && err == hipSuccess) {
      err = hipMemcpyAsync(body + body_pos, hb.d_body, w, hipMemcpyDeviceToHost, ax);
    }
    if (err != hipSuccess) return hip_fail(err, "D2H");
    if (ngpu) {
      err = launch_md5((const xs_md5_desc*)hb.d_mdesc, ngpu, hb.d_body, bsum, hb.d_digest, nullptr, st);
      if (err != hipSuccess) return hip_fail(err, "md5");
      dig.resize(16 * ngpu);
      err = hipMemcpyAsync(dig.data(), hb.d_digest, ngpu * 16, hipMemcpyDeviceToHost, st);
      if (err != hipSuccess) return hip_fail(err, "D2H");
    }
    err = hipStreamSynchronize(ax);
    if (err != hipSuccess) return hip_fail(err, "engine aux stream");
    for (size_t k = 0; k < host_obj.size(); k++) {
      const uint64_t i = host_obj[k];
      HostMd5Pool::Job j;
      memcpy(j.prefix, magic, 8);
      memcpy(j.prefix + 8, nonces + 24 * i, 24);
      j.body = body ? body + body_pos + wpos[i - o0] : hb.route[tag] + spos[k];
      j.len = wlen[i - o0];
      j.out = md5 + 16 * i;
      j.tag = body ? -1 : tag;
      host.push(j, host_threads);
    }
    // the host-side descriptor vectors are reused next group: wait for this group's copies
    err = hipStreamSynchronize(st);
    if (err != hipSuccess) return hip_fail(err, "engine stream");
    for (uint64_t k = 0; k < ngpu; k++) memcpy(md5 + 16 * gpu_obj[k], dig.data() + 16 * k, 16);
    body_pos += w;
    o0 = o1;
  }
  host.finish();
  if (host_routed) *host_routed = host.count;
  e->st_host_md5_objs += host.count;
  e->st_host_md5_bytes += host.bytes;
  e->st_md5_objs += nobj;
  return XS_OK;
}

extern "C" int xs_engine_seal_md5(xs_engine* e, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                                  const uint64_t* offs, const uint64_t* lens, const void* plain, uint8_t* md5) {
  if (!e) {
    set_error("xs_engine_seal_md5: null engine");
    return XS_ERR_INVALID;
  }
  return seal_md5_impl(e, key, nobj, nonces, offs, lens, plain, md5, nullptr,
                       e->host_md5_threads >= 0 ? e->host_md5_threads : host_md5_threads_default(), nullptr);
}

extern "C" uint64_t xs_put_body_bytes(uint64_t nobj, const uint64_t* lens) {
  uint64_t w = 0;
  for (uint64_t i = 0; i < nobj; i++) w += (body_bytes(lens[i]) + 15) & ~15ull;
  return w;
}

extern "C" int xs_engine_put_batch(xs_engine* e, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                                   const uint64_t* offs, const uint64_t* lens, const void* plain, void* body,
                                   uint8_t* md5) {
  if (nobj && !body) {
    set_error("xs_engine_put_batch: null body");
    return XS_ERR_INVALID;
  }
  if (!e) {
    set_error("xs_engine_put_batch: null engine");
    return XS_ERR_INVALID;
  }
  return seal_md5_impl(e, key, nobj, nonces, offs, lens, plain, md5, (uint8_t*)body,
                       e->host_md5_threads >= 0 ? e->host_md5_threads : host_md5_threads_default(), nullptr);
}

extern "C" void xs_engine_set_host_md5(xs_engine* e, int threads) {
  if (e) e->host_md5_threads = threads;
}

extern "C" void xs_engine_md5_stats(xs_engine* e, uint64_t out[3]) {
  if (!e || !out) return;
  out[0] = e->st_host_md5_objs.load();
  out[1] = e->st_host_md5_bytes.load();
  out[2] = e->st_md5_objs.load();
}

// ---------------------------------------------------------------- multi-device engine pool
// One rclone process runs many transfers and checkers at once (fs/sync/sync.go:544
// startTransfers, --transfers / --checkers); objects are independent, so a process spreads them
// over every GPU of the node: object streams take engines round-robin (xs_pool_next), batched
// put / cryptcheck calls split their objects into contiguous byte-balanced ranges, one per
// engine, run concurrently.  Several engines may sit on one device (a list like "0,0,0,0").
namespace xs {
std::vector<int> default_devices() {
  std::vector<int> v;
  const char* list = getenv("RCLONE_AMD_DEVICES");
  if (list && *list && parse_device_list(list, &v) > 0) return v;
  if (const char* one = getenv("RCLONE_AMD_DEVICE")) {
    v.assign(1, atoi(one));
    return v;
  }
  const int n = xs_device_count();
  // one process per GPU (torch.distributed.run and the like export LOCAL_RANK): that rank's
  // device only, not engines (~170 MB + 5 streams each) on every GPU from every rank
  if (const char* lr = getenv("LOCAL_RANK")) {
    if (*lr && n > 0) {
      v.assign(1, atoi(lr) % n);
      return v;
    }
  }
  for (int d = 0; d < n; d++) v.push_back(d);
  return v;
}
}  // namespace xs

struct xs_pool {
  std::vector<xs_engine*> engines;
  std::atomic<uint64_t> rr{0};
};

extern "C" xs_pool* xs_pool_create(const int* devices, int ndevices, uint32_t batch_blocks, int nslots) {
  std::vector<int> devs;
  if (devices && ndevices > 0) devs.assign(devices, devices + ndevices);
  else devs = default_devices();
  if (devs.empty()) {
    set_error("xs_pool_create: no HIP device");
    return nullptr;
  }
  xs_pool* p = new xs_pool();
  for (int d : devs) {
    xs_engine* e = xs_engine_create(d, batch_blocks, nslots);
    if (!e) {
      const std::string msg = xs_last_error();
      for (auto* x : p->engines) xs_engine_destroy(x);
      delete p;
      set_error("xs_pool_create: %s", msg.c_str());
      return nullptr;
    }
    p->engines.push_back(e);
  }
  return p;
}

extern "C" void xs_pool_destroy(xs_pool* p) {
  if (!p) return;
  for (auto* e : p->engines) xs_engine_destroy(e);
  delete p;
}

extern "C" int xs_pool_size(const xs_pool* p) { return p ? (int)p->engines.size() : 0; }

extern "C" xs_engine* xs_pool_engine(xs_pool* p, int i) {
  if (!p || i < 0 || i >= (int)p->engines.size()) return nullptr;
  return p->engines[i];
}

extern "C" xs_engine* xs_pool_next(xs_pool* p) {
  if (!p || p->engines.empty()) return nullptr;
  return p->engines[p->rr.fetch_add(1) % p->engines.size()];
}

// Objects [0, nobj) split into k contiguous ranges of about equal plaintext bytes, one engine
// each, run on their own threads; the first failure's message is passed to the caller's thread.
static int pool_seal_md5(xs_pool* p, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                         const uint64_t* offs, const uint64_t* lens, const void* plain, uint8_t* md5, uint8_t* body) {
  if (!p || p->engines.empty()) {
    set_error("xs_pool: no engines");
    return XS_ERR_INVALID;
  }
  if (nobj == 0) return XS_OK;
  if (!key || !nonces || !offs || !lens || !md5) {
    set_error("xs_pool_seal_md5: null argument");
    return XS_ERR_INVALID;
  }
  const uint64_t k = std::min<uint64_t>(p->engines.size(), nobj);
  uint64_t total = 0;
  for (uint64_t i = 0; i < nobj; i++) total += lens[i] + 1;  // +1: empty objects still count
  std::vector<uint64_t> cut{0};
  uint64_t acc = 0;
  for (uint64_t i = 0; i < nobj && cut.size() < k; i++) {
    acc += lens[i] + 1;
    if (acc * k >= total * cut.size() && i + 1 < nobj) cut.push_back(i + 1);
  }
  cut.push_back(nobj);
  const int ht = host_md5_threads_default();
  const int per = ht > 0 ? std::max(1, ht / (int)(cut.size() - 1)) : 0;
  std::vector<int> rc(cut.size() - 1, XS_OK);
  std::vector<std::string> msg(cut.size() - 1);
  std::vector<std::thread> th;
  uint64_t bpos = 0;
  const uint64_t first = p->rr.fetch_add(cut.size() - 1);  // distinct engines for the ranges
  for (size_t r = 0; r + 1 < cut.size(); r++) {
    const uint64_t a = cut[r], b = cut[r + 1];
    uint8_t* rb = body ? body + bpos : nullptr;
    for (uint64_t i = a; i < b; i++) bpos += (body_bytes(lens[i]) + 15) & ~15ull;
    xs_engine* e = p->engines[(first + r) % p->engines.size()];
    th.emplace_back([&, r, a, b, rb, e] {
      pin_thread_to_node(e->numa);
      rc[r] = seal_md5_impl(e, key, b - a, nonces + 24 * a, offs + a, lens + a, plain, md5 + 16 * a, rb,
                            e->host_md5_threads >= 0 ? e->host_md5_threads : per, nullptr);
      if (rc[r] != XS_OK) msg[r] = xs_last_error();
    });
  }
  for (auto& t : th) t.join();
  for (size_t r = 0; r < rc.size(); r++)
    if (rc[r] != XS_OK) {
      set_error("%s", msg[r].c_str());
      return rc[r];
    }
  return XS_OK;
}

extern "C" int xs_pool_seal_md5(xs_pool* p, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                                const uint64_t* offs, const uint64_t* lens, const void* plain, uint8_t* md5) {
  return pool_seal_md5(p, key, nobj, nonces, offs, lens, plain, md5, nullptr);
}

extern "C" int xs_pool_put_batch(xs_pool* p, const uint8_t key[32], uint64_t nobj, const uint8_t* nonces,
                                 const uint64_t* offs, const uint64_t* lens, const void* plain, void* body,
                                 uint8_t* md5) {
  if (nobj && !body) {
    set_error("xs_pool_put_batch: null body");
    return XS_ERR_INVALID;
  }
  return pool_seal_md5(p, key, nobj, nonces, offs, lens, plain, md5, (uint8_t*)body);
}
