// names_gpu.cpp -- the GPU half of the file-name cipher (names.cpp holds the host half): one
// name engine per device (stream, pinned staging, device buffer), the batched EME-AES-256 launch
// over every segment of an rc_names_run batch (xs_eme.hip), and the device-resident primitive
// xs_eme_batch_dev.  Reference: encryptSegment / decryptSegment, backend/crypt/cipher.go:264-312
// (eme.Transform, github.com/rfjakob/eme v1.2.0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "rc_internal.h"
#include "xs_internal.h"

namespace xs {
hipError_t launch_eme(bool encrypt, const aes::EmeKey& key, const xs_name_desc* desc, uint64_t n, const uint8_t* src,
                      uint8_t* dst, uint64_t buf_len, hipStream_t stream);
}

namespace rcn {

struct EmeSlot {
  uint8_t* d = nullptr;  // device
  uint8_t* h = nullptr;  // pinned
  size_t cap = 0;
  hipEvent_t k0 = nullptr, k1 = nullptr;  // around the slot's kernel
  hipEvent_t done = nullptr;              // after its D2H
  bool pending = false;
};

struct EmeDev {
  std::mutex mu;
  bool init = false, failed = false;
  int device = 0;
  hipStream_t s = nullptr;
  EmeSlot slot[2];
};

namespace {

// One name engine per device of the process's device list; concurrent rc_names_run calls take
// them round-robin (a listing is one batch, so batches -- not names -- are spread over GPUs).
struct NameEngines {
  std::once_flag once;
  std::vector<std::unique_ptr<EmeDev>> v;
  std::atomic<uint64_t> rr{0};
};
NameEngines g_names;

EmeDev& name_engine() {
  std::call_once(g_names.once, [] {
    std::vector<int> devs = xs::default_devices();
    std::sort(devs.begin(), devs.end());
    devs.erase(std::unique(devs.begin(), devs.end()), devs.end());
    if (devs.empty()) devs.push_back(0);  // ne_init reports the missing device
    for (int d : devs) {
      g_names.v.emplace_back(new EmeDev());
      g_names.v.back()->device = d;
    }
  });
  return *g_names.v[g_names.rr.fetch_add(1) % g_names.v.size()];
}

bool ne_init(EmeDev& e) {
  if (e.init) return true;
  if (e.failed) return false;
  bool ok = hipSetDevice(e.device) == hipSuccess && hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking) == hipSuccess;
  for (auto& sl : e.slot)
    ok = ok && hipEventCreate(&sl.k0) == hipSuccess && hipEventCreate(&sl.k1) == hipSuccess &&
         hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    xs::set_error("name engine: no HIP device %d", e.device);
    e.failed = true;
    return false;
  }
  e.init = true;
  return true;
}

}  // namespace

EmeDev* eme_open() {
  EmeDev& e = name_engine();
  e.mu.lock();
  if (!ne_init(e) || hipSetDevice(e.device) != hipSuccess) {
    e.mu.unlock();
    return nullptr;
  }
  return &e;
}

uint8_t* eme_slot(EmeDev* dev, int s, size_t bytes) {
  EmeSlot& sl = dev->slot[s];
  if (bytes <= sl.cap) return sl.h;
  size_t cap = sl.cap ? sl.cap : (1u << 20);
  while (cap < bytes) cap *= 2;
  if (sl.d) (void)hipFree(sl.d);
  if (sl.h) (void)hipHostFree(sl.h);
  sl.d = sl.h = nullptr;
  sl.cap = 0;
  if (hipMalloc(&sl.d, cap) != hipSuccess || hipHostMalloc(&sl.h, cap, hipHostMallocPortable) != hipSuccess) {
    xs::set_error("name engine: cannot allocate %zu bytes", cap);
    return nullptr;
  }
  sl.cap = cap;
  return sl.h;
}

int32_t eme_issue(EmeDev* dev, int s, bool encrypt, const rc_cipher* c, size_t desc_off, size_t ndesc,
                  size_t data_bytes, size_t total) {
  EmeDev& e = *dev;
  EmeSlot& sl = e.slot[s];
  hipError_t err = hipMemcpyAsync(sl.d, sl.h, total, hipMemcpyHostToDevice, e.s);
  if (err == hipSuccess) err = hipEventRecord(sl.k0, e.s);
  if (err == hipSuccess)
    err = xs::launch_eme(encrypt, c->eme, (const xs_name_desc*)(sl.d + desc_off), ndesc, sl.d, sl.d, data_bytes, e.s);
  if (err == hipSuccess) err = hipEventRecord(sl.k1, e.s);
  if (err == hipSuccess) err = hipMemcpyAsync(sl.h, sl.d, data_bytes, hipMemcpyDeviceToHost, e.s);
  if (err == hipSuccess) err = hipEventRecord(sl.done, e.s);
  sl.pending = true;  // waited for even after a failed issue: earlier work may be queued
  if (err != hipSuccess) {
    xs::set_error("name engine: %s", hipGetErrorString(err));
    return RC_ERR_GPU;
  }
  return RC_NIL;
}

int32_t eme_wait(EmeDev* dev, int s, double* ms) {
  EmeDev& e = *dev;
  EmeSlot& sl = e.slot[s];
  if (!sl.pending) return RC_NIL;
  sl.pending = false;
  hipError_t err = hipEventSynchronize(sl.done);
  if (err != hipSuccess) err = hipStreamSynchronize(e.s);
  if (err != hipSuccess) {
    xs::set_error("name engine: %s", hipGetErrorString(err));
    return RC_ERR_GPU;
  }
  float f = 0;
  if (hipEventElapsedTime(&f, sl.k0, sl.k1) == hipSuccess) *ms += f;
  return RC_NIL;
}

void eme_release(EmeDev* dev) {
  for (int s = 0; s < 2; s++) {
    double ms = 0;
    (void)eme_wait(dev, s, &ms);  // nothing may still write a slot once another call owns it
  }
  dev->mu.unlock();
}

}  // namespace rcn

extern "C" int xs_eme_batch_dev(int encrypt, const uint8_t name_key[32], const uint8_t tweak[16],
                                const xs_name_desc* d_desc, uint64_t n, const void* d_src, void* d_dst,
                                uint64_t buf_len, void* stream) {
  if (!name_key || !tweak || (n && (!d_desc || !d_src || !d_dst))) {
    xs::set_error("xs_eme_batch_dev: null argument");
    return XS_ERR_INVALID;
  }
  xs::aes::EmeKey k;
  xs::aes::expand_key(name_key, tweak, &k);
  hipError_t e = xs::launch_eme(encrypt != 0, k, d_desc, n, (const uint8_t*)d_src, (uint8_t*)d_dst, buf_len,
                                (hipStream_t)stream);
  if (e != hipSuccess) {
    xs::set_error("eme launch: %s", hipGetErrorString(e));
    return XS_ERR_HIP;
  }
  return XS_OK;
}
