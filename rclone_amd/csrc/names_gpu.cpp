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

struct EmeDev {
  std::mutex mu;
  bool init = false, failed = false;
  int device = 0;
  hipStream_t s = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint8_t* d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t* h_buf = nullptr;  // pinned
  size_t h_cap = 0;
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
  if (hipSetDevice(e.device) != hipSuccess || hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e.ev0) != hipSuccess || hipEventCreate(&e.ev1) != hipSuccess) {
    xs::set_error("name engine: no HIP device %d", e.device);
    e.failed = true;
    return false;
  }
  e.init = true;
  return true;
}

bool ne_reserve(EmeDev& e, size_t bytes) {
  if (bytes <= e.d_cap && bytes <= e.h_cap) return true;
  size_t cap = e.d_cap ? e.d_cap : (1u << 20);
  while (cap < bytes) cap *= 2;
  if (e.d_buf) (void)hipFree(e.d_buf);
  if (e.h_buf) (void)hipHostFree(e.h_buf);
  e.d_buf = e.h_buf = nullptr;
  e.d_cap = e.h_cap = 0;
  if (hipMalloc(&e.d_buf, cap) != hipSuccess || hipHostMalloc(&e.h_buf, cap, hipHostMallocPortable) != hipSuccess) {
    xs::set_error("name engine: cannot allocate %zu bytes", cap);
    return false;
  }
  e.d_cap = e.h_cap = cap;
  return true;
}

}  // namespace

EmeDev* eme_acquire(size_t bytes, uint8_t** host) {
  EmeDev& e = name_engine();
  e.mu.lock();
  if (!ne_init(e) || hipSetDevice(e.device) != hipSuccess || !ne_reserve(e, bytes)) {
    e.mu.unlock();
    return nullptr;
  }
  *host = e.h_buf;
  return &e;
}

int32_t eme_run(EmeDev* dev, bool encrypt, const rc_cipher* c, size_t desc_off, size_t ndesc, size_t data_bytes,
                size_t total, double* ms) {
  EmeDev& e = *dev;
  hipError_t err = hipMemcpyAsync(e.d_buf, e.h_buf, total, hipMemcpyHostToDevice, e.s);
  if (err == hipSuccess) err = hipEventRecord(e.ev0, e.s);
  if (err == hipSuccess)
    err = xs::launch_eme(encrypt, c->eme, (const xs_name_desc*)(e.d_buf + desc_off), ndesc, e.d_buf, e.d_buf,
                         data_bytes, e.s);
  if (err == hipSuccess) err = hipEventRecord(e.ev1, e.s);
  if (err == hipSuccess) err = hipMemcpyAsync(e.h_buf, e.d_buf, data_bytes, hipMemcpyDeviceToHost, e.s);
  if (err == hipSuccess) err = hipStreamSynchronize(e.s);
  if (err != hipSuccess) {
    xs::set_error("name engine: %s", hipGetErrorString(err));
    return RC_ERR_GPU;
  }
  float f = 0;
  if (hipEventElapsedTime(&f, e.ev0, e.ev1) == hipSuccess) *ms = f;
  return RC_NIL;
}

void eme_release(EmeDev* dev) { dev->mu.unlock(); }

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
