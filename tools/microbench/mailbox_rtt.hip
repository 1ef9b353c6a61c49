// Ranged-read dispatch latency (diagnostic): what a persistent reader
// kernel polling a pinned mailbox would save against one launch per read.
//
//   launch : hipLaunchKernelGGL of a one-wave kernel that stores a sequence number into pinned
//            host memory (system scope) as its first action; host time call -> word visible.
//   mailbox: one persistent wave polls a mailbox word in pinned host memory (system-scope loads,
//            optional s_sleep between polls); the host writes seq i (release) and times until the
//            wave's answer word reads i.  With --desc the wave also reads a 768-byte descriptor
//            area of the mailbox after seeing the word (what a reader needs per request), and
//            answers with a checksum of it.
// The persistent wave exits on seq 0xFFFFFFFF or after 0.5 s without a request (s_memrealtime),
// so it always drains.  Medians over --reps.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/mailbox_rtt.hip -o tools/microbench/mailbox_rtt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void word_kernel(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave; mbox[0] = request seq, mbox[16..16+192) = descriptor words; flag[0] = answered seq,
// flag[1] = checksum of the descriptor words of that request
__global__ void mailbox_kernel(const uint32_t* mbox, uint32_t* flag, int sleep_mode, int read_desc) {
  const uint32_t l = threadIdx.x;
  uint32_t last = 0;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t s = __hip_atomic_load(mbox, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s != last) {
      last = s;
      if (s == 0xFFFFFFFFu) break;
      uint32_t sum = 0;
      if (read_desc) {  // 768 bytes: three words per lane, one load each
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
          v += __hip_atomic_load(mbox + 16 + 64 * k + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
        sum = v;
      }
      if (l == 0) {
        __hip_atomic_store(flag + 1, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(flag, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      t_last = __builtin_amdgcn_s_memrealtime();
      continue;
    }
    if (__builtin_amdgcn_s_memrealtime() - t_last > 50000000ull) break;  // 0.5 s idle (100 MHz)
    if (sleep_mode == 1) __builtin_amdgcn_s_sleep(1);
    else if (sleep_mode == 2) __builtin_amdgcn_s_sleep(16);
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
  int reps = 5000;
  for (int i = 1; i < argc; i++)
    if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
  uint32_t *flag = nullptr, *mbox = nullptr;
  if (hipHostMalloc(&flag, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostMalloc(&mbox, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    fprintf(stderr, "pinned alloc failed\n");
    return 1;
  }
  memset(flag, 0, 64);
  memset(mbox, 0, 4096);
  uint32_t *dflag = nullptr, *dmbox = nullptr;
  (void)hipHostGetDevicePointer((void**)&dflag, flag, 0);
  (void)hipHostGetDevicePointer((void**)&dmbox, mbox, 0);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);

  // launch -> word
  std::vector<double> t;
  uint32_t seq = 0;
  for (int r = 0; r < reps + 100; r++) {
    seq++;
    const double t0 = now_us();
    hipLaunchKernelGGL(word_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    const double t1 = now_us();
    if (r >= 100) t.push_back(t1 - t0);
  }
  (void)hipStreamSynchronize(s);
  printf("{\"mode\": \"launch\", \"p50_us\": %.3f, \"p90_us\": %.3f, \"reps\": %d}\n", median(t), pct(t, 0.9), reps);

  for (int read_desc = 0; read_desc < 2; read_desc++) {
    for (int sleep_mode = 0; sleep_mode < 3; sleep_mode++) {
      memset(flag, 0, 64);
      __atomic_store_n(mbox, 0u, __ATOMIC_RELEASE);
      for (int i = 0; i < 192; i++) mbox[16 + i] = (uint32_t)i;
      hipLaunchKernelGGL(mailbox_kernel, dim3(1), dim3(64), 0, s, (const uint32_t*)dmbox, dflag, sleep_mode, read_desc);
      // let the wave start polling
      const double w0 = now_us();
      while (now_us() - w0 < 2000) __builtin_ia32_pause();
      t.clear();
      bool ok = true;
      for (uint32_t r = 1; r <= (uint32_t)reps + 100; r++) {
        mbox[16] = r;  // descriptor content changes per request (the checksum must follow it)
        const double t0 = now_us();
        __atomic_store_n(mbox, r, __ATOMIC_RELEASE);
        const double lim = t0 + 100000.0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != r) {
          __builtin_ia32_pause();
          if (now_us() > lim) {
            ok = false;
            break;
          }
        }
        const double t1 = now_us();
        if (!ok) break;
        if (read_desc) {
          const uint32_t want = r + (191u * 192u / 2u) - 0u;  // sum of 1..191 plus r in word 0
          if (__atomic_load_n(flag + 1, __ATOMIC_ACQUIRE) != want) ok = false;
        }
        if (r > 100) t.push_back(t1 - t0);
      }
      __atomic_store_n(mbox, 0xFFFFFFFFu, __ATOMIC_RELEASE);
      (void)hipStreamSynchronize(s);
      if (!ok || t.empty()) {
        printf("{\"mode\": \"mailbox\", \"sleep\": %d, \"desc\": %d, \"ok\": false}\n", sleep_mode, read_desc);
        continue;
      }
      printf("{\"mode\": \"mailbox\", \"sleep\": %d, \"desc\": %d, \"p50_us\": %.3f, \"p90_us\": %.3f, \"reps\": %d, \"ok\": true}\n",
             sleep_mode, read_desc, median(t), pct(t, 0.9), reps);
    }
  }
  (void)hipStreamDestroy(s);
  (void)hipHostFree(flag);
  (void)hipHostFree(mbox);
  return 0;
}
