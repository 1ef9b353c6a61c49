// Does a cold instruction cache slow a one-wave Salsa20 core?  The fused ranged-read kernel runs
// each piece of straight-line code once per launch (HSalsa20, then keystream block 0 through a
// second inlined copy of the same rounds), and its phase marks show ~2.8 us per core against
// ~1.4 us of issue.  This kernel runs the deferred-XOR rounds of xs_salsa_lazy.h in one wave:
// three passes through the same loop code (the first fetches it, the next two find it cached),
// then one pass through a second inlined copy.  Launched like a read: launch, spin on a pinned
// completion word, 20 us of host work, repeat.  The same is then timed (wave 0's passes) with
// company in the workgroup, as in the fused kernel: waves 4..7 polling an LDS flag, waves 1..3
// computing too, all eight computing.  Diagnostic tool.
//   usage: icache_probe [reps] [gap_us]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../rclone_amd/csrc/xs_salsa_lazy.h"

__device__ __forceinline__ uint32_t as_varying(uint32_t x) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(x));
  return v;
}

__device__ __forceinline__ void rounds(uint32_t (&x)[16]) {
  uint32_t t[16];
  xs_salsa_dr_lazy_enter(x, t);
#pragma unroll 1
  for (int i = 0; i < 9; i++) xs_salsa_dr_lazy(x, t);
#pragma unroll
  for (int i = 0; i < 16; i++)
    if ((XS_LAZY_MASK >> i) & 1u) x[i] ^= t[i];
}

// t[0..4]: s_memrealtime after each pass; out keeps the state alive
// mode 0: waves >= 1 exit at once; 1: waves 1..3 exit, 4..7 poll an LDS flag (s_sleep 1) until
// wave 0 is done; 2: waves 1..3 compute, 4..7 poll; 3: all waves compute
__global__ void __launch_bounds__(512) probe(const uint32_t* in, uint32_t* out, unsigned long long* t, unsigned* flag,
                                            unsigned seq, int mode) {
  __shared__ uint32_t done;
  const unsigned l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  const bool compute = w == 0 || (mode == 2 && w < 4) || mode == 3;
  if (!compute) {
    if (mode == 0 || w < 4) return;
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    const uint32_t fa = (uint32_t)(uintptr_t)(const lds_u32*)&done;  // the LDS offset, as the fused kernel polls
    for (;;) {
      uint32_t f;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(f) : "v"(fa) : "memory");
      if (__builtin_amdgcn_readfirstlane(f) != 0u) return;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = as_varying(in[i]);
  unsigned long long m[5];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  m[0] = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int it = 0; it < 3; it++) {
    rounds(x);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    if (it == 0) m[1] = r;
    else if (it == 1) m[2] = r;
    else m[3] = r;
  }
  rounds(x);  // a second inlined copy of the same rounds
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  m[4] = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= x[i];
  out[64 * w + l] = acc;
  if (w != 0) return;
  __hip_atomic_store(&done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (l < 5u) {
    unsigned long long v = m[0];
#pragma unroll
    for (int i = 1; i < 5; i++) v = l == (unsigned)i ? m[i] : v;
    t[l] = v;  // lane-indexed vector stores
  }
  __threadfence_system();
  if (l == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 400;
  const int gap_us = argc > 2 ? atoi(argv[2]) : 20;
  uint32_t *d_in, *d_out;
  if (hipMalloc(&d_in, 16 * sizeof(uint32_t)) != hipSuccess) return 1;
  if (hipMalloc(&d_out, 512 * sizeof(uint32_t)) != hipSuccess) return 1;
  uint32_t h_in[16];
  for (int i = 0; i < 16; i++) h_in[i] = 0x9e3779b9u * (uint32_t)(i + 1);
  if (hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice) != hipSuccess) return 1;
  unsigned long long* t;
  if (hipHostMalloc(&t, 8 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  unsigned long long* d_t;
  if (hipHostGetDevicePointer((void**)&d_t, t, 0) != hipSuccess) return 1;
  unsigned* flag;
  if (hipHostMalloc(&flag, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  unsigned* d_flag;
  if (hipHostGetDevicePointer((void**)&d_flag, flag, 0) != hipSuccess) return 1;
  *flag = 0;
  unsigned seq = 0;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  printf("{\"tool\": \"icache_probe\", \"reps\": %d, \"gap_us\": %d, \"wave0_us_p50\": [", reps, gap_us);
  const int modes[] = {0, 1, 2, 3};
  const char* names[] = {"alone", "4 waves polling", "4 computing + 4 polling", "8 computing"};
  for (int mi = 0; mi < 4; mi++) {
  const int mode = modes[mi];
  std::vector<double> p[4];
  for (int r = 0; r < reps; r++) {
    ++seq;
    hipLaunchKernelGGL(probe, dim3(1), dim3(mode == 0 ? 64 : 512), 0, s, d_in, d_out, d_t, d_flag, seq, mode);
    const auto w0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() > 5.0) {
        fprintf(stderr, "completion word never arrived\n");
        return 3;
      }
    }
    if (hipStreamSynchronize(s) != hipSuccess) return 2;
    if (r >= 10)
      for (int i = 0; i < 4; i++) p[i].push_back((double)(t[i + 1] - t[i]) * 0.01);
    const auto g0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count() < gap_us) {
    }
  }
  printf("%s{\"company\": \"%s\", \"pass1\": %.2f, \"pass2_same_code\": %.2f, \"pass3_same_code\": %.2f, \"second_copy\": %.2f}",
         mi ? ", " : "", names[mi], median(p[0]), median(p[1]), median(p[2]), median(p[3]));
  }
  printf("]}\n");
  (void)hipStreamDestroy(s);
  (void)hipHostFree(t);
  (void)hipHostFree(flag);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  return 0;
}
