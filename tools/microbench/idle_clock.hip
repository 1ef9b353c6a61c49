// Shader clock and fixed costs of a tiny one-wave kernel launched the way a ranged read does
// (launch, wait, some host work, repeat) -- the regime of xs_keygen_wide / xs_crypt_fused.
// The kernel runs a chain of N dependent integer VALU ops and records s_memtime (shader clock)
// and s_memrealtime (100 MHz) at entry and exit, then stores a completion word to pinned host
// memory; the host records launch -> completion word (spin) and launch -> hipStreamSynchronize.
// Diagnostic tool.   usage: idle_clock [reps] [gap_us]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(64) chain(unsigned n, unsigned* out, unsigned long long* t, unsigned* flag,
                                           unsigned seq) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned x = threadIdx.x + 1u, y = x * 3u;
  for (unsigned i = 0; i < n; i++) {  // 4 dependent VALU ops per iteration
    x = __builtin_amdgcn_alignbit(x, x, 7) ^ y;
    y = y + x;
    x = x + (y >> 3);
    y = y ^ (x << 5);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[threadIdx.x] = x ^ y;  // keep the chain alive
  if (threadIdx.x == 0) {
    t[0] = c1 - c0;
    t[1] = r1 - r0;
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // completion word in pinned memory
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 400;
  const int gap_us = argc > 2 ? atoi(argv[2]) : 20;
  unsigned* d_out;
  unsigned long long* t;  // pinned, written by the kernel
  if (hipMalloc(&d_out, 64 * sizeof(unsigned)) != hipSuccess) return 1;
  if (hipHostMalloc(&t, 2 * sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess) return 1;
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
  printf("{\"tool\": \"idle_clock\", \"gap_us\": %d, \"reps\": %d, \"runs\": [", gap_us, reps);
  const unsigned ns[] = {0u, 250u, 1000u, 4000u};
  for (int k = 0; k < 4; k++) {
    const unsigned n = ns[k];
    std::vector<double> ghz, kern_us, wall_us, flag_us;
    for (int r = 0; r < reps; r++) {
      const auto w0 = std::chrono::steady_clock::now();
      ++seq;
      hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, s, n, d_out, d_t, d_flag, seq);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
      }
      const auto wf = std::chrono::steady_clock::now();
      if (hipStreamSynchronize(s) != hipSuccess) return 2;
      const auto w1 = std::chrono::steady_clock::now();
      const double cyc = (double)t[0], us = (double)t[1] * 0.01;
      if (r >= 10) {
        kern_us.push_back(us);
        if (us > 0) ghz.push_back(cyc / (us * 1e3));
        wall_us.push_back(std::chrono::duration<double, std::micro>(w1 - w0).count());
        flag_us.push_back(std::chrono::duration<double, std::micro>(wf - w0).count());
      }
      const auto g0 = std::chrono::steady_clock::now();  // host work between reads
      while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count() < gap_us) {
      }
    }
    printf("%s{\"valu_ops\": %u, \"in_kernel_us_p50\": %.2f, \"shader_ghz_p50\": %.3f, \"launch_to_sync_us_p50\": %.2f, \"launch_to_flag_us_p50\": %.2f,"
           " \"ns_per_dependent_op\": %.3f}",
           k ? ", " : "", 4 * n, median(kern_us), median(ghz), median(wall_us), median(flag_us),
           n ? median(kern_us) * 1e3 / (4.0 * n) : 0.0);
  }
  printf("]}\n");
  (void)hipStreamDestroy(s);
  (void)hipHostFree(t);
  (void)hipHostFree(flag);
  (void)hipFree(d_out);
  return 0;
}
