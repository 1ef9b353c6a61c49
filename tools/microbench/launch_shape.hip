// Ranged-read dispatch overheads by launch shape (diagnostic): host launch ->
// completion word for kernels that only store the word, as the fused kernel's completion does
// (every wave fences at system scope, a barrier, thread 0 stores seq with a system-scope release):
//   64 threads; 576 threads (nine waves, the fused kernel's shape); 576 threads + 156 KB of LDS
//   (the fused kernel's); the same + a 1 KB kernel argument block (its inline descriptors).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/launch_shape.hip -o tools/microbench/launch_shape
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

struct Big {
  uint32_t w[256];
};
static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <int LDS_WORDS>
__global__ void shape_kernel(uint32_t* flag, uint32_t seq, Big big) {
  if (LDS_WORDS > 0) {
    __shared__ uint32_t lds[LDS_WORDS > 0 ? LDS_WORDS : 1];
    lds[threadIdx.x] = big.w[threadIdx.x & 255u];  // touch it so it is allocated
    __syncthreads();
    if (lds[(threadIdx.x + 1) % blockDim.x] == 0xFFFFFFFFu) flag[1] = 1;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t *flag = nullptr, *dflag = nullptr;
  if (hipHostMalloc(&flag, 64, hipHostMallocMapped) != hipSuccess) return 1;
  (void)hipHostGetDevicePointer((void**)&dflag, flag, 0);
  memset(flag, 0, 64);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  Big big{};
  const char* names[4] = {"64 threads", "576 threads", "576 threads + 156 KB LDS", "576 threads + 156 KB LDS + 1 KB args"};
  uint32_t seq = 0;
  for (int shape = 0; shape < 4; shape++) {
    std::vector<double> t;
    for (int r = 0; r < reps + 100; r++) {
      seq++;
      const double t0 = now_us();
      if (shape == 0) hipLaunchKernelGGL(shape_kernel<0>, dim3(1), dim3(64), 0, s, dflag, seq, Big{});
      else if (shape == 1) hipLaunchKernelGGL(shape_kernel<0>, dim3(1), dim3(576), 0, s, dflag, seq, Big{});
      else if (shape == 2) hipLaunchKernelGGL(shape_kernel<39936>, dim3(1), dim3(576), 0, s, dflag, seq, Big{});
      else hipLaunchKernelGGL(shape_kernel<39936>, dim3(1), dim3(576), 0, s, dflag, seq, big);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
      const double t1 = now_us();
      (void)hipStreamSynchronize(s);
      if (r >= 100) t.push_back(t1 - t0);
    }
    std::sort(t.begin(), t.end());
    printf("{\"shape\": \"%s\", \"launch_to_word_p50_us\": %.2f, \"p10\": %.2f, \"p90\": %.2f, \"reps\": %d}\n", names[shape],
           t[t.size() / 2], t[t.size() / 10], t[9 * t.size() / 10], reps);
  }
  return 0;
}
