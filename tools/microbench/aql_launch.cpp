// Launch latency: hipLaunchKernel vs a direct AQL dispatch on an HSA queue (diagnostic).
// One wave stores a sequence number into pinned host memory (system scope) as its first action;
// the host times call -> word visible, median over REPS, for both paths.  The HSA path loads the
// same kernel from a code object built by
//   hipcc --offload-arch=gfx950 --genco -O3 tools/microbench/aql_kernel.hip -o aql_kernel.hsaco, then
//   clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=aql_kernel.hsaco
//     --output=tools/microbench/aql_kernel.co (the raw gfx950 ELF)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/aql_launch.cpp tools/microbench/aql_kernel.hip
//        -o tools/microbench/aql_launch -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

__global__ void aql_word(uint32_t* flag, uint32_t seq);  // tools/microbench/aql_kernel.hip

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Found {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
  hsa_amd_memory_pool_t kernarg{};
  bool have_kernarg = false;
};

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  Found* f = (Found*)data;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) {
    f->gpu = a;
    f->have_gpu = true;
  }
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
    f->cpu = a;
    f->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* data) {
  Found* f = (Found*)data;
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !f->have_kernarg) {
    f->kernarg = p;
    f->have_kernarg = true;
  }
  return HSA_STATUS_SUCCESS;
}

#define CK(x)                                                      \
  do {                                                             \
    hsa_status_t s_ = (x);                                         \
    if (s_ != HSA_STATUS_SUCCESS) {                                \
      fprintf(stderr, "%s failed: %d (line %d)\n", #x, (int)s_, __LINE__); \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  const char* hsaco = argc > 2 ? argv[2] : "tools/microbench/aql_kernel.co";
  uint32_t* flag = nullptr;
  if (hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  memset(flag, 0, 64);
  uint32_t* dflag = nullptr;
  hipHostGetDevicePointer((void**)&dflag, flag, 0);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  // ---- HIP path
  std::vector<double> hip_us;
  uint32_t seq = 0;
  for (int r = 0; r < reps + 50; r++) {
    seq++;
    const double t0 = now_us();
    hipLaunchKernelGGL(aql_word, dim3(1), dim3(64), 0, st, dflag, seq);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    const double t1 = now_us();
    if (r >= 50) hip_us.push_back(t1 - t0);
    hipStreamSynchronize(st);
  }
  // ---- HSA path: same kernel from its code object, packet written straight into a queue
  CK(hsa_init());
  Found f;
  CK(hsa_iterate_agents(agent_cb, &f));
  if (!f.have_gpu || !f.have_cpu) return 2;
  CK(hsa_amd_agent_iterate_memory_pools(f.cpu, pool_cb, &f));
  if (!f.have_kernarg) return 3;
  std::ifstream in(hsaco, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    fprintf(stderr, "no code object %s\n", hsaco);
    return 4;
  }
  hsa_code_object_reader_t reader;
  CK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader));
  hsa_executable_t exe;
  CK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  CK(hsa_executable_load_agent_code_object(exe, f.gpu, reader, nullptr, nullptr));
  CK(hsa_executable_freeze(exe, nullptr));
  hsa_executable_symbol_t sym;
  CK(hsa_executable_get_symbol_by_name(exe, "_Z8aql_wordPjj.kd", &f.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t kargsz = 0, grp = 0, priv = 0;
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargsz));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &grp));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv));
  hsa_queue_t* q = nullptr;
  CK(hsa_queue_create(f.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  void* karg = nullptr;
  CK(hsa_amd_memory_pool_allocate(f.kernarg, std::max<uint32_t>(kargsz, 64) * 64, 0, &karg));
  CK(hsa_amd_agents_allow_access(1, &f.gpu, nullptr, karg));
  std::vector<double> aql_us;
  for (int r = 0; r < reps + 50; r++) {
    seq++;
    const double t0 = now_us();
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    uint8_t* ka = (uint8_t*)karg + (idx % 64) * std::max<uint32_t>(kargsz, 64);
    memset(ka, 0, kargsz);
    memcpy(ka, &dflag, 8);
    memcpy(ka + 8, &seq, 4);
    hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx % q->size);
    p->workgroup_size_x = 64;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->grid_size_x = 64;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = priv;
    p->group_segment_size = grp;
    p->kernel_object = kobj;
    p->kernarg_address = ka;
    p->completion_signal.handle = 0;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n((uint32_t*)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    const double t1 = now_us();
    if (r >= 50) aql_us.push_back(t1 - t0);
    // the packet slot is reusable once the queue's read index passed it (one in flight here)
    while (hsa_queue_load_read_index_scacquire(q) <= idx) __builtin_ia32_pause();
  }
  std::sort(hip_us.begin(), hip_us.end());
  std::sort(aql_us.begin(), aql_us.end());
  auto pct = [](const std::vector<double>& v, double p) { return v[std::min(v.size() - 1, (size_t)(p * v.size()))]; };
  printf("{\"tool\": \"aql_launch\", \"reps\": %d, \"hip_launch_to_word_us\": {\"p10\": %.2f, \"p50\": %.2f, \"p90\": %.2f}, "
         "\"aql_dispatch_to_word_us\": {\"p10\": %.2f, \"p50\": %.2f, \"p90\": %.2f}, \"kernarg_bytes\": %u}\n",
         reps, pct(hip_us, 0.1), pct(hip_us, 0.5), pct(hip_us, 0.9), pct(aql_us, 0.1), pct(aql_us, 0.5), pct(aql_us, 0.9),
         kargsz);
  hsa_queue_destroy(q);
  hsa_amd_memory_pool_free(karg);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(reader);
  return 0;
}
