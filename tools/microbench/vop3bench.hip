// Issue cost of 3-source VOP3 integer ops on gfx950 (v_xad_u32, v_bitop3_b32) vs 2-source
// ops, with source VGPRs in distinct or identical banks (bank = index mod 4).  Each kernel
// runs REPS x 64 independent instructions (explicit registers, 8 rotating destinations);
// grid = W waves per SIMD on every SIMD.  Prints shader cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define REPS 400
#define R8(x) x x x x x x x x
#define KERNEL(name, ins)                                                                          \
  __global__ void __launch_bounds__(64) name(unsigned long long* cyc, uint32_t* out) {           \
    asm volatile("v_mov_b32 v1, 1\n v_mov_b32 v2, 2\n v_mov_b32 v3, 3\n v_mov_b32 v5, 5\n"     \
                 "v_mov_b32 v9, 9\n v_mov_b32 v13, 13\n v_mov_b32 v6, 6\n v_mov_b32 v7, 7\n" ::  \
                     : "v1", "v2", "v3", "v5", "v6", "v7", "v9", "v13");                         \
    unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();  \
    for (int r = 0; r < REPS; r++) asm volatile(R8(ins) ::: "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23"); \
    unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    if (threadIdx.x == 0) { cyc[2 * blockIdx.x] = c1 - c0; cyc[2 * blockIdx.x + 1] = r1 - r0; }     \
  }
// 8 instructions per macro arg, R8 -> 64 per rep
KERNEL(k_add, "v_add_u32 v16, v1, v2\n v_add_u32 v17, v1, v2\n v_add_u32 v18, v1, v2\n v_add_u32 v19, v1, v2\n v_add_u32 v20, v1, v2\n v_add_u32 v21, v1, v2\n v_add_u32 v22, v1, v2\n v_add_u32 v23, v1, v2\n")
KERNEL(k_align, "v_alignbit_b32 v16, v1, v1, 25\n v_alignbit_b32 v17, v2, v2, 25\n v_alignbit_b32 v18, v1, v1, 25\n v_alignbit_b32 v19, v2, v2, 25\n v_alignbit_b32 v20, v1, v1, 25\n v_alignbit_b32 v21, v2, v2, 25\n v_alignbit_b32 v22, v1, v1, 25\n v_alignbit_b32 v23, v2, v2, 25\n")
KERNEL(k_xad_diff, "v_xad_u32 v16, v1, v2, v3\n v_xad_u32 v17, v1, v2, v3\n v_xad_u32 v18, v1, v2, v3\n v_xad_u32 v19, v1, v2, v3\n v_xad_u32 v20, v1, v2, v3\n v_xad_u32 v21, v1, v2, v3\n v_xad_u32 v22, v1, v2, v3\n v_xad_u32 v23, v1, v2, v3\n")
KERNEL(k_xad_same, "v_xad_u32 v16, v1, v5, v9\n v_xad_u32 v17, v1, v5, v9\n v_xad_u32 v18, v1, v5, v9\n v_xad_u32 v19, v1, v5, v9\n v_xad_u32 v20, v1, v5, v9\n v_xad_u32 v21, v1, v5, v9\n v_xad_u32 v22, v1, v5, v9\n v_xad_u32 v23, v1, v5, v9\n")
KERNEL(k_b3_diff, "v_bitop3_b32 v16, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v17, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v18, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v19, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v20, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v21, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v22, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v23, v1, v2, v3 bitop3:0x96\n")
KERNEL(k_b3_same, "v_bitop3_b32 v16, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v17, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v18, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v19, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v20, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v21, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v22, v1, v5, v9 bitop3:0x96\n v_bitop3_b32 v23, v1, v5, v9 bitop3:0x96\n")
KERNEL(k_add_same, "v_add_u32 v16, v1, v5\n v_add_u32 v17, v1, v5\n v_add_u32 v18, v1, v5\n v_add_u32 v19, v1, v5\n v_add_u32 v20, v1, v5\n v_add_u32 v21, v1, v5\n v_add_u32 v22, v1, v5\n v_add_u32 v23, v1, v5\n")
KERNEL(k_mix, "v_xad_u32 v16, v1, v2, v3\n v_alignbit_b32 v17, v6, v6, 25\n v_bitop3_b32 v18, v5, v6, v7 bitop3:0x96\n v_add_u32 v19, v1, v2\n v_xad_u32 v20, v13, v6, v3\n v_alignbit_b32 v21, v7, v7, 23\n v_bitop3_b32 v22, v1, v6, v3 bitop3:0x96\n v_xor_b32 v23, v1, v2\n")

int main() {
  unsigned long long* cyc;
  uint32_t* out;
  (void)hipMalloc(&cyc, 2 * 65536 * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipMalloc(&out, 4096);
  struct K { const char* n; void (*f)(unsigned long long*, uint32_t*); } ks[] = {
      {"v_add (2 src)", k_add}, {"v_add same bank", k_add_same}, {"v_alignbit", k_align},
      {"v_xad diff banks", k_xad_diff}, {"v_xad same bank", k_xad_same}, {"v_bitop3 diff banks", k_b3_diff},
      {"v_bitop3 same bank", k_b3_same}, {"mix", k_mix}};
  for (int W : {1, 2, 4, 8}) {
    const int nwg = 1024 * W;
    for (auto& k : ks) {
      for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k.f, dim3(nwg), dim3(64), 0, 0, cyc, out);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(nwg), dim3(64), 0, 0, cyc, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> h(2 * nwg);
      (void)hipMemcpy(h.data(), cyc, 2 * nwg * 8, hipMemcpyDeviceToHost);
      double sc = 0, sr = 0;
      for (int i = 0; i < nwg; i++) { sc += h[2 * i]; sr += h[2 * i + 1]; }
      const double ghz = sc / sr * 0.1;  // s_memrealtime ticks at 100 MHz
      // SIMD cycles per wave-instruction from the kernel time: time * clock * SIMDs / instructions
      const double simd_cpi = ms * 1e-3 * ghz * 1e9 * 1024.0 / ((double)nwg * REPS * 64.0);
      printf("W=%d %-20s per-wave %.2f cyc/inst | kernel %.3f ms  clock %.2f GHz  SIMD %.2f cyc per wave-inst\n", W,
             k.n, sc / nwg / (REPS * 64.0), ms, ghz, simd_cpi);
    }
  }
  return 0;
}
