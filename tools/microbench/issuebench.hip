// Issue-rate probe with in-kernel s_memtime, verified results.  One 64-thread workgroup per
// wave; grid = W * 1024 waves (W waves per SIMD on 256 CUs).  Body: Salsa20 column half-round
// (exact register pattern), 48 VALU instructions, repeated REPS times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define REPS 2000

__global__ void __launch_bounds__(64) k(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = seed * (i + 1) + threadIdx.x;
  uint32_t t0, t1, t2, t3;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll 1
  for (int r = 0; r < REPS; r++) {
    asm volatile(
        "v_add_u32 %16, %0, %12\n v_add_u32 %17, %5, %1\n v_add_u32 %18, %10, %6\n v_add_u32 %19, %15, %11\n"
        "v_alignbit_b32 %16, %16, %16, 25\n v_alignbit_b32 %17, %17, %17, 25\n v_alignbit_b32 %18, %18, %18, 25\n v_alignbit_b32 %19, %19, %19, 25\n"
        "v_xor_b32 %4, %4, %16\n v_xor_b32 %9, %9, %17\n v_xor_b32 %14, %14, %18\n v_xor_b32 %3, %3, %19\n"
        "v_add_u32 %16, %4, %0\n v_add_u32 %17, %9, %5\n v_add_u32 %18, %14, %10\n v_add_u32 %19, %3, %15\n"
        "v_alignbit_b32 %16, %16, %16, 23\n v_alignbit_b32 %17, %17, %17, 23\n v_alignbit_b32 %18, %18, %18, 23\n v_alignbit_b32 %19, %19, %19, 23\n"
        "v_xor_b32 %8, %8, %16\n v_xor_b32 %13, %13, %17\n v_xor_b32 %2, %2, %18\n v_xor_b32 %7, %7, %19\n"
        "v_add_u32 %16, %8, %4\n v_add_u32 %17, %13, %9\n v_add_u32 %18, %2, %14\n v_add_u32 %19, %7, %3\n"
        "v_alignbit_b32 %16, %16, %16, 19\n v_alignbit_b32 %17, %17, %17, 19\n v_alignbit_b32 %18, %18, %18, 19\n v_alignbit_b32 %19, %19, %19, 19\n"
        "v_xor_b32 %12, %12, %16\n v_xor_b32 %1, %1, %17\n v_xor_b32 %6, %6, %18\n v_xor_b32 %11, %11, %19\n"
        "v_add_u32 %16, %12, %8\n v_add_u32 %17, %1, %13\n v_add_u32 %18, %6, %2\n v_add_u32 %19, %11, %7\n"
        "v_alignbit_b32 %16, %16, %16, 14\n v_alignbit_b32 %17, %17, %17, 14\n v_alignbit_b32 %18, %18, %18, 14\n v_alignbit_b32 %19, %19, %19, 14\n"
        "v_xor_b32 %0, %0, %16\n v_xor_b32 %5, %5, %17\n v_xor_b32 %10, %10, %18\n v_xor_b32 %15, %15, %19\n"
        : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
          "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3));
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime();
  uint32_t a = 0;
  for (int i = 0; i < 16; i++) a = a * 31 + x[i];
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

__global__ void __launch_bounds__(64) k_e64(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = seed * (i + 1) + threadIdx.x;
  uint32_t t0, t1, t2, t3;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll 1
  for (int r = 0; r < REPS; r++) {
    asm volatile(
        "v_add_u32_e64 %16, %0, %12\n v_add_u32_e64 %17, %5, %1\n v_add_u32_e64 %18, %10, %6\n v_add_u32_e64 %19, %15, %11\n"
        "v_alignbit_b32 %16, %16, %16, 25\n v_alignbit_b32 %17, %17, %17, 25\n v_alignbit_b32 %18, %18, %18, 25\n v_alignbit_b32 %19, %19, %19, 25\n"
        "v_xor_b32_e64 %4, %4, %16\n v_xor_b32_e64 %9, %9, %17\n v_xor_b32_e64 %14, %14, %18\n v_xor_b32_e64 %3, %3, %19\n"
        "v_add_u32_e64 %16, %4, %0\n v_add_u32_e64 %17, %9, %5\n v_add_u32_e64 %18, %14, %10\n v_add_u32_e64 %19, %3, %15\n"
        "v_alignbit_b32 %16, %16, %16, 23\n v_alignbit_b32 %17, %17, %17, 23\n v_alignbit_b32 %18, %18, %18, 23\n v_alignbit_b32 %19, %19, %19, 23\n"
        "v_xor_b32_e64 %8, %8, %16\n v_xor_b32_e64 %13, %13, %17\n v_xor_b32_e64 %2, %2, %18\n v_xor_b32_e64 %7, %7, %19\n"
        "v_add_u32_e64 %16, %8, %4\n v_add_u32_e64 %17, %13, %9\n v_add_u32_e64 %18, %2, %14\n v_add_u32_e64 %19, %7, %3\n"
        "v_alignbit_b32 %16, %16, %16, 19\n v_alignbit_b32 %17, %17, %17, 19\n v_alignbit_b32 %18, %18, %18, 19\n v_alignbit_b32 %19, %19, %19, 19\n"
        "v_xor_b32_e64 %12, %12, %16\n v_xor_b32_e64 %1, %1, %17\n v_xor_b32_e64 %6, %6, %18\n v_xor_b32_e64 %11, %11, %19\n"
        "v_add_u32_e64 %16, %12, %8\n v_add_u32_e64 %17, %1, %13\n v_add_u32_e64 %18, %6, %2\n v_add_u32_e64 %19, %11, %7\n"
        "v_alignbit_b32 %16, %16, %16, 14\n v_alignbit_b32 %17, %17, %17, 14\n v_alignbit_b32 %18, %18, %18, 14\n v_alignbit_b32 %19, %19, %19, 14\n"
        "v_xor_b32_e64 %0, %0, %16\n v_xor_b32_e64 %5, %5, %17\n v_xor_b32_e64 %10, %10, %18\n v_xor_b32_e64 %15, %15, %19\n"
        : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
          "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3));
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime();
  uint32_t a = 0;
  for (int i = 0; i < 16; i++) a = a * 31 + x[i];
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}


__global__ void __launch_bounds__(64) k8(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t x[16], y[16];
  for (int i = 0; i < 16; i++) { x[i] = seed * (i + 1) + threadIdx.x; y[i] = seed * (i + 7) + threadIdx.x; }
  uint32_t t0, t1, t2, t3, u0, u1, u2, u3;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll 1
  for (int r = 0; r < REPS / 2; r++) {
    asm volatile(
        "v_add_u32 %16, %0, %12\n v_add_u32 %17, %5, %1\n v_add_u32 %18, %10, %6\n v_add_u32 %19, %15, %11\n"
        "v_add_u32 %36, %20, %32\n v_add_u32 %37, %25, %21\n v_add_u32 %38, %30, %26\n v_add_u32 %39, %35, %31\n"
        "v_alignbit_b32 %16, %16, %16, 25\n v_alignbit_b32 %17, %17, %17, 25\n v_alignbit_b32 %18, %18, %18, 25\n v_alignbit_b32 %19, %19, %19, 25\n"
        "v_alignbit_b32 %36, %36, %36, 25\n v_alignbit_b32 %37, %37, %37, 25\n v_alignbit_b32 %38, %38, %38, 25\n v_alignbit_b32 %39, %39, %39, 25\n"
        "v_xor_b32 %4, %4, %16\n v_xor_b32 %9, %9, %17\n v_xor_b32 %14, %14, %18\n v_xor_b32 %3, %3, %19\n"
        "v_xor_b32 %24, %24, %36\n v_xor_b32 %29, %29, %37\n v_xor_b32 %34, %34, %38\n v_xor_b32 %23, %23, %39\n"
        "v_add_u32 %16, %4, %0\n v_add_u32 %17, %9, %5\n v_add_u32 %18, %14, %10\n v_add_u32 %19, %3, %15\n"
        "v_add_u32 %36, %24, %20\n v_add_u32 %37, %29, %25\n v_add_u32 %38, %34, %30\n v_add_u32 %39, %23, %35\n"
        "v_alignbit_b32 %16, %16, %16, 23\n v_alignbit_b32 %17, %17, %17, 23\n v_alignbit_b32 %18, %18, %18, 23\n v_alignbit_b32 %19, %19, %19, 23\n"
        "v_alignbit_b32 %36, %36, %36, 23\n v_alignbit_b32 %37, %37, %37, 23\n v_alignbit_b32 %38, %38, %38, 23\n v_alignbit_b32 %39, %39, %39, 23\n"
        "v_xor_b32 %8, %8, %16\n v_xor_b32 %13, %13, %17\n v_xor_b32 %2, %2, %18\n v_xor_b32 %7, %7, %19\n"
        "v_xor_b32 %28, %28, %36\n v_xor_b32 %33, %33, %37\n v_xor_b32 %22, %22, %38\n v_xor_b32 %27, %27, %39\n"
        "v_add_u32 %16, %8, %4\n v_add_u32 %17, %13, %9\n v_add_u32 %18, %2, %14\n v_add_u32 %19, %7, %3\n"
        "v_add_u32 %36, %28, %24\n v_add_u32 %37, %33, %29\n v_add_u32 %38, %22, %34\n v_add_u32 %39, %27, %23\n"
        "v_alignbit_b32 %16, %16, %16, 19\n v_alignbit_b32 %17, %17, %17, 19\n v_alignbit_b32 %18, %18, %18, 19\n v_alignbit_b32 %19, %19, %19, 19\n"
        "v_alignbit_b32 %36, %36, %36, 19\n v_alignbit_b32 %37, %37, %37, 19\n v_alignbit_b32 %38, %38, %38, 19\n v_alignbit_b32 %39, %39, %39, 19\n"
        "v_xor_b32 %12, %12, %16\n v_xor_b32 %1, %1, %17\n v_xor_b32 %6, %6, %18\n v_xor_b32 %11, %11, %19\n"
        "v_xor_b32 %32, %32, %36\n v_xor_b32 %21, %21, %37\n v_xor_b32 %26, %26, %38\n v_xor_b32 %31, %31, %39\n"
        "v_add_u32 %16, %12, %8\n v_add_u32 %17, %1, %13\n v_add_u32 %18, %6, %2\n v_add_u32 %19, %11, %7\n"
        "v_add_u32 %36, %32, %28\n v_add_u32 %37, %21, %33\n v_add_u32 %38, %26, %22\n v_add_u32 %39, %31, %27\n"
        "v_alignbit_b32 %16, %16, %16, 14\n v_alignbit_b32 %17, %17, %17, 14\n v_alignbit_b32 %18, %18, %18, 14\n v_alignbit_b32 %19, %19, %19, 14\n"
        "v_alignbit_b32 %36, %36, %36, 14\n v_alignbit_b32 %37, %37, %37, 14\n v_alignbit_b32 %38, %38, %38, 14\n v_alignbit_b32 %39, %39, %39, 14\n"
        "v_xor_b32 %0, %0, %16\n v_xor_b32 %5, %5, %17\n v_xor_b32 %10, %10, %18\n v_xor_b32 %15, %15, %19\n"
        "v_xor_b32 %20, %20, %36\n v_xor_b32 %25, %25, %37\n v_xor_b32 %30, %30, %38\n v_xor_b32 %35, %35, %39\n"
        : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
          "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3),
          "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
          "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]), "+v"(y[14]), "+v"(y[15]),
          "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3));
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime();
  uint32_t a = 0;
  for (int i = 0; i < 16; i++) a = a * 31 + x[i] + y[i];
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

static uint32_t rl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

int main() {
  const int maxw = 8 * 1024;
  uint32_t* d; unsigned long long* cyc;
  (void)hipMalloc(&d, maxw * 64 * 4); (void)hipMalloc(&cyc, maxw * 8);
  for (int W : {1, 2, 4, 8}) {
    int blocks = W * 1024;
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<<<blocks, 64>>>(d, cyc, 3); (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0); k<<<blocks, 64>>>(d, cyc, 3); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> hc(blocks); std::vector<uint32_t> ho(64);
    (void)hipMemcpy(hc.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho.data(), d, 64 * 4, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : hc) avg += v; avg /= blocks;
    // CPU check of lane 0 / block 0
    uint32_t x[16]; for (int i = 0; i < 16; i++) x[i] = 3u * (i + 1) + 0;
    for (int r = 0; r < REPS; r++) {
      int q[4][4] = {{0, 4, 8, 12}, {5, 9, 13, 1}, {10, 14, 2, 6}, {15, 3, 7, 11}};
      for (auto& Q : q) { uint32_t &A = x[Q[0]], &B = x[Q[1]], &C = x[Q[2]], &D = x[Q[3]];
        B ^= rl(A + D, 7); C ^= rl(B + A, 9); D ^= rl(C + B, 13); A ^= rl(D + C, 18); }
    }
    uint32_t a = 0; for (int i = 0; i < 16; i++) a = a * 31 + x[i];
    double instr = 48.0 * REPS;
    printf("W=%d waves/SIMD: kernel %.3f ms, per-wave %.0f cycles -> %.2f cycles/instr per wave, %.2f per SIMD; check %s\n",
           W, ms, avg, avg / instr, avg / instr / W, a == ho[0] ? "OK" : "MISMATCH");
  }
  // equal total work, large grid: 4-chain vs 8-chain by wall time
  for (int rep = 0; rep < 2; rep++) {
    const int big = 256 * 64;  // waves (one per 64-thread WG)
    uint32_t* dd; unsigned long long* cc; (void)hipMalloc(&dd, big * 64 * 4); (void)hipMalloc(&cc, big * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<<<big, 64>>>(dd, cc, 3); k8<<<big, 64>>>(dd, cc, 3); k_e64<<<big, 64>>>(dd, cc, 3); (void)hipDeviceSynchronize();
    float m4, m8, me;
    (void)hipEventRecord(e0); k_e64<<<big, 64>>>(dd, cc, 3); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&me, e0, e1);
    (void)hipEventRecord(e0); k<<<big, 64>>>(dd, cc, 3); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&m4, e0, e1);
    (void)hipEventRecord(e0); k8<<<big, 64>>>(dd, cc, 3); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&m8, e0, e1);
    double instr_per_simd = (double)big / 1024 * 48.0 * REPS;
    printf("big grid: VOP3-encoded 4-chain %.3f ms\n", me);
    printf("big grid: 4-chain %.3f ms (%.2f cyc/instr/SIMD @2.39GHz), 8-chain %.3f ms (%.2f)\n", m4,
           m4 * 1e-3 * 2.39e9 / instr_per_simd, m8, m8 * 1e-3 * 2.39e9 / instr_per_simd);
    (void)hipFree(dd); (void)hipFree(cc);
  }
  return 0;
}
