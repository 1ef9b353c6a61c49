// Microbenchmark 2: more gfx950 VALU forms relevant to Salsa20/Poly1305.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define CH 8

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t a[CH]; uint64_t q[CH];
  for (int i = 0; i < CH; i++) { a[i] = seed * (threadIdx.x + 1) + i; q[i] = a[i] * 7ull + 3; }
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if constexpr (OP == 0) asm volatile("v_lshrrev_b64 %0, 26, %0" : "+v"(q[i]));
      if constexpr (OP == 1) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i+1)%CH]));
      if constexpr (OP == 2) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc");
      if constexpr (OP == 3) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 4) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 5) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 6) asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 7) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 8) asm volatile("v_lshlrev_b32_e32 %0, 7, %0" : "+v"(a[i]));
      if constexpr (OP == 9) asm volatile("v_and_b32_e32 %0, 0x3ffffff, %0" : "+v"(a[i]));
      if constexpr (OP == 10) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 11) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(a[i]) : "s"(b));
      if constexpr (OP == 12) asm volatile("v_alignbit_b32 %0, %0, %1, 26" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 13) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 14) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 15) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 16) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i+1)%CH]));
      if constexpr (OP == 17) asm volatile("v_or3_b32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 18) asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 19) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(0x05040100u));
      if constexpr (OP == 20) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 21) asm volatile("v_mad_u64_u32 %0, s[10:11], %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "s"(b) : "s10", "s11");
    }
  }
  uint32_t s = 0; for (int i = 0; i < CH; i++) s += a[i] + (uint32_t)q[i] + (uint32_t)(q[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP> void run(const char* name, uint32_t* d, int blocks) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k<OP><<<blocks, 256>>>(d, 1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; r++) k<OP><<<blocks, 256>>>(d, r + 2);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = 5.0 * blocks * 256.0 * ITERS * CH;
  printf("%-26s %8.2f T lane-instr/s\n", name, lane_ops / (ms * 1e-3) / 1e12);
}

int main() {
  uint32_t* d; int blocks = 256 * 8 * 4;
  (void)hipMalloc(&d, blocks * 256 * 4);
  run<20>("v_add_u32_e64 (ref)", d, blocks);
  run<0>("v_lshrrev_b64", d, blocks);
  run<1>("v_lshl_add_u64", d, blocks);
  run<2>("v_add_co_u32_e32", d, blocks);
  run<3>("v_add3_u32", d, blocks);
  run<4>("v_lshl_add_u32", d, blocks);
  run<5>("v_xad_u32", d, blocks);
  run<6>("v_add_u32_dpp", d, blocks);
  run<7>("v_xor_b32_dpp", d, blocks);
  run<16>("v_mov_b32_dpp", d, blocks);
  run<8>("v_lshlrev_b32_e32", d, blocks);
  run<9>("v_and_b32 (literal)", d, blocks);
  run<10>("v_cndmask_b32_e32", d, blocks);
  run<11>("v_add_u32 (sgpr)", d, blocks);
  run<12>("v_alignbit_b32 (2 src)", d, blocks);
  run<13>("v_pk_add_u16", d, blocks);
  run<14>("v_lshl_or_b32", d, blocks);
  run<15>("v_mad_u32_u24", d, blocks);
  run<17>("v_or3_b32", d, blocks);
  run<18>("v_bfi_b32", d, blocks);
  run<19>("v_perm_b32", d, blocks);
  run<21>("v_mad_u64_u32 sdst", d, blocks);
  return 0;
}
