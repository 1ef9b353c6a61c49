// Salsa20 double round with the four independent quarter-rounds of each half-round
// interleaved by hand (gfx950 inline asm).  hipcc (ROCm 7.2) otherwise routes every
// quarter-round through one temporary and issues the 320 add/rotate/xor steps as a single
// dependency chain: ~3.9 cycles per instruction measured, against ~1.4 for this order
// (tools/microbench/bankbench.hip, corebench.hip).  The add/xor and v_alignbit (rotate)
// instructions of the four chains co-issue.
#pragma once
#include <stdint.h>

// One half-round: QR(a_i, b_i, c_i, d_i) for i = 0..3, step-interleaved.
// QR: b ^= rotl(a+d,7); c ^= rotl(b+a,9); d ^= rotl(c+b,13); a ^= rotl(d+c,18).
// rotl(x, n) == v_alignbit_b32(x, x, 32-n).
#define XS_HALF_ROUND(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3)              \
  asm volatile(                                                                                     \
      "v_add_u32 %16, %0, %3\n\t v_add_u32 %17, %4, %7\n\t v_add_u32 %18, %8, %11\n\t v_add_u32 %19, %12, %15\n\t" \
      "v_alignbit_b32 %16, %16, %16, 25\n\t v_alignbit_b32 %17, %17, %17, 25\n\t"                  \
      "v_alignbit_b32 %18, %18, %18, 25\n\t v_alignbit_b32 %19, %19, %19, 25\n\t"                  \
      "v_xor_b32 %1, %1, %16\n\t v_xor_b32 %5, %5, %17\n\t v_xor_b32 %9, %9, %18\n\t v_xor_b32 %13, %13, %19\n\t" \
      "v_add_u32 %16, %1, %0\n\t v_add_u32 %17, %5, %4\n\t v_add_u32 %18, %9, %8\n\t v_add_u32 %19, %13, %12\n\t" \
      "v_alignbit_b32 %16, %16, %16, 23\n\t v_alignbit_b32 %17, %17, %17, 23\n\t"                  \
      "v_alignbit_b32 %18, %18, %18, 23\n\t v_alignbit_b32 %19, %19, %19, 23\n\t"                  \
      "v_xor_b32 %2, %2, %16\n\t v_xor_b32 %6, %6, %17\n\t v_xor_b32 %10, %10, %18\n\t v_xor_b32 %14, %14, %19\n\t" \
      "v_add_u32 %16, %2, %1\n\t v_add_u32 %17, %6, %5\n\t v_add_u32 %18, %10, %9\n\t v_add_u32 %19, %14, %13\n\t" \
      "v_alignbit_b32 %16, %16, %16, 19\n\t v_alignbit_b32 %17, %17, %17, 19\n\t"                  \
      "v_alignbit_b32 %18, %18, %18, 19\n\t v_alignbit_b32 %19, %19, %19, 19\n\t"                  \
      "v_xor_b32 %3, %3, %16\n\t v_xor_b32 %7, %7, %17\n\t v_xor_b32 %11, %11, %18\n\t v_xor_b32 %15, %15, %19\n\t" \
      "v_add_u32 %16, %3, %2\n\t v_add_u32 %17, %7, %6\n\t v_add_u32 %18, %11, %10\n\t v_add_u32 %19, %15, %14\n\t" \
      "v_alignbit_b32 %16, %16, %16, 14\n\t v_alignbit_b32 %17, %17, %17, 14\n\t"                  \
      "v_alignbit_b32 %18, %18, %18, 14\n\t v_alignbit_b32 %19, %19, %19, 14\n\t"                  \
      "v_xor_b32 %0, %0, %16\n\t v_xor_b32 %4, %4, %17\n\t v_xor_b32 %8, %8, %18\n\t v_xor_b32 %12, %12, %19" \
      : "+v"(a0), "+v"(b0), "+v"(c0), "+v"(d0), "+v"(a1), "+v"(b1), "+v"(c1), "+v"(d1), "+v"(a2),   \
        "+v"(b2), "+v"(c2), "+v"(d2), "+v"(a3), "+v"(b3), "+v"(c3), "+v"(d3), "=&v"(t0_), "=&v"(t1_), \
        "=&v"(t2_), "=&v"(t3_))

// 20 rounds (10 double rounds) over x[16] in place.
__device__ __forceinline__ void xs_salsa20_rounds_asm(uint32_t (&x)[16]) {
  uint32_t t0_, t1_, t2_, t3_;
#pragma unroll 1
  for (int i = 0; i < 10; i++) {
    // column round: (0,4,8,12) (5,9,13,1) (10,14,2,6) (15,3,7,11)
    XS_HALF_ROUND(x[0], x[4], x[8], x[12], x[5], x[9], x[13], x[1], x[10], x[14], x[2], x[6], x[15], x[3], x[7], x[11]);
    // row round: (0,1,2,3) (5,6,7,4) (10,11,8,9) (15,12,13,14)
    XS_HALF_ROUND(x[0], x[1], x[2], x[3], x[5], x[6], x[7], x[4], x[10], x[11], x[8], x[9], x[15], x[12], x[13], x[14]);
  }
}
