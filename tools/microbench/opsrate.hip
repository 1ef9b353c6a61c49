// Microbenchmark: throughput of the integer VALU instructions the
// XSalsa20/Poly1305 kernels are built from (gfx950). Each lane runs 8
// independent dependency chains so issue rate, not latency, is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
#define CH 8

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t a[CH]; uint64_t q[CH];
  for (int i = 0; i < CH; i++) { a[i] = seed * (threadIdx.x + 1) + i; q[i] = a[i] * 7ull; }
  uint32_t b = seed ^ 0x9e3779b9u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[i]));
      if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 4) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "v"(b) : "vcc");
      if constexpr (OP == 5) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 6) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      if constexpr (OP == 7) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "s"(b) : "vcc");
      if constexpr (OP == 8) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(a[i]), "+v"(b), "+v"(a[(i+1)%CH]) :: "vcc");
      if constexpr (OP == 9) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    }
  }
  uint32_t s = 0; for (int i = 0; i < CH; i++) s += a[i] + (uint32_t)q[i] + (uint32_t)(q[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP> void run(const char* name, uint32_t* d, int blocks, int insts_per_iter) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<OP><<<blocks, 256>>>(d, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) k<OP><<<blocks, 256>>>(d, r + 2);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = 5.0 * blocks * 256.0 * ITERS * CH * insts_per_iter;
  printf("%-22s %8.2f T lane-instr/s  (%.3f ms)\n", name, lane_ops / (ms * 1e-3) / 1e12, ms);
}

int main() {
  uint32_t* d; int blocks = 256 * 8 * 4;
  hipMalloc(&d, blocks * 256 * 4);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run<0>("v_add_u32", d, blocks, 1);
  run<9>("v_xor_b32", d, blocks, 1);
  run<1>("v_alignbit_b32", d, blocks, 1);
  run<2>("v_mul_lo_u32", d, blocks, 1);
  run<3>("v_mul_hi_u32", d, blocks, 1);
  run<4>("v_mad_u64_u32 (v,v)", d, blocks, 1);
  run<7>("v_mad_u64_u32 (v,s)", d, blocks, 1);
  run<5>("v_mul_u32_u24", d, blocks, 1);
  run<6>("v_mul_hi_u32_u24", d, blocks, 1);
  run<8>("v_add_co+v_addc_co", d, blocks, 2);
  return 0;
}
