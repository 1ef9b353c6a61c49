// Does VGPR bank (reg % 4) of the two sources matter on gfx950?  8 independent add chains
// with explicit physical registers: sources in the same bank as the destination or not.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
template <int V>
__global__ void __launch_bounds__(256) k(uint32_t* out) {
  uint32_t r;
  asm volatile(
      "v_mov_b32 v8, 1\n v_mov_b32 v9, 2\n v_mov_b32 v10, 3\n v_mov_b32 v11, 4\n"
      "v_mov_b32 v12, 5\n v_mov_b32 v13, 6\n v_mov_b32 v14, 7\n v_mov_b32 v15, 8\n"
      "v_mov_b32 v16, 9\n v_mov_b32 v17, 10\n v_mov_b32 v18, 11\n v_mov_b32 v19, 12\n"
      "v_mov_b32 v20, 13\n v_mov_b32 v21, 14\n v_mov_b32 v22, 15\n v_mov_b32 v23, 16\n"
      "v_mov_b32 v24, 17\n v_mov_b32 v25, 18\n v_mov_b32 v26, 19\n v_mov_b32 v27, 20\n"
      "s_mov_b32 s20, %1\n"
      "1:\n"
#define L8(op) op
      ".rept 16\n"
#if V == 0   /* add: dst/src0 v8..v15, src1 v16..v23 -> src banks equal (8%4 == 16%4) */
      "v_add_u32 v8, v8, v16\n v_add_u32 v9, v9, v17\n v_add_u32 v10, v10, v18\n v_add_u32 v11, v11, v19\n"
      "v_add_u32 v12, v12, v20\n v_add_u32 v13, v13, v21\n v_add_u32 v14, v14, v22\n v_add_u32 v15, v15, v23\n"
#elif V == 1 /* add: src1 shifted by one register -> different banks */
      "v_add_u32 v8, v8, v17\n v_add_u32 v9, v9, v18\n v_add_u32 v10, v10, v19\n v_add_u32 v11, v11, v20\n"
      "v_add_u32 v12, v12, v21\n v_add_u32 v13, v13, v22\n v_add_u32 v14, v14, v23\n v_add_u32 v15, v15, v24\n"
#elif V == 2 /* alignbit same register twice */
      "v_alignbit_b32 v8, v8, v8, 7\n v_alignbit_b32 v9, v9, v9, 7\n v_alignbit_b32 v10, v10, v10, 7\n v_alignbit_b32 v11, v11, v11, 7\n"
      "v_alignbit_b32 v12, v12, v12, 7\n v_alignbit_b32 v13, v13, v13, 7\n v_alignbit_b32 v14, v14, v14, 7\n v_alignbit_b32 v15, v15, v15, 7\n"
#elif V == 3 /* xor same bank */
      "v_xor_b32 v8, v8, v16\n v_xor_b32 v9, v9, v17\n v_xor_b32 v10, v10, v18\n v_xor_b32 v11, v11, v19\n"
      "v_xor_b32 v12, v12, v20\n v_xor_b32 v13, v13, v21\n v_xor_b32 v14, v14, v22\n v_xor_b32 v15, v15, v23\n"
#elif V == 4 /* xor different bank */
      "v_xor_b32 v8, v8, v17\n v_xor_b32 v9, v9, v18\n v_xor_b32 v10, v10, v19\n v_xor_b32 v11, v11, v20\n"
      "v_xor_b32 v12, v12, v21\n v_xor_b32 v13, v13, v22\n v_xor_b32 v14, v14, v23\n v_xor_b32 v15, v15, v24\n"
#elif V == 5 /* salsa-like mix: add(diff bank) -> alignbit -> xor(diff bank), 4 chains */
      "v_add_u32 v16, v8, v13\n v_add_u32 v17, v9, v14\n v_add_u32 v18, v10, v15\n v_add_u32 v19, v11, v12\n"
      "v_alignbit_b32 v16, v16, v16, 25\n v_alignbit_b32 v17, v17, v17, 25\n v_alignbit_b32 v18, v18, v18, 25\n v_alignbit_b32 v19, v19, v19, 25\n"
      "v_xor_b32 v12, v12, v16\n v_xor_b32 v13, v13, v17\n v_xor_b32 v14, v14, v18\n v_xor_b32 v15, v15, v19\n"
#elif V == 6 /* salsa-like mix, same banks: add(v8+v12) etc */
      "v_add_u32 v16, v8, v12\n v_add_u32 v17, v9, v13\n v_add_u32 v18, v10, v14\n v_add_u32 v19, v11, v15\n"
      "v_alignbit_b32 v16, v16, v16, 25\n v_alignbit_b32 v17, v17, v17, 25\n v_alignbit_b32 v18, v18, v18, 25\n v_alignbit_b32 v19, v19, v19, 25\n"
      "v_xor_b32 v20, v20, v16\n v_xor_b32 v21, v21, v17\n v_xor_b32 v22, v22, v18\n v_xor_b32 v23, v23, v19\n"
#elif V == 7 /* exact Salsa column half-round (x_i in v8+i), temps v24..v27 */
      "v_add_u32 v24, v8, v20\n v_add_u32 v25, v13, v9\n v_add_u32 v26, v18, v14\n v_add_u32 v27, v23, v19\n"
      "v_alignbit_b32 v24, v24, v24, 25\n v_alignbit_b32 v25, v25, v25, 25\n v_alignbit_b32 v26, v26, v26, 25\n v_alignbit_b32 v27, v27, v27, 25\n"
      "v_xor_b32 v12, v12, v24\n v_xor_b32 v17, v17, v25\n v_xor_b32 v22, v22, v26\n v_xor_b32 v11, v11, v27\n"
      "v_add_u32 v24, v12, v8\n v_add_u32 v25, v17, v13\n v_add_u32 v26, v22, v18\n v_add_u32 v27, v11, v23\n"
      "v_alignbit_b32 v24, v24, v24, 23\n v_alignbit_b32 v25, v25, v25, 23\n v_alignbit_b32 v26, v26, v26, 23\n v_alignbit_b32 v27, v27, v27, 23\n"
      "v_xor_b32 v16, v16, v24\n v_xor_b32 v21, v21, v25\n v_xor_b32 v10, v10, v26\n v_xor_b32 v15, v15, v27\n"
      "v_add_u32 v24, v16, v12\n v_add_u32 v25, v21, v17\n v_add_u32 v26, v10, v22\n v_add_u32 v27, v15, v11\n"
      "v_alignbit_b32 v24, v24, v24, 19\n v_alignbit_b32 v25, v25, v25, 19\n v_alignbit_b32 v26, v26, v26, 19\n v_alignbit_b32 v27, v27, v27, 19\n"
      "v_xor_b32 v20, v20, v24\n v_xor_b32 v9, v9, v25\n v_xor_b32 v14, v14, v26\n v_xor_b32 v19, v19, v27\n"
      "v_add_u32 v24, v20, v16\n v_add_u32 v25, v9, v21\n v_add_u32 v26, v14, v10\n v_add_u32 v27, v19, v15\n"
      "v_alignbit_b32 v24, v24, v24, 14\n v_alignbit_b32 v25, v25, v25, 14\n v_alignbit_b32 v26, v26, v26, 14\n v_alignbit_b32 v27, v27, v27, 14\n"
      "v_xor_b32 v8, v8, v24\n v_xor_b32 v13, v13, v25\n v_xor_b32 v18, v18, v26\n v_xor_b32 v23, v23, v27\n"
#endif
      ".endr\n"
      "s_sub_u32 s20, s20, 1\n"
      "s_cmp_lg_u32 s20, 0\n"
      "s_cbranch_scc1 1b\n"
      "v_add_u32 %0, v8, v15\n"
      : "=v"(r) : "s"(ITERS) : "v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","s20","scc");
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int V> void run(const char* name, uint32_t* d, int blocks, int ops_per_rep) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k<V><<<blocks, 256>>>(d); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0); for (int r = 0; r < 3; r++) k<V><<<blocks, 256>>>(d); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double ops = 3.0 * blocks * 256.0 * ITERS * 16 * ops_per_rep;
  double cyc = ms * 1e-3 * 2.4e9 * 1024;  // SIMD-cycles at 2.4 GHz
  printf("%-34s %7.2f T lane-instr/s  %.2f cycles per wave-instr\n", name, ops / (ms * 1e-3) / 1e12, cyc / (ops / 64));
}
int main() {
  uint32_t* d; int blocks = 256 * 8 * 2; (void)hipMalloc(&d, blocks * 256 * 4);
  run<0>("add  src banks equal", d, blocks, 8);
  run<1>("add  src banks differ", d, blocks, 8);
  run<2>("alignbit (x,x)", d, blocks, 8);
  run<3>("xor  src banks equal", d, blocks, 8);
  run<4>("xor  src banks differ", d, blocks, 8);
  run<5>("salsa-mix diff banks (4 chains)", d, blocks, 12);
  run<6>("salsa-mix same banks (4 chains)", d, blocks, 12);
  run<7>("salsa half-round exact pattern", d, blocks, 48);
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
