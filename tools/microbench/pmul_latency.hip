// Poly1305 field-multiply latency on one wave (diagnostic): the ranged-read kernel's
// key schedule is a chain of ~13 dependent multiplies (the power levels up to r^4096), measured at
// 0.72-0.96 us per level step inside the fused kernel.  This times chains of dependent multiplies
// in one wave64 with s_memtime (shader clock) / s_memrealtime (100 MHz), alone on the chip:
//   pmul   : the product form (radix 2^26, 5 limbs, 25 v_mad_u64_u32, carry-first columns)
//   psq    : a squaring (15 products: the cross terms doubled)
// (timing only: the chains' values are written out so nothing is optimised away)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/pmul_latency.hip -o tools/microbench/pmul_latency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstring>

constexpr uint32_t M26 = 0x3ffffffu;
struct P5 {
  uint32_t v[5];
};

__device__ __forceinline__ P5 pmul(const P5& h, const P5& m) {
  const uint32_t s1 = m.v[1] * 5, s2 = m.v[2] * 5, s3 = m.v[3] * 5, s4 = m.v[4] * 5;
  uint64_t d0 = (uint64_t)h.v[0] * m.v[0] + (uint64_t)h.v[1] * s4 + (uint64_t)h.v[2] * s3 + (uint64_t)h.v[3] * s2 +
                (uint64_t)h.v[4] * s1;
  P5 o;
  o.v[0] = (uint32_t)d0 & M26;
  uint64_t d1 = (d0 >> 26) + (uint64_t)h.v[0] * m.v[1] + (uint64_t)h.v[1] * m.v[0] + (uint64_t)h.v[2] * s4 +
                (uint64_t)h.v[3] * s3 + (uint64_t)h.v[4] * s2;
  o.v[1] = (uint32_t)d1 & M26;
  uint64_t d2 = (d1 >> 26) + (uint64_t)h.v[0] * m.v[2] + (uint64_t)h.v[1] * m.v[1] + (uint64_t)h.v[2] * m.v[0] +
                (uint64_t)h.v[3] * s4 + (uint64_t)h.v[4] * s3;
  o.v[2] = (uint32_t)d2 & M26;
  uint64_t d3 = (d2 >> 26) + (uint64_t)h.v[0] * m.v[3] + (uint64_t)h.v[1] * m.v[2] + (uint64_t)h.v[2] * m.v[1] +
                (uint64_t)h.v[3] * m.v[0] + (uint64_t)h.v[4] * s4;
  o.v[3] = (uint32_t)d3 & M26;
  uint64_t d4 = (d3 >> 26) + (uint64_t)h.v[0] * m.v[4] + (uint64_t)h.v[1] * m.v[3] + (uint64_t)h.v[2] * m.v[2] +
                (uint64_t)h.v[3] * m.v[1] + (uint64_t)h.v[4] * m.v[0];
  o.v[4] = (uint32_t)d4 & M26;
  uint32_t c = (uint32_t)(d4 >> 26);
  o.v[0] += c * 5;
  c = o.v[0] >> 26;
  o.v[0] &= M26;
  o.v[1] += c;
  return o;
}

// h^2: d_k = sum_{i+j=k} h_i h_j + 5 sum_{i+j=k+5} h_i h_j, cross terms doubled
__device__ __forceinline__ P5 psq(const P5& h) {
  const uint32_t a0 = h.v[0], a1 = h.v[1], a2 = h.v[2], a3 = h.v[3], a4 = h.v[4];
  const uint32_t d0x = 2 * a0, d1x = 2 * a1, s4 = 5 * a4, s3 = 5 * a3;
  uint64_t d0 = (uint64_t)a0 * a0 + (uint64_t)(2 * a1) * s4 + (uint64_t)a2 * (2 * s3);
  P5 o;
  o.v[0] = (uint32_t)d0 & M26;
  uint64_t d1 = (d0 >> 26) + (uint64_t)d0x * a1 + (uint64_t)a2 * (2 * s4) + (uint64_t)a3 * s3;
  o.v[1] = (uint32_t)d1 & M26;
  uint64_t d2 = (d1 >> 26) + (uint64_t)d0x * a2 + (uint64_t)a1 * a1 + (uint64_t)a3 * (2 * s4);
  o.v[2] = (uint32_t)d2 & M26;
  uint64_t d3 = (d2 >> 26) + (uint64_t)d0x * a3 + (uint64_t)d1x * a2 + (uint64_t)a4 * s4;
  o.v[3] = (uint32_t)d3 & M26;
  uint64_t d4 = (d3 >> 26) + (uint64_t)d0x * a4 + (uint64_t)d1x * a3 + (uint64_t)a2 * a2;
  o.v[4] = (uint32_t)d4 & M26;
  uint32_t c = (uint32_t)(d4 >> 26);
  o.v[0] += c * 5;
  c = o.v[0] >> 26;
  o.v[0] &= M26;
  o.v[1] += c;
  return o;
}

template <int MODE>
__global__ void chain(const uint32_t* in, uint32_t* out, unsigned long long* clk, int n) {
  const uint32_t l = threadIdx.x;
  P5 h, m;
  for (int i = 0; i < 5; i++) {
    h.v[i] = in[10 * l + i] & M26;
    m.v[i] = in[10 * l + 5 + i] & M26;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < n; k++) {
    if (MODE == 0) h = pmul(h, m);
    else h = psq(h);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 5; i++) out[5 * l + i] = h.v[i];
  if (l == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

int main() {
  const int n = 4096;
  uint32_t hin[640];
  uint64_t s = 0x1234567;
  for (auto& x : hin) x = (uint32_t)((s = s * 6364136223846793005ull + 1442695040888963407ull) >> 33);
  uint32_t *din, *dout;
  unsigned long long* dclk;
  (void)hipMalloc(&din, sizeof hin);
  (void)hipMalloc(&dout, 320 * 4);
  (void)hipMalloc(&dclk, 16);
  (void)hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice);
  const char* names[2] = {"pmul", "psq"};
  uint32_t res[2][320];
  for (int mode = 0; mode < 2; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, din, dout, dclk, n);
      else hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, din, dout, dclk, n);
      (void)hipDeviceSynchronize();
      unsigned long long clk[2];
      (void)hipMemcpy(clk, dclk, 16, hipMemcpyDeviceToHost);
      (void)hipMemcpy(res[mode], dout, sizeof res[mode], hipMemcpyDeviceToHost);
      if (rep == 2)
        printf("{\"op\": \"%s\", \"chain\": %d, \"shader_cycles_per_op\": %.1f, \"ns_per_op\": %.1f, \"clock_ghz\": %.3f}\n",
               names[mode], n, (double)clk[0] / n, clk[1] * 10.0 / n, (double)clk[0] / (clk[1] * 10.0));
    }
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  (void)hipFree(dclk);
  return 0;
}
