// Phase timing of the fused v2 / v3 ranged-read kernels (diagnostic).  Built with
// -DXS_F2_PROBE against rclone_amd/csrc/xs_kernels.hip directly: the kernel records
// s_memrealtime (100 MHz) at its phase boundaries for workgroup 0; one full 64 KiB block is
// sealed and opened from pinned host memory (the engine's zero-copy path) REPS times and the
// median offset of every mark from the kernel's entry is printed per wave, in microseconds.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DXS_F2_PROBE tools/fused_probe.cpp -o tools/fused_probe
#include "../rclone_amd/csrc/xs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

namespace xs {
void set_error(const char*, ...) {}
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int only_open = argc > 2 ? atoi(argv[2]) : 0;  // 1: seal once, then open only (warm code)
  const int ncw = argc > 3 ? atoi(argv[3]) : 4;        // crypt waves: 4 (v2) or 8 (v3)
  const int nw = ncw + 2;                              // crypt waves, key-schedule wave, keygen marks (row 9)
  const int inline_desc = argc > 4 ? atoi(argv[4]) : 1;  // 0: the kernel reads the pinned descriptor
  // OPEN group window (xs_engine_open_range): bit g = decrypt 4 KiB group g; 0 = the whole block
  const uint32_t window = argc > 5 ? (uint32_t)strtoul(argv[5], nullptr, 0) & 0xFFFFu : 0u;
  uint8_t *plain, *wire, *back, *ok;
  xs_block_desc* desc;
  if (hipHostMalloc((void**)&plain, 65536, hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc((void**)&wire, 65552, hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc((void**)&back, 65536, hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc((void**)&ok, 64, hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc((void**)&desc, sizeof(xs_block_desc), hipHostMallocMapped) != hipSuccess)
    return 1;
  for (int i = 0; i < 65536; i++) plain[i] = (uint8_t)(i * 7 + 1);
  xs::KeyArg key;
  for (int i = 0; i < 8; i++) key.k[i] = 0x01020304u * (i + 1);
  xs::NonceArg bounds{};
  const uint64_t cap = 1 << 20;
  bounds.n[0] = (uint32_t)cap;
  bounds.n[2] = (uint32_t)cap;
  void *dp, *dw, *db, *dok, *dd;
  hipHostGetDevicePointer(&dp, plain, 0);
  hipHostGetDevicePointer(&dw, wire, 0);
  hipHostGetDevicePointer(&db, back, 0);
  hipHostGetDevicePointer(&dok, ok, 0);
  hipHostGetDevicePointer(&dd, desc, 0);
  std::vector<std::vector<double>> d(2 * 10 * 16), clk(2 * 10 * 16);
  for (int r = 0; r < reps; r++) {
    for (int dir = (only_open && r > 0) ? 1 : 0; dir < 2; dir++) {
      memset(desc, 0, sizeof *desc);
      desc->len = 65536;
      for (int i = 0; i < 24; i++) desc->nonce[i] = (uint8_t)(i + 1);
      // bounds are offsets within [base, base + cap): plain/wire/back are separate allocations,
      // so address them from each buffer's own base
      {  // no stale marks from the other direction or version
        unsigned long long z[2 * 10 * 16] = {};
        hipMemcpyToSymbol(HIP_SYMBOL(xs::xs_f2_probe), z, sizeof z);
      }
      xs::XsInlineDescs inl{};  // the engine passes small batches' descriptors in the kernel arguments
      inl.d[0] = *desc;
      inl.n = inline_desc ? 1u : 0u;
      const bool seal = dir == 0;
      if (!seal && window) inl.d[0].reserved = desc->reserved = xs::XS_DESC_WINDOW | window;
      const uint8_t* src = (const uint8_t*)(seal ? dp : dw);
      uint8_t* dst = (uint8_t*)(seal ? dw : db);
      if (ncw == 8) {
        if (seal)
          hipLaunchKernelGGL((xs::xs_crypt_fused2<true, 8>), dim3(1), dim3(576), 0, 0, key, bounds,
                             (const xs_block_desc*)dd, inl, 1, src, dst, (uint8_t*)dok, nullptr, nullptr, 0);
        else
          hipLaunchKernelGGL((xs::xs_crypt_fused2<false, 8>), dim3(1), dim3(576), 0, 0, key, bounds,
                             (const xs_block_desc*)dd, inl, 1, src, dst, (uint8_t*)dok, nullptr, nullptr, 0);
      } else {
        if (seal)
          hipLaunchKernelGGL((xs::xs_crypt_fused2<true, 4>), dim3(1), dim3(320), 0, 0, key, bounds,
                             (const xs_block_desc*)dd, inl, 1, src, dst, (uint8_t*)dok, nullptr, nullptr, 0);
        else
          hipLaunchKernelGGL((xs::xs_crypt_fused2<false, 4>), dim3(1), dim3(320), 0, 0, key, bounds,
                             (const xs_block_desc*)dd, inl, 1, src, dst, (uint8_t*)dok, nullptr, nullptr, 0);
      }
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      unsigned long long t[2 * 10 * 16];
      hipMemcpyFromSymbol(t, HIP_SYMBOL(xs::xs_f2_probe), sizeof t);
      const unsigned long long t0 = t[0];
      for (int w = 0; w < 10; w++)
        for (int s = 0; s < 16; s++)
          if (t[16 * w + s] >= t0 && t[16 * w + s] - t0 < 100000) {
            d[(dir * 10 + w) * 16 + s].push_back((t[16 * w + s] - t0) / 100.0);
            // shader clock since the previous mark of this wave (GHz), in clk[]
            int p = s - 1;
            while (p >= 0 && !(t[16 * w + p] > t0 - 1 && t[16 * w + p] <= t[16 * w + s])) p--;
            if (p >= 0 && t[16 * w + s] > t[16 * w + p])
              clk[(dir * 10 + w) * 16 + s].push_back((double)(t[160 + 16 * w + s] - t[160 + 16 * w + p]) /
                                                      (double)(t[16 * w + s] - t[16 * w + p]) / 10.0);
          }
    }
  }
  bool same = true;
  for (int g = 0; g < 16; g++) {  // group g = plaintext [4096g - 32, 4096g + 4064); the last 32 bytes always
    const int g0 = g ? 4096 * g - 32 : 0, g1 = g == 15 ? 65536 : 4096 * g + 4064;
    if ((!window || ((window >> g) & 1u)) && memcmp(back + g0, plain + g0, g1 - g0)) same = false;
  }
  if (!ok[0] || !same) {
    fprintf(stderr, "round trip failed (ok=%d)\n", ok[0]);
    return 3;
  }
  const char* names[16] = {"entry", "desc", "subkey|keygen", "ks0|Z", "data0", "ks1", "data1", "ks2", "data2",
                           "ks3", "data3", "phase1", "B1", "B2", "final|loads", "hsalsa"};
  printf("{\"tool\": \"fused_probe\", \"reps\": %d, \"us_from_entry_median\": {", reps);
  bool first = true;
  for (int dir = 0; dir < 2; dir++)
    for (int w = 0; w < 10; w++) {
      if (w >= nw - 1 && w < 9) continue;
      printf("%s\"%s_w%d\": {", first ? "" : ", ", dir ? "open" : "seal", w);
      first = false;
      bool f2 = true;
      for (int s = 0; s < 16; s++) {
        auto& v = d[(dir * 10 + w) * 16 + s];
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        auto& c = clk[(dir * 10 + w) * 16 + s];
        std::sort(c.begin(), c.end());
        printf("%s\"%s\": [%.2f, %.2f]", f2 ? "" : ", ", names[s], v[v.size() / 2], c.empty() ? 0.0 : c[c.size() / 2]);
        f2 = false;
      }
      printf("}");
    }
  printf("}}\n");
  return 0;
}
