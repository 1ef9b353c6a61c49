// Diagnostic: time xs_crypt<seal> / <open> over 100k resident 64 KiB blocks, linked against a kernel
// TU (the product xs_kernels.hip, or an ablation copy made by tools/archive/ablate_variant.py).  Not part of
// the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include "../rclone_amd/csrc/xs_internal.h"

int main(int argc, char** argv) {
  const uint64_t nb = 100000;
  uint8_t *plain, *body; xs::BlockKey* ws;
  (void)hipMalloc(&plain, nb * 65536); (void)hipMalloc(&body, nb * 65552); (void)hipMalloc(&ws, nb * sizeof(xs::BlockKey));
  (void)xs::launch_fill(reinterpret_cast<uint64_t*>(plain), nb * 65536 / 8, 12345, 0, 1, 0);  // random, like bench.py
  xs::KeyArg k{}; xs::NonceArg n{};
  for (int i = 0; i < 8; i++) k.k[i] = 0x01020304u * (i + 1);
  uint8_t* okb; xs::BlockKey* ws2; uint8_t* out;
  (void)hipMalloc(&okb, nb); (void)hipMalloc(&ws2, nb * sizeof(xs::BlockKey)); (void)hipMalloc(&out, nb * 65536);
  (void)xs::launch_keygen(0, k, n, 0, nb * 65536, nb, nullptr, ws, 0);
  (void)xs::launch_keygen(1, k, n, 0, nb * 65552, nb, nullptr, ws2, 0);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int dir = 0; dir < 2; dir++) {
    auto go = [&] {
      if (dir == 0) (void)xs::launch_crypt(true, ws, nb, plain, body, nullptr, 0);
      else (void)xs::launch_crypt(false, ws2, nb, body, out, okb, 0);
    };
    for (int r = 0; r < 2; r++) go();
    (void)hipDeviceSynchronize();
    std::vector<float> t;
    for (int r = 0; r < 25; r++) {
      (void)hipEventRecord(a);
      go();
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%s %s: min %.3f ms median %.3f ms  (%.1f GiB/s at median)  err=%s\n", argc > 1 ? argv[1] : "",
           dir ? "open" : "seal", t[0], t[12], nb * 65536.0 / 1073741824.0 / (t[12] * 1e-3),
           hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
