// Diagnostic: time xs_crypt<seal> over 100k resident 64 KiB blocks for ablation builds of
// xs_kernels.hip (-DXS_ABLATE=N).  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../rclone_amd/csrc/xs_internal.h"

int main(int argc, char** argv) {
  const uint64_t nb = 100000;
  uint8_t *plain, *body; xs::BlockKey* ws;
  (void)hipMalloc(&plain, nb * 65536); (void)hipMalloc(&body, nb * 65552); (void)hipMalloc(&ws, nb * sizeof(xs::BlockKey));
  (void)hipMemset(plain, 7, nb * 65536);
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
    float best = 1e9, tot = 0;
    for (int r = 0; r < 5; r++) {
      (void)hipEventRecord(a);
      go();
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); tot += ms; if (ms < best) best = ms;
    }
    printf("%s %s: best %.3f ms avg %.3f ms  (%.1f GiB/s)  err=%s\n", argc > 1 ? argv[1] : "", dir ? "open" : "seal",
           best, tot / 5, nb * 65536.0 / 1073741824.0 / (best * 1e-3), hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
