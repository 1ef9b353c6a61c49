// Throughput of the crypt kernels working on pinned host memory directly (zero-copy over
// PCIe) vs the device-resident rate, for batches of B blocks (keygen in HBM).  Diagnostic.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../rclone_amd/csrc/xs_internal.h"

int main(int argc, char** argv) {
  const uint64_t nb = argc > 1 ? atoll(argv[1]) : 16384, plen = nb * 65536, blen = nb * 65552;
  uint8_t *hp, *hb, *ho, *hok;
  xs::BlockKey *ws, *ws2;
  if (hipHostMalloc(&hp, plen) || hipHostMalloc(&hb, blen) || hipHostMalloc(&ho, plen) || hipHostMalloc(&hok, nb) ||
      hipMalloc(&ws, nb * sizeof(xs::BlockKey)) || hipMalloc(&ws2, nb * sizeof(xs::BlockKey)))
    return 1;
  memset(hp, 0x5a, plen);
  xs::KeyArg k{};
  xs::NonceArg n{};
  (void)xs::launch_keygen(0, k, n, 0, plen, nb, nullptr, ws, 0);
  (void)xs::launch_keygen(1, k, n, 0, blen, nb, nullptr, ws2, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int dir = 0; dir < 2; dir++) {
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      (void)hipEventRecord(a, 0);
      if (dir == 0) (void)xs::launch_crypt(true, ws, nb, hp, hb, nullptr, 0);
      else (void)xs::launch_crypt(false, ws2, nb, hb, ho, hok, 0);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    printf("%s host->host %llu blocks: %.3f ms  %.2f GiB/s  err=%s\n", dir ? "open" : "seal", (unsigned long long)nb,
           best, plen / 1073741824.0 / (best * 1e-3), hipGetErrorString(hipGetLastError()));
  }
  int okall = 1;
  for (uint64_t i = 0; i < nb; i++) okall &= hok[i];
  printf("round trip %s\n", okall && !memcmp(hp, ho, plen) ? "ok" : "BAD");
  return 0;
}
