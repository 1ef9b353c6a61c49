// Probe: can the crypt kernels read their input from and write their output to pinned host
// memory directly (hipHostMalloc, zero-copy over PCIe)?  Seals and opens a few blocks with
// src/dst in host memory and compares with the all-device path.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../rclone_amd/csrc/xs_internal.h"

int main() {
  const uint64_t nb = 8, plen = nb * 65536 - 1000, blen = plen + nb * 16;
  uint8_t *hp, *hb, *ho, *hok, *dp, *db, *dok;
  xs::BlockKey* ws;
  if (hipHostMalloc(&hp, plen) || hipHostMalloc(&hb, blen) || hipHostMalloc(&ho, plen) || hipHostMalloc(&hok, nb) ||
      hipMalloc(&dp, plen) || hipMalloc(&db, blen) || hipMalloc(&dok, nb) || hipMalloc(&ws, nb * sizeof(xs::BlockKey)))
    return 1;
  for (uint64_t i = 0; i < plen; i++) hp[i] = (uint8_t)(i * 7 + (i >> 9));
  xs::KeyArg k{};
  xs::NonceArg n{};
  for (int i = 0; i < 8; i++) k.k[i] = 0x01020304u * (i + 1);
  // device reference
  (void)hipMemcpy(dp, hp, plen, hipMemcpyHostToDevice);
  (void)xs::launch_keygen(0, k, n, 0, plen, nb, nullptr, ws, 0);
  (void)xs::launch_crypt(true, ws, nb, dp, db, nullptr, 0);
  std::vector<uint8_t> ref(blen);
  (void)hipMemcpy(ref.data(), db, blen, hipMemcpyDeviceToHost);
  // zero-copy seal: host in, host out
  (void)xs::launch_crypt(true, ws, nb, hp, hb, nullptr, 0);
  hipError_t e = hipDeviceSynchronize();
  printf("seal host->host: %s, equal %d\n", hipGetErrorString(e), e == hipSuccess && !memcmp(ref.data(), hb, blen));
  (void)xs::launch_keygen(1, k, n, 0, blen, nb, nullptr, ws, 0);
  (void)xs::launch_crypt(false, ws, nb, hb, ho, hok, 0);
  e = hipDeviceSynchronize();
  int okall = 1;
  for (uint64_t i = 0; i < nb; i++) okall &= hok[i] == 1;
  printf("open host->host: %s, equal %d, ok %d\n", hipGetErrorString(e), e == hipSuccess && !memcmp(hp, ho, plen), okall);
  return 0;
}
