// Paired A/B timing of two builds of the crypt kernels in ONE process: build A is namespace
// xs (this tree's defaults), build B is xs_kernels.hip compiled with -Dxs=xs_b plus the
// variant's macros.  Launches alternate A, B, A, B, ... over 100k resident random blocks, so
// clock/power drift hits both; reports medians and the median of per-pair ratios B/A.
// Diagnostic only.  Build: see tools/abtest.sh.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "../rclone_amd/csrc/xs_internal.h"

namespace xs_b {  // build B: same layout, its own namespace
struct BlockKey;
hipError_t launch_crypt(bool seal, const BlockKey* keys, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                        uint8_t* ok, hipStream_t stream);
}
static const xs_b::BlockKey* B(const xs::BlockKey* k) { return reinterpret_cast<const xs_b::BlockKey*>(k); }

int main(int argc, char** argv) {
  const uint64_t nb = 100000;
  const int pairs = argc > 1 ? atoi(argv[1]) : 30;
  uint8_t *plain, *body, *out, *okb;
  xs::BlockKey *ws, *ws2;
  (void)hipMalloc(&plain, nb * 65536); (void)hipMalloc(&body, nb * 65552); (void)hipMalloc(&out, nb * 65536);
  (void)hipMalloc(&okb, nb); (void)hipMalloc(&ws, nb * sizeof(xs::BlockKey)); (void)hipMalloc(&ws2, nb * sizeof(xs::BlockKey));
  (void)xs::launch_fill(reinterpret_cast<uint64_t*>(plain), nb * 65536 / 8, 12345, 0, 1, 0);
  xs::KeyArg k{}; xs::NonceArg n{};
  for (int i = 0; i < 8; i++) k.k[i] = 0x01020304u * (i + 1);
  (void)xs::launch_keygen(0, k, n, 0, nb * 65536, nb, nullptr, ws, 0);
  (void)xs::launch_keygen(1, k, n, 0, nb * 65552, nb, nullptr, ws2, 0);
  (void)xs::launch_crypt(true, ws, nb, plain, body, nullptr, 0);
  hipEvent_t e[3];
  for (auto& x : e) (void)hipEventCreate(&x);
  for (int dir = 0; dir < 2; dir++) {
    auto go = [&](bool b) {
      if (dir == 0) (void)(b ? xs_b::launch_crypt(true, B(ws), nb, plain, body, nullptr, 0)
                             : xs::launch_crypt(true, ws, nb, plain, body, nullptr, 0));
      else (void)(b ? xs_b::launch_crypt(false, B(ws2), nb, body, out, okb, 0)
                    : xs::launch_crypt(false, ws2, nb, body, out, okb, 0));
    };
    for (int w = 0; w < 3; w++) { go(false); go(true); }
    (void)hipDeviceSynchronize();
    std::vector<float> ta, tb, ratio;
    for (int r = 0; r < pairs; r++) {
      const bool bfirst = r & 1;  // alternate the order inside a pair too
      (void)hipEventRecord(e[0]);
      go(bfirst);
      (void)hipEventRecord(e[1]);
      go(!bfirst);
      (void)hipEventRecord(e[2]);
      (void)hipEventSynchronize(e[2]);
      float t1, t2;
      (void)hipEventElapsedTime(&t1, e[0], e[1]);
      (void)hipEventElapsedTime(&t2, e[1], e[2]);
      const float a = bfirst ? t2 : t1, b = bfirst ? t1 : t2;
      ta.push_back(a); tb.push_back(b); ratio.push_back(b / a);
    }
    std::sort(ta.begin(), ta.end()); std::sort(tb.begin(), tb.end()); std::sort(ratio.begin(), ratio.end());
    printf("%s %s: A median %.3f ms  B median %.3f ms  B/A median %.4f  [p10 %.4f p90 %.4f]  err=%s\n",
           argc > 2 ? argv[2] : "", dir ? "open" : "seal", ta[pairs / 2], tb[pairs / 2], ratio[pairs / 2],
           ratio[pairs / 10], ratio[pairs * 9 / 10], hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
