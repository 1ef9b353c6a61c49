// Paired A/B timing of two builds of the crypt kernels in ONE process: build A is namespace
// xs (xs_kernels.hip at a git revision, see tools/archive/abtest.sh), build B is the working tree
// compiled with -Dxs=xs_b plus the variant's macros.  Each build runs its own keygen.
// Launches alternate A, B, A, B, ... over 100k resident random blocks, so clock/power drift
// hits both; reports medians and the median of per-pair ratios B/A for keygen, seal and open,
// and checks that B's wire body, plaintext and tag verdicts equal A's byte for byte.
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>
#include "../rclone_amd/csrc/xs_internal.h"

namespace xs_b {  // build B: same layout, its own namespace
struct BlockKey;
hipError_t launch_crypt(bool seal, const BlockKey* keys, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                        uint8_t* ok, hipStream_t stream);
}  // namespace xs_b
namespace xs_b {
// the B object's KeyArg/NonceArg are layout-identical structs in namespace xs_b
struct KeyArg { uint32_t k[8]; };
struct NonceArg { uint32_t n[6]; };
hipError_t launch_keygen(int mode, const KeyArg& key, const NonceArg& nonce0, uint64_t first_block,
                         uint64_t total_len, uint64_t nblocks, const xs_block_desc* desc, BlockKey* out,
                         hipStream_t stream);
}  // namespace xs_b
static xs_b::BlockKey* B(xs::BlockKey* k) { return reinterpret_cast<xs_b::BlockKey*>(k); }

static bool same(const uint8_t* a, const uint8_t* b, size_t n) {
  std::vector<uint8_t> ha(1 << 26), hb(1 << 26);
  for (size_t off = 0; off < n; off += ha.size()) {
    const size_t m = std::min(ha.size(), n - off);
    (void)hipMemcpy(ha.data(), a + off, m, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb.data(), b + off, m, hipMemcpyDeviceToHost);
    if (memcmp(ha.data(), hb.data(), m)) return false;
  }
  return true;
}

int main(int argc, char** argv) {
  const uint64_t nb = 100000;
  const int pairs = argc > 1 ? atoi(argv[1]) : 30;
  uint8_t *plain, *bodyA, *bodyB, *outA, *outB, *okA, *okB;
  xs::BlockKey *wsA, *wsA2, *wsB, *wsB2;
  (void)hipMalloc(&plain, nb * 65536);
  (void)hipMalloc(&bodyA, nb * 65552); (void)hipMalloc(&bodyB, nb * 65552);
  (void)hipMalloc(&outA, nb * 65536); (void)hipMalloc(&outB, nb * 65536);
  (void)hipMalloc(&okA, nb); (void)hipMalloc(&okB, nb);
  for (auto p : {&wsA, &wsA2, &wsB, &wsB2}) (void)hipMalloc(p, nb * 4096);  // >= either build's BlockKey
  (void)xs::launch_fill(reinterpret_cast<uint64_t*>(plain), nb * 65536 / 8, 12345, 0, 1, 0);
  xs::KeyArg k{};
  xs::NonceArg n{};
  for (int i = 0; i < 8; i++) k.k[i] = 0x01020304u * (i + 1);
  for (int i = 0; i < 6; i++) n.n[i] = 0x9e3779b9u * (i + 3);
  xs_b::KeyArg kb;
  xs_b::NonceArg nbb;
  memcpy(&kb, &k, sizeof k);
  memcpy(&nbb, &n, sizeof n);
  auto keygen = [&](bool b, bool seal) {
    if (b) return xs_b::launch_keygen(seal ? 0 : 1, kb, nbb, 0, nb * (seal ? 65536 : 65552), nb, nullptr,
                                      B(seal ? wsB : wsB2), 0);
    return xs::launch_keygen(seal ? 0 : 1, k, n, 0, nb * (seal ? 65536 : 65552), nb, nullptr, seal ? wsA : wsA2, 0);
  };
  for (bool b : {false, true})
    for (bool seal : {true, false}) (void)keygen(b, seal);
  (void)xs::launch_crypt(true, wsA, nb, plain, bodyA, nullptr, 0);
  (void)xs_b::launch_crypt(true, B(wsB), nb, plain, bodyB, nullptr, 0);
  (void)hipDeviceSynchronize();
  const bool body_eq = same(bodyA, bodyB, nb * 65552);
  (void)xs::launch_crypt(false, wsA2, nb, bodyA, outA, okA, 0);
  (void)xs_b::launch_crypt(false, B(wsB2), nb, bodyA, outB, okB, 0);
  (void)hipDeviceSynchronize();
  const bool out_eq = same(outA, outB, nb * 65536) && same(okA, okB, nb) && same(outA, plain, nb * 65536);
  printf("B == A: body %s, open %s\n", body_eq ? "yes" : "NO", out_eq ? "yes" : "NO");
  hipEvent_t e[3];
  for (auto& x : e) (void)hipEventCreate(&x);
  const char* names[3] = {"keygen", "seal", "open"};
  for (int dir = 0; dir < 3; dir++) {
    auto go = [&](bool b) {
      if (dir == 0) (void)keygen(b, true);
      // both builds time on the same input and output buffers (placement differences between
      // allocations otherwise bias the pair by several percent)
      else if (dir == 1) (void)(b ? xs_b::launch_crypt(true, B(wsB), nb, plain, bodyB, nullptr, 0)
                                  : xs::launch_crypt(true, wsA, nb, plain, bodyB, nullptr, 0));
      else (void)(b ? xs_b::launch_crypt(false, B(wsB2), nb, bodyA, outB, okB, 0)
                    : xs::launch_crypt(false, wsA2, nb, bodyA, outB, okB, 0));
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
    printf("%s %s: A median %.4f ms  B median %.4f ms  B/A median %.4f  [p10 %.4f p90 %.4f]  err=%s\n",
           argc > 2 ? argv[2] : "", names[dir], ta[pairs / 2], tb[pairs / 2], ratio[pairs / 2],
           ratio[pairs / 10], ratio[pairs * 9 / 10], hipGetErrorString(hipGetLastError()));
  }
  return body_eq && out_eq ? 0 : 1;
}
