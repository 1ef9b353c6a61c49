// Scalar host MD5, round-2 step order (tools/microbench/xs_host_md5_r02.h, a copy of that
// revision) vs the current xs_host_md5.h, alternating on one core; digests must agree.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../rclone_amd/csrc/xs_host_md5.h"
#include "xs_host_md5_r02.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  std::vector<uint8_t> b(64 << 20);
  for (size_t i = 0; i < b.size(); i++) b[i] = (uint8_t)(i * 131 + (i >> 9));
  double best_old = 0, best_new = 0;
  uint8_t d0[16], d1[16];
  for (int r = 0; r < 5; r++) {
    double t = now();
    xs_r02::HostMd5 a;
    a.update(b.data(), b.size());
    a.final(d0);
    best_old = std::max(best_old, b.size() / (now() - t) / 1e9);
    t = now();
    xs::HostMd5 c;
    c.update(b.data(), b.size());
    c.final(d1);
    best_new = std::max(best_new, b.size() / (now() - t) / 1e9);
  }
  printf("{\"round2_GB_s\": %.3f, \"round3_GB_s\": %.3f, \"same_digest\": %s}\n", best_old, best_new,
         memcmp(d0, d1, 16) ? "false" : "true");
  return memcmp(d0, d1, 16) ? 1 : 0;
}
