// MD5 rate on this host's cores: scalar (xs_host_md5.h) vs 8 and 16 streams per core
// (md5_x16.h), checked against the scalar digests.  Diagnostic.
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "../../rclone_amd/csrc/md5_x16.h"
#include "md5_x8.h"
#include "../../rclone_amd/csrc/xs_host_md5.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t per = 8 << 20;  // bytes per stream
  std::vector<uint8_t> big(16 * per);
  std::mt19937_64 rng(7);
  for (auto& b : big) b = (uint8_t)rng();
  uint32_t ref[16][4];
  double t = now();
  for (int l = 0; l < 16; l++) {
    xs::HostMd5 m;
    m.update(big.data() + l * per, per);
    for (int w = 0; w < 4; w++) ref[l][w] = m.state()[w];
  }
  const double scalar = 16.0 * per / (now() - t) / 1e9;
  int bad = 0;
  double x16 = 0, x8 = 0;
  if (xs::md5_x16_supported()) {
    uint32_t st[4][16];
    const uint8_t* p[16];
    uint32_t stride[16];
    for (int l = 0; l < 16; l++) {
      for (int w = 0; w < 4; w++) st[w][l] = xs::HostMd5().state()[w];
      p[l] = big.data() + l * per;
      stride[l] = 64;
    }
    t = now();
    xs::md5_x16_blocks(st, p, stride, per / 64);
    x16 = 16.0 * per / (now() - t) / 1e9;
    for (int l = 0; l < 16; l++)
      for (int w = 0; w < 4; w++) bad += st[w][l] != ref[l][w];
  }
  if (xs::md5_x8_supported()) {
    t = now();
    for (int h = 0; h < 2; h++) {
      uint32_t st[4][8];
      const uint8_t* p[8];
      uint32_t stride[8];
      for (int l = 0; l < 8; l++) {
        for (int w = 0; w < 4; w++) st[w][l] = xs::HostMd5().state()[w];
        p[l] = big.data() + (8 * h + l) * per;
        stride[l] = 64;
      }
      xs::md5_x8_blocks(st, p, stride, per / 64);
      for (int l = 0; l < 8; l++)
        for (int w = 0; w < 4; w++) bad += st[w][l] != ref[8 * h + l][w];
    }
    x8 = 16.0 * per / (now() - t) / 1e9;
  }
  printf("{\"scalar_GB_s_per_core\": %.3f, \"x8_GB_s_per_core\": %.3f, \"x8_GB_s_per_stream\": %.3f, "
         "\"x16_GB_s_per_core\": %.3f, \"x16_GB_s_per_stream\": %.3f, \"mismatches\": %d}\n",
         scalar, x8, x8 / 8, x16, x16 / 16, bad);
  return bad ? 1 : 0;
}
