// Aggregate scalar MD5 rate of T concurrent streams on this host (xs_host_md5.h), T swept.
// This is the ceiling of the per-object shapes: with C checkers or
// transfers at most C MD5 chains run at once, each one stream's chain.  Every thread hashes its
// own 32 MiB buffer (cache-cold at that size, as a stream of file bytes is) for a fixed time;
// the digests of one pass are checked against a single-threaded pass.
// Usage: md5_threads [seconds per T] [T ...]   (default 1.5 s; T = 1 2 4 8 12 16)
// MD5_MIB=n: n MiB per thread instead of 32 (e.g. 512: far larger than any L3, DRAM-fed like a
// stream's freshly DMA'd wire buffers).
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../rclone_amd/csrc/xs_host_md5.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 1.5;
  std::vector<int> ts;
  for (int i = 2; i < argc; i++) ts.push_back(atoi(argv[i]));
  if (ts.empty()) ts = {1, 2, 4, 8, 12, 16};
  int tmax = 0;
  for (int t : ts) tmax = t > tmax ? t : tmax;
  const char* mib = getenv("MD5_MIB");
  const size_t per = (size_t)(mib ? atoi(mib) : 32) << 20;
  std::vector<std::vector<uint8_t>> buf(tmax, std::vector<uint8_t>(per));
  std::vector<std::array<uint32_t, 4>> ref(tmax);
  for (int i = 0; i < tmax; i++) {
    std::mt19937_64 rng(100 + i);
    for (size_t j = 0; j < per; j += 8) {
      const uint64_t v = rng();
      memcpy(buf[i].data() + j, &v, 8);
    }
    xs::HostMd5 m;
    m.update(buf[i].data(), per);
    for (int w = 0; w < 4; w++) ref[i][w] = m.state()[w];
  }
  int bad = 0;
  for (int T : ts) {
    std::atomic<bool> go{false};
    std::atomic<int> ready{0};
    std::vector<double> bytes(T, 0.0);
    std::vector<int> mism(T, 0);
    std::vector<std::thread> th;
    double t_end = 0;
    for (int i = 0; i < T; i++)
      th.emplace_back([&, i] {
        ready++;
        while (!go.load()) std::this_thread::yield();
        bool first = true;
        while (now() < t_end) {
          xs::HostMd5 m;
          m.update(buf[i].data(), per);
          if (first) {
            for (int w = 0; w < 4; w++) mism[i] += m.state()[w] != ref[i][w];
            first = false;
          }
          bytes[i] += per;
        }
      });
    while (ready.load() < T) std::this_thread::yield();
    const double t0 = now();
    t_end = t0 + secs;
    go = true;
    for (auto& x : th) x.join();
    const double el = now() - t0;
    double tot = 0, mn = 1e30;
    for (int i = 0; i < T; i++) {
      tot += bytes[i];
      mn = bytes[i] < mn ? bytes[i] : mn;
      bad += mism[i];
    }
    printf("{\"mib_per_thread\": %zu, \"threads\": %d, \"GB_s\": %.3f, \"GB_s_per_stream\": %.3f, \"slowest_stream_GB_s\": %.3f, \"seconds\": %.2f}\n",
           per >> 20, T, tot / el / 1e9, tot / el / 1e9 / T, mn / el / 1e9, el);
    fflush(stdout);
  }
  printf("{\"mismatches\": %d}\n", bad);
  return bad ? 1 : 0;
}
