// TEST INFRASTRUCTURE: how the CPU baseline's windowed open (oracle/xsalsa_simd.c
// orc_simd_open_window, the per-read work of a ranged 4 KiB read on a host core) scales with
// threads on this host, without the cipher layer -- the ceiling tools/seek_latency.cpp's CPU build
// is compared with.  usage: par_open THREADS [OPENS_PER_THREAD]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" int orc_simd_open_window(uint8_t*, const uint8_t*, size_t, const uint8_t*, const uint8_t*, size_t, size_t);
extern "C" void orc_simd_secretbox_seal(uint8_t*, const uint8_t*, size_t, const uint8_t*, const uint8_t*);

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 1;
  const int n = argc > 2 ? atoi(argv[2]) : 4000;
  uint8_t key[32] = {1}, nonce[24] = {2};
  std::vector<uint8_t> p(65536, 3), box(65552);
  orc_simd_secretbox_seal(box.data(), p.data(), p.size(), nonce, key);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&] {
      std::vector<uint8_t> out(65536);
      for (int i = 0; i < n; i++) orc_simd_open_window(out.data(), box.data(), box.size(), nonce, key, 4096, 8192);
    });
  for (auto& x : th) x.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"tool\": \"par_open\", \"threads\": %d, \"opens_per_s\": %.0f, \"us_per_open_per_thread\": %.2f}\n", threads,
         threads * (double)n / el, el / n * 1e6);
  return 0;
}
