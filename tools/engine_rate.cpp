// One-block open rate of one engine under T concurrent callers, without the cipher.go mirror on
// top (diagnostic): each thread opens its own pinned 64 KiB wire block in a loop
// (zero-copy fused batches), every verdict checked.  Separates the engine's submission path from
// the decrypter's per-read work in tools/seek_latency.
//   usage: engine_rate [threads] [seconds]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/rclone_crypt_gpu.h"

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  const double secs = argc > 2 ? atof(argv[2]) : 2.0;
  xs_engine* e = xs_engine_create(0, 256, 3);
  if (!e) {
    fprintf(stderr, "engine: %s\n", xs_last_error());
    return 1;
  }
  uint8_t key[32], nonce[24];
  for (int i = 0; i < 32; i++) key[i] = (uint8_t)(i * 5 + 1);
  for (int i = 0; i < 24; i++) nonce[i] = (uint8_t)(i * 3 + 2);
  uint8_t* plain = (uint8_t*)xs_host_alloc(65536);
  uint8_t* wire = (uint8_t*)xs_host_alloc(65552);
  for (int i = 0; i < 65536; i++) plain[i] = (uint8_t)(i * 7);
  if (xs_engine_seal(e, key, nonce, 0, plain, 65536, wire) != XS_OK) return 1;
  std::atomic<long> ops{0}, bad{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&] {
      uint8_t* w = (uint8_t*)xs_host_alloc(65552);
      uint8_t* out = (uint8_t*)xs_host_alloc(65536);
      memcpy(w, wire, 65552);
      uint8_t ok = 0;
      while (!stop.load(std::memory_order_relaxed)) {
        if (xs_engine_open(e, key, nonce, 0, w, 65552, out, &ok) != XS_OK || !ok) bad++;
        ops++;
      }
      if (memcmp(out, plain, 65536)) bad++;
      xs_host_free(w);
      xs_host_free(out);
    });
  const auto t0 = std::chrono::steady_clock::now();
  std::this_thread::sleep_for(std::chrono::duration<double>(secs));
  stop = true;
  for (auto& x : th) x.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t st[3];
  xs_engine_stats(e, st);
  printf("{\"tool\": \"engine_rate\", \"threads\": %d, \"opens_per_s\": %.0f, \"batches\": %llu, \"requests\": %llu, "
         "\"bad\": %ld}\n",
         T, ops.load() / el, (unsigned long long)st[0], (unsigned long long)st[1], bad.load());
  xs_engine_destroy(e);
  return bad.load() ? 1 : 0;
}
