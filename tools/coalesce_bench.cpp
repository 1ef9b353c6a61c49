// Host-path throughput of many concurrent small objects through the rc_* cipher.go mirror
// (rc_encrypt_data + rc_decrypt_data from memory readers), T threads sharing one cipher --
// rclone's --transfers pattern.  Run with XS_ENGINE_COALESCE=0/1 to compare one GPU round trip
// per handle batch against cross-handle coalescing.  Verifies every round trip.
// usage: coalesce_bench <threads> <objects_per_thread> <object_bytes> [readahead_first_blocks]
//        (readahead 1 = default adaptive read-ahead; 0 = full batch_blocks from the first refill)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include "../include/rclone_crypt_gpu.h"

struct Mem {
  const uint8_t* p;
  int64_t n, pos;
};
static int64_t mem_read(void* u, uint8_t* dst, int64_t n, int32_t* err) {
  Mem* m = (Mem*)u;
  int64_t k = m->n - m->pos < n ? m->n - m->pos : n;
  memcpy(dst, m->p + m->pos, (size_t)k);
  m->pos += k;
  *err = m->pos >= m->n ? RC_EOF : RC_NIL;
  return k;
}
static int32_t mem_close(void*) { return RC_NIL; }

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  const int K = argc > 2 ? atoi(argv[2]) : 200;
  const int64_t S = argc > 3 ? atoll(argv[3]) : 65536;
  int32_t e = 0;
  rc_cipher* c = rc_cipher_new("potato", "", &e);
  if (!c) return 1;
  rc_cipher_set_batch_blocks(c, argc > 5 ? (uint32_t)atoi(argv[5]) : 64);  // argv[5]: batch blocks per refill
  if (argc > 4) rc_cipher_set_readahead(c, (uint32_t)atoi(argv[4]));
  std::vector<uint8_t> src((size_t)S);
  for (int64_t i = 0; i < S; i++) src[(size_t)i] = (uint8_t)(i * 7 + 3);
  // warm the engine
  {
    Mem m{src.data(), S, 0};
    rc_reader r{mem_read, nullptr, nullptr, &m};
    rc_encrypter* h = rc_encrypt_data(c, r, nullptr, &e);
    std::vector<uint8_t> out(rc_encrypted_size(S) + 16);
    int64_t got = 0;
    while (true) {
      int64_t k = rc_encrypter_read(h, out.data() + got, (int64_t)out.size() - got, &e);
      got += k;
      if (e != RC_NIL) break;
    }
    rc_encrypter_free(h);
  }
  std::atomic<int> bad{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) {
    th.emplace_back([&, t] {
      std::vector<uint8_t> ct((size_t)rc_encrypted_size(S) + 64), back((size_t)S + 64);
      for (int k = 0; k < K; k++) {
        int32_t err = 0;
        Mem m{src.data(), S, 0};
        rc_encrypter* h = rc_encrypt_data(c, rc_reader{mem_read, nullptr, nullptr, &m}, nullptr, &err);
        int64_t got = 0;
        while (true) {
          int64_t n = rc_encrypter_read(h, ct.data() + got, (int64_t)ct.size() - got, &err);
          got += n;
          if (err != RC_NIL) break;
        }
        rc_encrypter_free(h);
        if (err != RC_EOF || got != rc_encrypted_size(S)) { bad++; continue; }
        Mem mc{ct.data(), got, 0};
        rc_decrypter* d = rc_decrypt_data(c, rc_reader{mem_read, mem_close, nullptr, &mc}, &err);
        if (!d) { bad++; continue; }
        int64_t pg = 0;
        while (true) {
          int64_t n = rc_decrypter_read(d, back.data() + pg, (int64_t)back.size() - pg, &err);
          pg += n;
          if (err != RC_NIL) break;
        }
        rc_decrypter_close(d);
        rc_decrypter_free(d);
        if (err != RC_EOF || pg != S || memcmp(back.data(), src.data(), (size_t)S)) bad++;
      }
    });
  }
  for (auto& x : th) x.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double gib = 2.0 * T * K * (double)S / (1 << 30);  // encrypt + decrypt
  const char* co = getenv("XS_ENGINE_COALESCE");
  printf("{\"threads\": %d, \"objects\": %d, \"object_bytes\": %lld, \"coalesce\": %s, \"seconds\": %.4f, "
         "\"GiB_s\": %.3f, \"objects_s\": %.0f, \"readahead\": %d, \"bad\": %d}\n",
         T, T * K, (long long)S, (co && atoi(co) == 0) ? "false" : "true", el, gib / el, 2.0 * T * K / el,
         argc > 4 ? atoi(argv[4]) : 1, bad.load());
  rc_cipher_free(c);
  return bad.load() != 0;
}
