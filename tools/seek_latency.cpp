// Ranged-read latency through the cipher.go mirror (VFS / chunked-reader
// style short random reads, cipher.go:935-1039 DecryptDataSeek + RangeSeek).  An object of
// --mib MiB is encrypted once (rc_encrypt_data) into host memory; then --reads random
// (offset, --len) reads each open a fresh rc_decrypt_data_seek over a memory open-callback
// that serves the requested underlying range, read --len plaintext bytes and check them.
// Reports per-read latency percentiles and reads/s for --threads concurrent readers.
// Diagnostic / measurement tool (GPU behind the C ABI).
//   usage: seek_latency [--mib M] [--reads K] [--len L] [--threads T] [--batch-blocks B]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/rclone_crypt_gpu.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Span {  // a reader over bytes [pos, end) of a buffer
  const uint8_t* p;
  int64_t pos, end;
};
static int64_t span_read(void* u, uint8_t* dst, int64_t n, int32_t* err) {
  Span* s = (Span*)u;
  const int64_t k = std::min(n, s->end - s->pos);
  memcpy(dst, s->p + s->pos, (size_t)k);
  s->pos += k;
  *err = s->pos >= s->end ? RC_EOF : RC_NIL;
  return k;
}
static int32_t span_close(void* u) {
  delete (Span*)u;
  return RC_NIL;
}
struct Store {
  const uint8_t* ct;
  int64_t len;
};
// OpenRangeSeek (cipher.go:77): the underlying object from offset, limit bytes (-1 = to end)
static int32_t open_range(void* user, int64_t offset, int64_t limit, rc_reader* out) {
  Store* st = (Store*)user;
  Span* s = new Span{st->ct, std::min(offset, st->len), limit < 0 ? st->len : std::min(st->len, offset + limit)};
  *out = rc_reader{span_read, span_close, nullptr, s};
  return RC_NIL;
}

int main(int argc, char** argv) {
  int64_t mib = 256, reads = 2000, len = 4096;
  int threads = 1, batch = 0;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto nx = [&] { return std::string(i + 1 < argc ? argv[++i] : "0"); };
    if (a == "--mib") mib = atoll(nx().c_str());
    else if (a == "--reads") reads = atoll(nx().c_str());
    else if (a == "--len") len = atoll(nx().c_str());
    else if (a == "--threads") threads = atoi(nx().c_str());
    else if (a == "--batch-blocks") batch = atoi(nx().c_str());
    else return 2;
  }
  const int64_t size = mib << 20;
  std::vector<uint8_t> plain((size_t)size);
  uint64_t s = 0x5EED;
  for (int64_t k = 0; k < size; k += 8) {
    const uint64_t v = splitmix(s);
    memcpy(plain.data() + k, &v, 8);
  }
  int32_t err = 0;
  rc_cipher* c = rc_cipher_new("potato", "", &err);
  if (!c) return 1;
  if (batch > 0) rc_cipher_set_batch_blocks(c, (uint32_t)batch);
  std::vector<uint8_t> ct((size_t)rc_encrypted_size(size));
  {
    Span* src = new Span{plain.data(), 0, size};
    rc_encrypter* h = rc_encrypt_data(c, rc_reader{span_read, span_close, nullptr, src}, nullptr, &err);
    if (!h) return 1;
    int64_t got = 0;
    for (;;) {
      const int64_t k = rc_encrypter_read(h, ct.data() + got, (int64_t)ct.size() - got, &err);
      got += k;
      if (err != RC_NIL || got == (int64_t)ct.size()) break;
    }
    rc_encrypter_free(h);
    span_close(src);
    if (got != (int64_t)ct.size()) {
      fprintf(stderr, "encrypt short %lld\n", (long long)got);
      return 1;
    }
  }
  Store st{ct.data(), (int64_t)ct.size()};
  std::vector<std::vector<double>> lat(threads);
  std::atomic<int64_t> bad{0};
  // per-phase time sums (microseconds): seek-open, read, close + free
  std::atomic<int64_t> ph_open{0}, ph_read{0}, ph_close{0};
  auto one = [&](uint64_t& rs, std::vector<uint8_t>& buf) {
    const int64_t off = (int64_t)(splitmix(rs) % (uint64_t)(size - len + 1));
    const double t0 = now();
    int32_t e = 0;
    rc_decrypter* d = rc_decrypt_data_seek(c, open_range, &st, off, len, &e);
    const double t1 = now();
    double t2 = t1;
    int64_t got = 0;
    if (d) {
      for (;;) {
        const int64_t k = rc_decrypter_read(d, buf.data() + got, len - got, &e);
        got += k;
        if (e != RC_NIL || got == len) break;
      }
      t2 = now();
      rc_decrypter_close(d);
      rc_decrypter_free(d);
    }
    const double dt = now() - t0;
    ph_open += (int64_t)((t1 - t0) * 1e6);
    ph_read += (int64_t)((t2 - t1) * 1e6);
    ph_close += (int64_t)((t0 + dt - t2) * 1e6);
    if (got != len || memcmp(buf.data(), plain.data() + off, (size_t)len)) {
      if (bad++ < 4) {
        int64_t first = -1;
        for (int64_t i = 0; i < got && first < 0; i++)
          if (buf[(size_t)i] != plain[(size_t)(off + i)]) first = i;
        fprintf(stderr, "bad read: off %lld got %lld err %d (%s) first mismatch %lld xs: %s\n", (long long)off,
                (long long)got, (int)e, rc_error_string(e), (long long)first, xs_last_error());
      }
    }
    return dt;
  };
  {  // warm-up (engine creation, first launches)
    uint64_t rs = 1;
    std::vector<uint8_t> buf((size_t)len);
    for (int i = 0; i < 20; i++) one(rs, buf);
  }
  uint64_t st0[3] = {0, 0, 0}, st1[3] = {0, 0, 0};  // engine: combined batches, requests, blocks
  xs_engine* eng = xs_pool_engine(rc_default_pool(), 0);
  xs_engine_stats(eng, st0);
  const double t0 = now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      uint64_t rs = 1000 + t;
      std::vector<uint8_t> buf((size_t)len);
      for (int64_t i = t; i < reads; i += threads) lat[t].push_back(one(rs, buf));
    });
  for (auto& x : th) x.join();
  const double el = now() - t0;
  xs_engine_stats(eng, st1);
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(p * all.size()))] * 1e6; };
  const char* sm = getenv("XS_SPLIT_MAX");
  printf("{\"split_max_env\": \"%s\", \"p25_us\": %.1f, \"p75_us\": %.1f, ", sm ? sm : "", pct(0.25), pct(0.75));
  const double nr = (double)std::max<size_t>(all.size() + 20, 1);
  printf("\"mean_open_us\": %.1f, \"mean_read_us\": %.1f, \"mean_close_us\": %.1f, ", ph_open / nr, ph_read / nr,
         ph_close / nr);
  printf("\"engine_batches\": %llu, \"engine_requests\": %llu, ", (unsigned long long)(st1[0] - st0[0]),
         (unsigned long long)(st1[1] - st0[1]));
  printf("\"tool\": \"seek_latency\", \"object_mib\": %lld, \"read_len\": %lld, \"threads\": %d, \"reads\": %zu, "
         "\"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, \"reads_per_s\": %.0f, \"bad\": %lld}\n",
         (long long)mib, (long long)len, threads, all.size(), pct(0.5), pct(0.9), pct(0.99), all.size() / el,
         (long long)bad.load());
  rc_cipher_free(c);
  return bad ? 1 : 0;
}
