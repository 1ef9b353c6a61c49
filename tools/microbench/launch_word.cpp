// Ranged-read dispatch diagnostic: host launch -> completion word of one fused
// open (windowed or whole block), with the host key setup or without (XS_KEY_PRE_MAX), on the null
// stream / a non-blocking stream / a high-priority stream (the engine's express lane).  Includes the
// kernel file itself.  usage: launch_word [reps] [host_key 0|1] [stream 0|1|2] [window mask, 0 = whole]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Irclone_amd/csrc -Iinclude tools/microbench/launch_word.cpp -o tools/microbench/launch_word
#include "xs_kernels.hip"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
namespace xs { void set_error(const char*, ...) {} }
static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 1000, use_pre = argc > 2 ? atoi(argv[2]) : 0, stype = argc > 3 ? atoi(argv[3]) : 0;
  const uint32_t window = argc > 4 ? (uint32_t)strtoul(argv[4], nullptr, 0) : 0x2u;
  setenv("XS_KEY_PRE_MAX", use_pre ? "2" : "0", 1);  // read once, at the first launch
  const int nb = 256;
  uint8_t *plain, *wire, *back, *ok; uint32_t* flag; uint32_t* ctr;
  if (hipHostMalloc((void**)&plain, 65536, hipHostMallocPortable) || hipHostMalloc((void**)&wire, 65552ull * nb, hipHostMallocPortable) ||
      hipHostMalloc((void**)&back, 65536, hipHostMallocPortable) || hipHostMalloc((void**)&ok, 64, hipHostMallocPortable) ||
      hipHostMalloc((void**)&flag, 64, hipHostMallocPortable) || hipMalloc((void**)&ctr, 64) || hipMemset(ctr, 0, 64)) return 1;
  for (int i = 0; i < 65536; i++) plain[i] = (uint8_t)(i * 7 + 1);
  xs::KeyArg key; for (int i = 0; i < 8; i++) key.k[i] = 0x01020304u * (i + 1);
  xs::NonceArg bounds{}; bounds.n[0] = bounds.n[2] = 1u << 20;
  hipStream_t s = nullptr;
  if (stype == 1) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (stype == 2) { int lo, hi; (void)hipDeviceGetStreamPriorityRange(&lo, &hi); (void)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi); }
  xs_block_desc d{}; d.len = 65536; for (int i = 0; i < 24; i++) d.nonce[i] = (uint8_t)(i + 1);
  for (int i = 0; i < nb; i++)  // seal nb copies (same plaintext, same nonce: same bytes)
    if (xs::launch_crypt_fused(true, key, bounds, &d, &d, 1, plain, wire + 65552ull * i, nullptr, nullptr, nullptr, 0, s)) return 2;
  if (hipStreamSynchronize(s)) return 2;
  std::vector<double> t;
  xs_block_desc od = d; od.reserved = window ? (xs::XS_DESC_WINDOW | window) : 0u;
  for (int r = 0; r < reps + 50; r++) {
    const uint32_t seq = (uint32_t)r + 1u;
    const double t0 = now_us();
    if (xs::launch_crypt_fused(false, key, bounds, &od, &od, 1, wire + 65552ull * (r % nb), back, ok, ctr, flag, seq, s)) return 3;
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    const double t1 = now_us();
    if (r >= 50) t.push_back(t1 - t0);
    (void)hipStreamSynchronize(s);
  }
  if (!ok[0] || memcmp(back + 4096, plain + 4096, 4000)) { fprintf(stderr, "bad open\n"); return 4; }
  std::sort(t.begin(), t.end());
  printf("{\"pre\": %d, \"stream\": %d, \"window\": %u, \"launch_to_word_p50_us\": %.2f, \"p10\": %.2f, \"p90\": %.2f}\n", use_pre, stype, window, t[t.size() / 2], t[t.size() / 10], t[9 * t.size() / 10]);
  return 0;
}
