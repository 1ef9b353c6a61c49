// BASELINE configs[4] end-to-end harness: `rclone sync <local tree> crypt:` with crypt over an
// in-memory remote (backend/memory), then `rclone cryptcheck`, in one process, through the C ABI
// the Go side would bind (include/rclone_crypt_gpu.h).  Diagnostic / measurement tool, not the
// product; the crypt work runs on the GPU through librclone_crypt.so.
//
// Flow (reference: crypt.go:497-563 Fs.put, memory.go:580-588 Object.Hash, crypt.go:784-852 +
// cmd/cryptcheck/cryptcheck.go:67-117):
//   tree   : files with log-uniform sizes in [4 KiB, 8 MiB] (+ 0/1/65536/65537-byte edge files),
//            SplitMix64 content, written under --dir (page cache: the local backend's reads
//            come from memory, as in a warm rclone run).
//   sync   : batch mode (default) -- groups of whole files are read in parallel into a pinned
//            staging buffer and handed to xs_engine_put_batch: one H2D, seal + MD5 of the crypt
//            file on the GPU (the hash crypt.put tees off the ciphertext), the wire bodies D2H
//            straight into the memory remote's (pinned) arena.  Two lanes (two engines) overlap
//            one group's file reads and PCIe with the other's.
//            stream mode (--mode stream) -- the reference's per-object shape (an unchanged
//            fs/sync + crypt.put): --transfers threads each run rc_encrypt_data over the open file
//            (GPU behind the encrypter, cross-caller coalescing) and the memory remote's Put reads
//            the stream into the object's buffer.  The tee MD5 of the ciphertext is taken by the
//            encrypter (rc_encrypter_set_md5, host workers; --tee encrypter, the default) or by
//            the reading thread (--tee reader, crypt.go:516-533's TeeReader as is).
//            Either way crypt.put then compares the tee hash with the remote's Object.Hash
//            (CPU MD5 of the stored bytes, cached) unless --check-dst-hash 0.  That check is part of
//            each put (crypt.go:542-560: Put returns only after o.Hash, memory.go:580-588), so by
//            default (--put-check inline) it runs inside the transfer, right after the object is
//            stored: in stream mode on the transfer's own thread, in batch mode on --hash-threads
//            workers fed as each group lands (other groups' reads and seals go on meanwhile).
//            sync_GiB_s is the rate with every put's check done; put_only_GiB_s counts to the last
//            stored object only.  --put-check after runs the checks as a phase after all puts (the
//            round-4 accounting).
//   check  : cryptcheck, batch (--check-mode batch, default) -- every local file re-sealed with the
//            nonce read back from the stored header and MD5'd on the GPU (xs_engine_seal_md5),
//            compared with the remote's hash; stream (--check-mode stream) -- the unchanged
//            cmd/cryptcheck's shape (cryptcheck.go:91-114): --checkers threads, each per object
//            reading the nonce through newDecrypter over the header (rc_decrypt_data) and calling
//            computeHashWithNonce (rc_compute_hash_with_nonce) on the open local file.
//   verify : sampled objects decrypted back through rc_decrypt_data (GPU) and compared with the
//            local bytes; one stored object corrupted -> cryptcheck must flag exactly that one.
// Prints one JSON line.
//   anchor : with --anchor FILE, one JSON line per sampled object (the edge files, ~64 spread
//            over the tree, the largest): plaintext seed and size, nonce, SHA-256 of the stored
//            crypt file (header || wire body as the memory remote holds it) and the tee MD5 --
//            tests/test_e2e_anchor_gpu.py recomputes them with the CPU oracle.
//   tee-all: with --tee-all FILE, one text line per object ("index size seed nonce tee_md5", hex):
//            every stored object's tee MD5, which put's check already equated with the MD5 of the
//            bytes the remote stored -- tests/test_e2e_anchor_gpu.py recomputes all of them with the
//            CPU oracle, so every stored byte of the tree is pinned, not a sample.
//   devices: --devices 0,1,... puts lane l's engine on device list[l % n] and the rc_* handles
//            and name engines on the same list (RCLONE_AMD_DEVICES): one process over several GPUs.
//   usage: e2e_sync [--gib G] [--dir D] [--transfers T] [--mode batch|stream]
//                   [--tee encrypter|reader] [--check-mode batch|stream] [--checkers C]
//                   [--check-dst-hash 0|1] [--put-check inline|after] [--hash-threads H]
//                   [--group-mib M] [--lanes L] [--keep]
//                   [--anchor FILE] [--tee-all FILE] [--devices LIST]
#include <fcntl.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/rclone_crypt_gpu.h"
#include "../rclone_amd/csrc/xs_host_md5.h"

// ---------------------------------------------------------------- MD5 (RFC 1321), host
// The memory remote's Object.Hash and the reading thread's TeeReader (--tee reader) hash with the
// same host MD5 the library uses (about the speed of Go's crypto/md5 assembly / OpenSSL), so the
// tee placements compare like for like.
using Md5 = xs::HostMd5;

// ---------------------------------------------------------------- SHA-256 (FIPS 180-4), host
// for --anchor: digests of sampled stored crypt files, checked by the test suite against the
// oracle's crypt files (tests/test_e2e_anchor_gpu.py)
struct Sha256 {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint8_t buf[64];
  uint64_t n = 0;
  static uint32_t ror(uint32_t x, int c) { return (x >> c) | (x << (32 - c)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t len) {
    size_t have = n & 63;
    n += len;
    if (have) {
      const size_t k = std::min(len, 64 - have);
      memcpy(buf + have, p, k);
      p += k;
      len -= k;
      if (have + k < 64) return;
      block(buf);
    }
    for (; len >= 64; p += 64, len -= 64) block(p);
    memcpy(buf, p, len);
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = n * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while ((n & 63) != 56) update(&zero, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(lb, 8);
    for (int i = 0; i < 8; i++)
      for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
  }
};
static std::string hexs(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; i++) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

// ---------------------------------------------------------------- helpers
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void parallel_for(size_t n, int threads, const std::function<void(size_t)>& f) {
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < std::max(1, threads); t++)
    th.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : th) t.join();
}
static bool read_file(const std::string& path, uint8_t* dst, uint64_t len) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  uint64_t got = 0;
  while (got < len) {
    const ssize_t k = pread(fd, dst + got, len - got, (off_t)got);
    if (k <= 0) break;
    got += (uint64_t)k;
  }
  close(fd);
  return got == len;
}
static uint64_t body_bytes(uint64_t plain) { return plain + ((plain + 65535) / 65536) * 16; }
static uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }
static const uint8_t kMagic[8] = {'R', 'C', 'L', 'O', 'N', 'E', 0, 0};

// memory remote (backend/memory): objects keep header + body bytes and a lazily cached MD5
struct Obj {
  std::string name;          // local file
  std::string rel;           // path relative to the synced root (what crypt encrypts)
  std::string remote;        // EncryptFileName(rel): the object's key on the wrapped remote
  uint64_t size = 0;         // plaintext size (local file)
  uint8_t header[32];        // magic || nonce
  uint8_t* body = nullptr;   // wire body in the arena
  uint64_t body_len = 0;
  uint8_t tee[16];           // crypt.put's hash of the ciphertext stream
  uint8_t dst[16];           // Object.Hash (memory.go:580-588), computed on demand
  bool dst_ok = false;
};
static void dst_hash(Obj& o) {
  if (o.dst_ok) return;
  Md5 m;
  m.update(o.header, 32);
  m.update(o.body, o.body_len);
  m.final(o.dst);
  o.dst_ok = true;
}

// rc_reader over a file descriptor (ReadFill semantics are done by the rc_* layer)
struct FdReader {
  int fd;
};
static int64_t fd_read(void* u, uint8_t* p, int64_t n, int32_t* err) {
  const ssize_t k = read(((FdReader*)u)->fd, p, (size_t)n);
  if (k < 0) {
    *err = RC_USER_BASE + 1;
    return 0;
  }
  *err = k == 0 ? RC_EOF : RC_NIL;
  return k;
}
static int32_t fd_close(void* u) {
  close(((FdReader*)u)->fd);
  return RC_NIL;
}
struct MemReader {
  const uint8_t* a;
  uint64_t na;
  const uint8_t* b;
  uint64_t nb, pos;
};
static int64_t mem_read(void* u, uint8_t* p, int64_t n, int32_t* err) {
  MemReader* m = (MemReader*)u;
  int64_t k = 0;
  while (k < n && m->pos < m->na + m->nb) {
    const bool first = m->pos < m->na;
    const uint8_t* src = first ? m->a + m->pos : m->b + (m->pos - m->na);
    const uint64_t avail = first ? m->na - m->pos : m->na + m->nb - m->pos;
    const uint64_t c = std::min<uint64_t>(avail, (uint64_t)(n - k));
    memcpy(p + k, src, c);
    k += (int64_t)c;
    m->pos += c;
  }
  *err = m->pos >= m->na + m->nb ? RC_EOF : RC_NIL;
  return k;
}
static int32_t mem_close(void*) { return RC_NIL; }

static const int kSubdirs = 64;
// which engine is behind the C ABI: librclone_crypt.so (the GPU), or the CPU baseline build of this
// same harness over tests/native/cpu_engine.cpp (-DE2E_ENGINE=\"cpu\")
#ifndef E2E_ENGINE
#define E2E_ENGINE "gpu"
#endif

// EncryptFileName / DecryptFileName for every object in one batch (rc_names_run: one EME launch)
static bool names_batch(rc_cipher* c, int32_t op, const std::vector<const std::string*>& in, std::vector<std::string>& out) {
  std::vector<const char*> p(in.size());
  std::vector<uint64_t> l(in.size());
  for (size_t i = 0; i < in.size(); i++) {
    p[i] = in[i]->data();
    l[i] = in[i]->size();
  }
  rc_names* r = nullptr;
  if (rc_names_run(c, op, in.size(), p.data(), l.data(), &r) != RC_NIL) return false;
  out.resize(in.size());
  bool ok = true;
  for (size_t i = 0; i < in.size(); i++) {
    const char* s;
    uint64_t n;
    int32_t e;
    int64_t a;
    rc_names_get(r, i, &s, &n, &e, &a);
    if (e != RC_NIL) ok = false;
    out[i].assign(s, n);
  }
  rc_names_free(r);
  return ok;
}

int main(int argc, char** argv) {
  double gib = 8.0;
  std::string dir = "/tmp/rc_e2e_src", mode = "batch";
  int transfers = 16, check_dst = 1, keep = 0, nlanes = 4, checkers = 8, hash_threads = 0;
  uint64_t group_mib = 4096;
  std::string anchor, tee_all, devices, tee_mode = "encrypter", check_mode = "batch", put_check = "inline";
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto nx = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--gib") gib = atof(nx().c_str());
    else if (a == "--dir") dir = nx();
    else if (a == "--transfers") transfers = atoi(nx().c_str());
    else if (a == "--mode") mode = nx();
    else if (a == "--check-dst-hash") check_dst = atoi(nx().c_str());
    else if (a == "--group-mib") group_mib = strtoull(nx().c_str(), nullptr, 10);
    else if (a == "--keep") keep = 1;
    else if (a == "--lanes") nlanes = std::max(1, atoi(nx().c_str()));
    else if (a == "--anchor") anchor = nx();
    else if (a == "--tee-all") tee_all = nx();
    else if (a == "--devices") devices = nx();
    else if (a == "--tee") tee_mode = nx();
    else if (a == "--check-mode") check_mode = nx();
    else if (a == "--checkers") checkers = std::max(1, atoi(nx().c_str()));
    else if (a == "--put-check") put_check = nx();
    else if (a == "--hash-threads") hash_threads = std::max(1, atoi(nx().c_str()));
    else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (mode != "batch" && mode != "stream") return 2;
  if (tee_mode != "encrypter" && tee_mode != "reader") return 2;
  if (check_mode != "batch" && check_mode != "stream") return 2;
  if (put_check != "inline" && put_check != "after") return 2;
  if (!hash_threads) hash_threads = transfers;
  const bool inline_check = check_dst && put_check == "inline";
  std::vector<int> devs;
  if (!devices.empty()) {
    setenv("RCLONE_AMD_DEVICES", devices.c_str(), 1);  // rc_* handles and name engines
    for (const char* p = devices.c_str(); *p;) {
      char* end = nullptr;
      const long d = strtol(p, &end, 10);
      if (end == p) break;
      devs.push_back((int)d);
      p = end;
      while (*p == ',') p++;
    }
  }
  if (devs.empty()) devs.push_back(0);
  // ---- local tree
  std::vector<Obj> objs;
  {
    uint64_t s = 0x5EED, total = 0;
    const uint64_t edge[4] = {0, 1, 65536, 65537};
    for (int i = 0; i < 4; i++) {
      Obj o;
      o.size = edge[i];
      objs.push_back(o);
      total += edge[i];
    }
    const double lo = std::log(4096.0), hi = std::log(8.0 * 1048576.0);
    while ((double)total < gib * 1073741824.0) {
      const double u = (double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0);
      Obj o;
      o.size = (uint64_t)std::exp(lo + u * (hi - lo));
      total += o.size;
      objs.push_back(o);
    }
    for (size_t i = 0; i < objs.size(); i++) {
      objs[i].rel = "d" + std::to_string(i % kSubdirs) + "/f" + std::to_string(i) + ".dat";
      objs[i].name = dir + "/" + objs[i].rel;
    }
  }
  mkdir(dir.c_str(), 0755);
  for (int d = 0; d < kSubdirs; d++) mkdir((dir + "/d" + std::to_string(d)).c_str(), 0755);
  uint64_t total = 0;
  for (auto& o : objs) total += o.size;
  const double tg0 = now();
  parallel_for(objs.size(), transfers, [&](size_t i) {
    std::vector<uint8_t> b(objs[i].size);
    uint64_t s = 0xF11E0000ull + i;
    for (uint64_t k = 0; k < b.size(); k += 8) {
      const uint64_t v = splitmix(s);
      memcpy(b.data() + k, &v, std::min<uint64_t>(8, b.size() - k));
    }
    const int fd = open(objs[i].name.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0 || write(fd, b.data(), b.size()) != (ssize_t)b.size()) {
      fprintf(stderr, "cannot write %s\n", objs[i].name.c_str());
      exit(1);
    }
    close(fd);
  });
  const double t_gen = now() - tg0;
  fprintf(stderr, "e2e: tree of %zu objects written in %.1f s\n", objs.size(), t_gen);

  int32_t err = 0;
  rc_cipher* c = rc_cipher_new("potato", "", &err);
  if (!c) {
    fprintf(stderr, "rc_cipher_new failed %d\n", err);
    return 1;
  }
  uint8_t key[32], nk[32], nt[16];
  rc_cipher_keys(c, key, nk, nt);
  // memory remote arena (pinned, so D2H lands in it directly)
  std::vector<uint64_t> lens(objs.size()), boff(objs.size());
  uint64_t arena_bytes = 0;
  for (size_t i = 0; i < objs.size(); i++) {
    lens[i] = objs[i].size;
    boff[i] = arena_bytes;
    arena_bytes += r16(body_bytes(objs[i].size));
  }
  uint8_t* arena = (uint8_t*)xs_host_alloc(arena_bytes ? arena_bytes : 16);
  if (!arena) {
    fprintf(stderr, "arena alloc failed: %s\n", xs_last_error());
    return 1;
  }
  for (size_t i = 0; i < objs.size(); i++) {
    objs[i].body = arena + boff[i];
    objs[i].body_len = body_bytes(objs[i].size);
  }
  // groups of whole files, <= group_mib of plaintext (a larger file is a group of its own)
  std::vector<std::pair<size_t, size_t>> groups;
  for (size_t i = 0; i < objs.size();) {
    size_t j = i;
    uint64_t g = 0;
    while (j < objs.size() && (j == i || g + r16(objs[j].size) <= (group_mib << 20))) g += r16(objs[j++].size);
    groups.push_back({i, j});
    i = j;
  }
  uint64_t max_group = 0;
  for (auto& g : groups) {
    uint64_t b = 0;
    for (size_t i = g.first; i < g.second; i++) b += r16(objs[i].size);
    max_group = std::max(max_group, b);
  }
  std::vector<uint8_t> nonces(24 * objs.size());
  if (getrandom(nonces.data(), nonces.size(), 0) != (ssize_t)nonces.size()) return 1;  // crypto/rand
  for (size_t i = 0; i < objs.size(); i++) {
    memcpy(objs[i].header, kMagic, 8);
    memcpy(objs[i].header + 8, nonces.data() + 24 * i, 24);
  }
  // lanes (engine + pinned group staging) serve the batch shapes only
  const int lanes = (mode == "batch" || check_mode == "batch") ? nlanes : 0;
  std::vector<xs_engine*> eng(lanes);
  std::vector<uint8_t*> stage(lanes);
  for (int l = 0; l < lanes; l++) {
    eng[l] = xs_engine_create(devs[l % devs.size()], 256, 1);
    stage[l] = (uint8_t*)xs_host_alloc(max_group ? max_group : 16);
    if (!eng[l] || !stage[l]) {
      fprintf(stderr, "engine/staging: %s\n", xs_last_error());
      return 1;
    }
  }
  std::atomic<int> failures{0};
  std::mutex tmu;
  double t_read = 0, t_gpu = 0;  // summed over lanes (per phase: reset below)
  // one group through one lane: parallel file reads into staging, then `gpu` on it
  auto run_groups = [&](const std::function<void(int lane, size_t g, const std::vector<uint64_t>& offs)>& gpu) {
    std::vector<std::thread> th;
    for (int l = 0; l < lanes; l++)
      th.emplace_back([&, l] {
        for (size_t g = l; g < groups.size(); g += lanes) {
          const size_t a = groups[g].first, b = groups[g].second;
          std::vector<uint64_t> offs(b - a);
          uint64_t pos = 0;
          for (size_t i = a; i < b; i++) {
            offs[i - a] = pos;
            pos += r16(objs[i].size);
          }
          const double t0 = now();
          parallel_for(b - a, std::max(1, transfers / lanes), [&](size_t k) {
            if (!read_file(objs[a + k].name, stage[l] + offs[k], objs[a + k].size)) failures++;
          });
          const double t1 = now();
          gpu(l, g, offs);
          std::lock_guard<std::mutex> lk(tmu);
          t_read += t1 - t0;
          t_gpu += now() - t1;
        }
      });
    for (auto& t : th) t.join();
  };
  // ---- sync
  double t_sync = 0, t_dst = 0, sync_read = 0, sync_gpu = 0, t_names_enc = 0, t_names_dec = 0;
  double t_puts = 0;  // to the last stored object (put's own hash checks not awaited)
  uint64_t put_mismatch = 0, name_mismatch = 0;
  std::atomic<uint64_t> bad_put{0};
  // crypt.put's tail (crypt.go:542-560): the remote's MD5 of what it stored vs the tee hash
  auto put_check_one = [&](size_t i) {
    dst_hash(objs[i]);
    if (memcmp(objs[i].tee, objs[i].dst, 16)) bad_put++;
  };
  const double tn0 = now();
  {  // crypt.Put's remote name: EncryptFileName(rel) for the whole listing (crypt.go:517)
    std::vector<const std::string*> in(objs.size());
    std::vector<std::string> out;
    for (size_t i = 0; i < objs.size(); i++) in[i] = &objs[i].rel;
    if (!names_batch(c, RC_OP_ENCRYPT_FILE_NAME, in, out)) failures++;
    for (size_t i = 0; i < objs.size() && i < out.size(); i++) objs[i].remote = std::move(out[i]);
  }
  t_names_enc = now() - tn0;
  if (mode == "batch") {
    const double t0 = now();
    // inline put checks: workers take each object as soon as its group is stored
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<size_t> q;
    bool closing = false;
    std::vector<std::thread> hashers;
    if (inline_check)
      for (int t = 0; t < hash_threads; t++)
        hashers.emplace_back([&] {
          for (;;) {
            size_t i;
            {
              std::unique_lock<std::mutex> lk(qmu);
              qcv.wait(lk, [&] { return closing || !q.empty(); });
              if (q.empty()) return;
              i = q.front();
              q.pop_front();
            }
            put_check_one(i);
          }
        });
    run_groups([&](int l, size_t g, const std::vector<uint64_t>& offs) {
      const size_t a = groups[g].first, n = groups[g].second - a;
      std::vector<uint8_t> md5(16 * n);
      if (xs_engine_put_batch(eng[l], key, n, nonces.data() + 24 * a, offs.data(), lens.data() + a, stage[l],
                              arena + boff[a], md5.data()) != XS_OK) {
        fprintf(stderr, "put_batch: %s\n", xs_last_error());
        failures++;
        return;
      }
      for (size_t k = 0; k < n; k++) memcpy(objs[a + k].tee, md5.data() + 16 * k, 16);
      if (inline_check) {
        {
          std::lock_guard<std::mutex> lk(qmu);
          for (size_t k = 0; k < n; k++) q.push_back(a + k);
        }
        qcv.notify_all();
      }
    });
    t_puts = now() - t0 + t_names_enc;
    {
      std::lock_guard<std::mutex> lk(qmu);
      closing = true;
    }
    qcv.notify_all();
    for (auto& t : hashers) t.join();
    t_sync = now() - t0 + t_names_enc;
    sync_read = t_read;
    sync_gpu = t_gpu;
  } else {
    const bool tee_on_enc = tee_mode == "encrypter";
    const double t0 = now();
    parallel_for(objs.size(), transfers, [&](size_t i) {
      Obj& o = objs[i];
      FdReader fr{open(o.name.c_str(), O_RDONLY)};
      if (fr.fd < 0) {
        failures++;
        return;
      }
      rc_reader r{fd_read, nullptr, nullptr, &fr};  // the encrypter does not close its source
      int32_t e = 0;
      rc_encrypter* h = rc_encrypt_data(c, r, nonces.data() + 24 * i, &e);
      if (!h || (tee_on_enc && rc_encrypter_set_md5(h, 1) != RC_NIL)) {
        failures++;
        if (h) rc_encrypter_free(h);
        fd_close(&fr);
        return;
      }
      // the memory backend's Put reads the stream into the object's buffer (io.ReadAll): header,
      // then the wire body straight into the remote's arena; crypt.put tees the MD5 of what it
      // read -- in the encrypter, or here on the reading thread (TeeReader)
      Md5 tee;
      uint64_t got = 0;
      const uint64_t want = 32 + o.body_len;
      for (;;) {
        uint8_t* dst = got < 32 ? o.header + got : o.body + (got - 32);
        const uint64_t room = got < 32 ? 32 - got : want - got;
        uint8_t probe;  // past the end: the read that returns EOF
        const int64_t k = rc_encrypter_read(h, room ? dst : &probe, room ? (int64_t)std::min<uint64_t>(room, 1 << 20) : 1, &e);
        if (k > 0 && !room) {
          got = want + 1;  // longer than the object: a failure
          break;
        }
        if (!tee_on_enc && k > 0) tee.update(dst, (size_t)k);
        got += (uint64_t)k;
        if (e != RC_NIL) break;
      }
      if (tee_on_enc) e = e == RC_EOF && rc_encrypter_md5(h, o.tee) == RC_NIL ? RC_EOF : RC_ERR_INVALID;
      else tee.final(o.tee);
      rc_encrypter_free(h);
      fd_close(&fr);
      if (e != RC_EOF || got != want || memcmp(o.header, kMagic, 8) || memcmp(o.header + 8, nonces.data() + 24 * i, 24)) {
        failures++;
        return;
      }
      if (inline_check) put_check_one(i);  // the same transfer, before Put returns
    });
    t_sync = now() - t0 + t_names_enc;
    t_puts = t_sync;
  }
  if (check_dst && !inline_check) {  // --put-check after: the checks as a phase of their own
    const double t0 = now();
    parallel_for(objs.size(), transfers, put_check_one);
    t_dst = now() - t0;
    t_puts = t_sync;
    t_sync += t_dst;
  }
  if (check_dst) fprintf(stderr, "e2e: sync %.1f s with put checks (%s), puts alone %.1f s\n", t_sync, put_check.c_str(), t_puts);
  put_mismatch = bad_put;
  // ---- cryptcheck: re-seal each local file with the stored nonce, MD5 on the GPU, compare
  auto cryptcheck = [&](std::vector<uint8_t>& differ) {
    differ.assign(objs.size(), 0);
    if (check_mode == "stream") {  // cmd/cryptcheck as is: --checkers goroutines, one object each
      parallel_for(objs.size(), checkers, [&](size_t i) {
        Obj& o = objs[i];
        dst_hash(o);  // underlyingDst.Hash (memory.go:580-588; cached by put's check)
        // ComputeHash (crypt.go:816-852): open the stored object's header range, newDecrypter
        // reads the nonce, close; then computeHashWithNonce over the opened source
        MemReader hr{o.header, 32, nullptr, 0, 0};
        int32_t e = 0;
        rc_decrypter* d = rc_decrypt_data(c, rc_reader{mem_read, mem_close, nullptr, &hr}, &e);
        if (!d) {
          failures++;
          return;
        }
        uint8_t nonce[24], md5[16];
        rc_decrypter_nonce(d, nonce);
        e = rc_decrypter_close(d);
        rc_decrypter_free(d);
        FdReader fr{open(o.name.c_str(), O_RDONLY)};
        if (e != RC_NIL || fr.fd < 0) {
          failures++;
          if (fr.fd >= 0) close(fr.fd);
          return;
        }
        if (rc_compute_hash_with_nonce(c, rc_reader{fd_read, fd_close, nullptr, &fr}, nonce, md5) != RC_NIL) {
          failures++;
          return;
        }
        differ[i] = memcmp(md5, o.dst, 16) != 0;
      });
      return;
    }
    run_groups([&](int l, size_t g, const std::vector<uint64_t>& offs) {
      const size_t a = groups[g].first, n = groups[g].second - a;
      std::vector<uint8_t> ns(24 * n), md5(16 * n);
      for (size_t k = 0; k < n; k++) memcpy(ns.data() + 24 * k, objs[a + k].header + 8, 24);  // nonce from the remote
      if (xs_engine_seal_md5(eng[l], key, n, ns.data(), offs.data(), lens.data() + a, stage[l], md5.data()) != XS_OK) {
        failures++;
        return;
      }
      for (size_t k = 0; k < n; k++) {
        Obj& o = objs[a + k];
        dst_hash(o);  // underlying object's hash (cached by put's check)
        differ[a + k] = memcmp(md5.data() + 16 * k, o.dst, 16) != 0;
      }
    });
  };
  std::vector<uint8_t> differ;
  t_read = t_gpu = 0;
  const double tc0 = now();
  {  // cryptcheck lists crypt: -> DecryptFileName of every remote key, matched to the source paths
    std::vector<const std::string*> in(objs.size());
    std::vector<std::string> out;
    for (size_t i = 0; i < objs.size(); i++) in[i] = &objs[i].remote;
    if (!names_batch(c, RC_OP_DECRYPT_FILE_NAME, in, out)) failures++;
    for (size_t i = 0; i < objs.size() && i < out.size(); i++) name_mismatch += out[i] != objs[i].rel;
  }
  t_names_dec = now() - tc0;
  cryptcheck(differ);
  const double t_check = now() - tc0, check_read = t_read, check_gpu = t_gpu;
  fprintf(stderr, "e2e: cryptcheck %.1f s\n", t_check);
  uint64_t ndiff = 0;
  for (auto d : differ) ndiff += d;
  // ---- verify: decrypt sampled objects through rc_decrypt_data and compare with the files
  uint64_t verified = 0, verify_bad = 0;
  for (size_t i = 0; i < objs.size(); i += std::max<size_t>(1, objs.size() / 64)) {
    Obj& o = objs[i];
    MemReader mr{o.header, 32, o.body, o.body_len, 0};
    rc_reader r{mem_read, mem_close, nullptr, &mr};
    int32_t e = 0;
    rc_decrypter* d = rc_decrypt_data(c, r, &e);
    std::vector<uint8_t> want(o.size), got(o.size + 1);
    if (!d || !read_file(o.name, want.data(), o.size)) {
      verify_bad++;
      continue;
    }
    uint64_t n = 0;
    for (;;) {
      const int64_t k = rc_decrypter_read(d, got.data() + n, (int64_t)(got.size() - n), &e);
      n += (uint64_t)k;
      if (e != RC_NIL || n == got.size()) break;
    }
    rc_decrypter_close(d);
    rc_decrypter_free(d);
    if (n != o.size || memcmp(got.data(), want.data(), o.size) || (e != RC_EOF && e != RC_NIL)) verify_bad++;
    verified++;
  }
  uint64_t tee_listed = 0;
  if (!tee_all.empty()) {  // before the corruption below
    FILE* f = fopen(tee_all.c_str(), "w");
    if (!f) {
      failures++;
    } else {
      for (size_t i = 0; i < objs.size(); i++) {
        const Obj& o = objs[i];
        fprintf(f, "%zu %llu %llu %s %s\n", i, (unsigned long long)o.size, (unsigned long long)(0xF11E0000ull + i),
                hexs(o.header + 8, 24).c_str(), hexs(o.tee, 16).c_str());
        tee_listed++;
      }
      fclose(f);
    }
  }
  uint64_t anchored = 0;
  if (!anchor.empty()) {  // before the corruption below: the objects as sync stored them
    std::vector<size_t> pick = {0, 1, 2, 3};
    for (size_t i = 4; i < objs.size(); i += std::max<size_t>(1, objs.size() / 64)) pick.push_back(i);
    size_t largest = 0;
    for (size_t i = 0; i < objs.size(); i++)
      if (objs[i].size > objs[largest].size) largest = i;
    pick.push_back(largest);
    pick.push_back(objs.size() - 1);
    std::sort(pick.begin(), pick.end());
    pick.erase(std::unique(pick.begin(), pick.end()), pick.end());
    FILE* f = fopen(anchor.c_str(), "w");
    if (!f) {
      failures++;
    } else {
      for (size_t i : pick) {
        const Obj& o = objs[i];
        Sha256 h;
        h.update(o.header, 32);
        h.update(o.body, o.body_len);
        uint8_t d[32];
        h.final(d);
        fprintf(f, "{\"index\": %zu, \"size\": %llu, \"seed\": %llu, \"nonce\": \"%s\", \"sha256\": \"%s\", "
                "\"tee_md5\": \"%s\"}\n", i, (unsigned long long)o.size, (unsigned long long)(0xF11E0000ull + i),
                hexs(o.header + 8, 24).c_str(), hexs(d, 32).c_str(), hexs(o.tee, 16).c_str());
        anchored++;
      }
      fclose(f);
    }
  }
  // corruption: flip one ciphertext byte of one stored object, drop its cached hash
  size_t victim = objs.size() / 2;
  while (victim < objs.size() && objs[victim].body_len < 100) victim++;
  uint64_t flagged = 0;
  bool only_victim = false;
  if (victim < objs.size()) {
    objs[victim].body[objs[victim].body_len / 2] ^= 0x01;
    objs[victim].dst_ok = false;
    std::vector<uint8_t> d2;
    cryptcheck(d2);
    for (auto d : d2) flagged += d;
    only_victim = flagged == 1 && d2[victim];
  }
  const bool ok = failures == 0 && put_mismatch == 0 && ndiff == 0 && verify_bad == 0 && only_victim && name_mismatch == 0;
  const double g = (double)total / 1073741824.0;
  printf("{\"config\": \"configs[4] e2e: sync local tree -> crypt(memory), cryptcheck\", \"engine\": \"" E2E_ENGINE "\", "
         "\"mode\": \"%s\", "
         "\"tee\": \"%s\", \"check_mode\": \"%s\", \"checkers\": %d, "
         "\"objects\": %zu, \"gib\": %.3f, \"transfers\": %d, \"lanes\": %d, \"group_mib\": %llu, "
         "\"put_check\": \"%s\", \"hash_threads\": %d, "
         "\"sync_s\": %.3f, \"sync_GiB_s\": %.2f, \"put_only_s\": %.3f, \"put_only_GiB_s\": %.2f, \"dst_hash_phase_s\": %.3f, "
         "\"cryptcheck_s\": %.3f, \"cryptcheck_GiB_s\": %.2f, \"put_hash_mismatches\": %llu, "
         "\"cryptcheck_differences\": %llu, \"verified_objects\": %llu, \"verify_failures\": %llu, "
         "\"corruption_flagged\": %llu, \"names_encrypt_s\": %.4f, \"names_decrypt_s\": %.4f, "
         "\"name_mismatches\": %llu, \"example_remote_name\": \"%s\", "
         "\"anchored_objects\": %llu, \"tee_listed\": %llu, \"devices\": \"%s\", \"tree_write_s\": %.2f, \"lane_seconds\": {\"sync_read\": %.3f, "
         "\"sync_gpu\": %.3f, \"check_read\": %.3f, \"check_gpu\": %.3f}, \"ok\": %s}\n",
         mode.c_str(), mode == "stream" ? tee_mode.c_str() : E2E_ENGINE, check_mode.c_str(), checkers, objs.size(), g, transfers, lanes, (unsigned long long)group_mib,
         check_dst ? put_check.c_str() : "off", hash_threads, t_sync, g / t_sync, t_puts, g / t_puts, t_dst, t_check, g / t_check, (unsigned long long)put_mismatch,
         (unsigned long long)ndiff, (unsigned long long)verified, (unsigned long long)verify_bad,
         (unsigned long long)flagged, t_names_enc, t_names_dec, (unsigned long long)name_mismatch,
         objs.empty() ? "" : objs.back().remote.c_str(), (unsigned long long)anchored, (unsigned long long)tee_listed, devices.c_str(), t_gen, sync_read, sync_gpu, check_read, check_gpu, ok ? "true" : "false");
  for (int l = 0; l < lanes; l++) {
    xs_engine_destroy(eng[l]);
    xs_host_free(stage[l]);
  }
  xs_host_free(arena);
  rc_cipher_free(c);
  if (!keep) {
    for (auto& o : objs) unlink(o.name.c_str());
    for (int d = 0; d < kSubdirs; d++) rmdir((dir + "/d" + std::to_string(d)).c_str());
    rmdir(dir.c_str());
  }
  return ok ? 0 : 1;
}
