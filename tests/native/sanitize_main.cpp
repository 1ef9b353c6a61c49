// TEST INFRASTRUCTURE: sanitizer harness for the host C++ of the drop-in.
//
// Built by tests/native/Makefile twice -- with AddressSanitizer + UBSan and with ThreadSanitizer --
// from rclone_amd/csrc/{cipher,names,scrypt}.cpp plus tests/native/stub_engine.cpp (the GPU side
// replaced by the CPU oracle), and run by tests/test_native_sanitize.py.  It drives the rc_* C ABI
// the way backend/crypt/cipher_test.go drives cipher.go and feeds it malformed input:
//   * stream round trips against orc_encrypt_file, every read-ahead / batch / reader-chunk shape
//     (testEncryptDecrypt, cipher_test.go:1080-1121);
//   * truncated crypt files at every length near the header and block edges, and bit flips in
//     magic, nonce, tags and payload, with and without pass_bad_blocks (TestDecrypterRead
//     :1485-1560): the error value and the bytes served before it are checked exactly;
//   * reader errors passed through at every position class (:1194-1205, :1266-1280);
//   * a seek / limit grid through DecryptDataSeek and RangeSeek (TestNewDecrypterSeekLimit
//     :1282-1431);
//   * the name cipher's decoders and Decrypt{File,Dir}Name on random and crafted garbage in
//     every mode and encoding (cipher_test.go:273-336), plus encrypt/decrypt round trips;
//   * concurrency (meaningful under TSan): many encrypters/decrypters sharing one cipher on
//     several threads, and one rc_names_run batch over 16 host threads.
// Exit status 0 and a final "sanitize ok" line mean every check passed.
#include <sched.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rclone_crypt_gpu.h"
#include "../../rclone_amd/csrc/xs_host_md5.h"
#include "../../rclone_amd/csrc/xs_topo.h"
#include "../../rclone_amd/csrc/md5_workers.h"

extern "C" {
void orc_encrypt_file(uint8_t* out, const uint8_t* in, int64_t len, const uint8_t nonce0[24], const uint8_t key[32]);
void orc_nonce_add(uint8_t n[24], uint64_t x);
// stub_engine.cpp's failure injection
long stub_engine_submissions(void);
long stub_engine_failed(void);
void stub_engine_fail(long from, long count);
}

static int g_fail = 0;
static std::atomic<long> g_checks{0};
#define CHECK(cond, ...)                                   \
  do {                                                     \
    g_checks++;                                            \
    if (!(cond)) {                                         \
      if (g_fail++ < 30) {                                 \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                      \
        fprintf(stderr, "\n");                             \
      }                                                    \
    }                                                      \
  } while (0)

static uint64_t g_rng = 0x5EED;
static uint64_t rnd() {
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static std::vector<uint8_t> rbytes(size_t n) {
  std::vector<uint8_t> v(n);
  for (auto& b : v) b = (uint8_t)rnd();
  return v;
}

// ---------------------------------------------------------------- readers (user = handle)
struct Src {
  const uint8_t* p = nullptr;
  size_t n = 0, pos = 0;
  size_t chunk = 1 << 30;
  int64_t fail_at = -1;  // return a user error once pos reaches this
  int32_t fail_err = RC_USER_BASE + 5;
  int reads = 0, closes = 0;
};
static int64_t src_read(void* u, uint8_t* p, int64_t want, int32_t* err) {
  Src* s = (Src*)u;
  s->reads++;
  if (s->fail_at >= 0 && (int64_t)s->pos >= s->fail_at) {
    *err = s->fail_err;
    return 0;
  }
  size_t k = s->n - s->pos;
  if (k > (size_t)want) k = (size_t)want;
  if (k > s->chunk) k = s->chunk;
  if (s->fail_at >= 0 && (int64_t)(s->pos + k) > s->fail_at) k = (size_t)s->fail_at - s->pos;
  if (k) memcpy(p, s->p + s->pos, k);
  s->pos += k;
  *err = (k == 0 && s->pos == s->n) ? RC_EOF : RC_NIL;
  return (int64_t)k;
}
static int32_t src_close(void* u) {
  ((Src*)u)->closes++;
  return RC_NIL;
}
static rc_reader mk(Src* s) { return rc_reader{src_read, src_close, nullptr, s}; }
// a source whose Close fails (fs.CheckClose must surface it when nothing else failed)
static int32_t src_close_fail(void* u) {
  ((Src*)u)->closes++;
  return RC_USER_BASE + 9;
}
static std::vector<uint8_t> md5_of(const uint8_t* p, size_t n) {
  xs::HostMd5 m;
  m.update(p, n);
  std::vector<uint8_t> d(16);
  m.final(d.data());
  return d;
}

// read a whole stream with varying read sizes; returns the final error
static int32_t drain_enc(rc_encrypter* e, std::vector<uint8_t>& out) {
  int32_t err = RC_NIL;
  static const int64_t sizes[] = {1, 31, 32, 100, 65536, 65537, 4096, 7};
  for (int k = 0;; k++) {
    uint8_t buf[70000];
    int64_t n = rc_encrypter_read(e, buf, sizes[k % 8], &err);
    out.insert(out.end(), buf, buf + n);
    if (err != RC_NIL) return err;
  }
}
static int32_t drain_dec(rc_decrypter* d, std::vector<uint8_t>& out) {
  int32_t err = RC_NIL;
  static const int64_t sizes[] = {65536, 1, 4096, 65537, 7, 131072};
  for (int k = 0;; k++) {
    std::vector<uint8_t> buf(sizes[k % 6]);
    int64_t n = rc_decrypter_read(d, buf.data(), (int64_t)buf.size(), &err);
    out.insert(out.end(), buf.begin(), buf.begin() + n);
    if (err != RC_NIL) return err;
  }
}

static std::vector<uint8_t> oracle_file(const std::vector<uint8_t>& plain, const uint8_t nonce[24], const uint8_t key[32]) {
  std::vector<uint8_t> f((size_t)rc_encrypted_size((int64_t)plain.size()));
  orc_encrypt_file(f.data(), plain.data(), (int64_t)plain.size(), nonce, key);
  return f;
}

// ---------------------------------------------------------------- data path
static void test_round_trips(rc_cipher* c, const uint8_t key[32]) {
  const size_t lens[] = {0, 1, 15, 16, 17, 65535, 65536, 65537, 131075, 300001};
  const size_t chunks[] = {7, 4096, 65537, 1 << 30};
  const uint32_t batches[] = {1, 3, 64};
  for (size_t L : lens)
    for (size_t ch : chunks)
      for (uint32_t b : batches)
        for (uint32_t ra : {1u, 0u}) {
          if (ch == 7 && L > 70000) continue;
          std::vector<uint8_t> plain = rbytes(L);
          std::vector<uint8_t> nonce = rbytes(24);
          if (L == 300001) memset(nonce.data(), 0xFF, 8);  // block adds carry out of byte 7
          rc_cipher_set_batch_blocks(c, b);
          rc_cipher_set_readahead(c, ra);
          Src s;
          s.p = plain.data();
          s.n = L;
          s.chunk = ch;
          int32_t err = 0;
          rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
          CHECK(e && err == RC_NIL, "encrypt_data err %d", err);
          if (!e) continue;
          std::vector<uint8_t> ct;
          err = drain_enc(e, ct);
          const std::vector<uint8_t> want = oracle_file(plain, nonce.data(), key);
          CHECK(err == RC_EOF && ct == want, "encrypt L=%zu chunk=%zu batch=%u ra=%u err=%d len=%zu/%zu", L, ch, b, ra,
                err, ct.size(), want.size());
          uint8_t fin[24], exp[24];
          rc_encrypter_nonce(e, fin);
          memcpy(exp, nonce.data(), 24);
          orc_nonce_add(exp, (L + 65535) / 65536);
          CHECK(!memcmp(fin, exp, 24), "final nonce L=%zu", L);
          rc_encrypter_free(e);
          Src d;
          d.p = want.data();
          d.n = want.size();
          d.chunk = ch;
          rc_decrypter* h = rc_decrypt_data(c, mk(&d), &err);
          CHECK(h && err == RC_NIL, "decrypt_data err %d", err);
          if (!h) continue;
          std::vector<uint8_t> pt;
          err = drain_dec(h, pt);
          CHECK(err == RC_EOF && pt == plain, "decrypt L=%zu chunk=%zu batch=%u err=%d", L, ch, b, err);
          CHECK(rc_decrypter_close(h) == RC_NIL && d.closes == 1, "close");
          CHECK(rc_decrypter_close(h) == RC_ERR_FILE_CLOSED && d.closes == 1, "second close");
          rc_decrypter_free(h);
        }
  rc_cipher_set_batch_blocks(c, 64);
  rc_cipher_set_readahead(c, 1);
}

// What the reference returns for a (possibly damaged) crypt file, block by block
// (cipher.go:793-818 newDecrypter, :862-898 fillBuffer).
static void expect_damaged(const std::vector<uint8_t>& f, const std::vector<uint8_t>& plain, int64_t bad_block,
                           bool pass_bad, std::vector<uint8_t>& bytes, int32_t* err, bool* open_fails) {
  bytes.clear();
  *open_fails = false;
  if (f.size() < 32) {
    *open_fails = true;
    *err = RC_ERR_FILE_TOO_SHORT;
    return;
  }
  if (memcmp(f.data(), "RCLONE\0\0", 8)) {
    *open_fails = true;
    *err = RC_ERR_BAD_MAGIC;
    return;
  }
  size_t pos = 32;
  for (int64_t b = 0;; b++) {
    if (pos >= f.size()) {
      *err = RC_EOF;
      return;
    }
    size_t n = f.size() - pos < 65552 ? f.size() - pos : 65552;
    if (n <= 16) {
      *err = RC_ERR_FILE_BAD_HEADER;
      return;
    }
    const size_t plen = n - 16;
    const bool intact = b != bad_block && (size_t)(b * 65536) + plen <= plain.size() &&
                        (n == 65552 || pos + n == 32 + plain.size() + 16 * ((plain.size() + 65535) / 65536));
    if (!intact) {
      if (!pass_bad) {
        *err = RC_ERR_BAD_BLOCK;
        return;
      }
      bytes.insert(bytes.end(), plen, 0);
    } else {
      bytes.insert(bytes.end(), plain.begin() + b * 65536, plain.begin() + b * 65536 + plen);
    }
    pos += n;
  }
}

static void run_damaged(rc_cipher* c, const std::vector<uint8_t>& f, const std::vector<uint8_t>& plain, int64_t bad,
                        bool pass, const char* what, size_t arg) {
  std::vector<uint8_t> want;
  int32_t werr;
  bool wopen;
  expect_damaged(f, plain, bad, pass, want, &werr, &wopen);
  rc_cipher_set_pass_bad_blocks(c, pass);
  Src s;
  s.p = f.data();
  s.n = f.size();
  s.chunk = 1000 + (arg % 70000);
  int32_t err = 0;
  rc_decrypter* h = rc_decrypt_data(c, mk(&s), &err);
  if (wopen) {
    CHECK(!h && err == werr && s.closes == 1, "%s %zu: open err %d want %d closes %d", what, arg, err, werr, s.closes);
    if (h) rc_decrypter_free(h);
    return;
  }
  CHECK(h && err == RC_NIL, "%s %zu: open failed %d", what, arg, err);
  if (!h) return;
  std::vector<uint8_t> got;
  err = drain_dec(h, got);
  CHECK(err == werr && got == want, "%s %zu (pass=%d): err %d want %d, %zu bytes want %zu", what, arg, pass, err, werr,
        got.size(), want.size());
  rc_decrypter_close(h);
  rc_decrypter_free(h);
  rc_cipher_set_pass_bad_blocks(c, 0);
}

static void test_damaged(rc_cipher* c, const uint8_t key[32]) {
  const std::vector<uint8_t> plain = rbytes(150000);
  const std::vector<uint8_t> nonce = rbytes(24);
  const std::vector<uint8_t> f = oracle_file(plain, nonce.data(), key);
  // truncation: every length near the header and the block edges, a stride elsewhere
  std::vector<size_t> cuts;
  for (size_t k = 0; k <= 80; k++) cuts.push_back(k);
  for (size_t e : {(size_t)32 + 65552, (size_t)32 + 2 * 65552, f.size()})
    for (int d = -20; d <= 20; d++)
      if ((int64_t)e + d >= 0 && e + d <= f.size()) cuts.push_back(e + d);
  for (size_t k = 81; k < f.size(); k += 977) cuts.push_back(k);
  for (size_t cut : cuts) {
    std::vector<uint8_t> t(f.begin(), f.begin() + cut);
    run_damaged(c, t, plain, -1, false, "truncate", cut);
  }
  // bit flips: magic, nonce, tags, first/last payload byte of each block, random
  std::vector<size_t> pos = {0, 7, 8, 20, 31};
  for (size_t b = 0; b < 3; b++) {
    const size_t base = 32 + b * 65552;
    for (size_t o : {(size_t)0, (size_t)15, (size_t)16, (size_t)17, (size_t)65551})
      if (base + o < f.size()) pos.push_back(base + o);
  }
  pos.push_back(f.size() - 1);
  for (int k = 0; k < 40; k++) pos.push_back(rnd() % f.size());
  for (size_t p : pos)
    for (bool pass : {false, true}) {
      std::vector<uint8_t> t = f;
      t[p] ^= (uint8_t)(1u << (rnd() % 8));
      const int64_t bad = p < 32 ? 0 : (int64_t)((p - 32) / 65552);  // a nonce flip breaks every block
      if (p >= 8 && p < 32) {
        // every block's nonce is derived from the header: all blocks fail
        std::vector<uint8_t> want;
        rc_cipher_set_pass_bad_blocks(c, pass);
        Src s;
        s.p = t.data();
        s.n = t.size();
        int32_t err = 0;
        rc_decrypter* h = rc_decrypt_data(c, mk(&s), &err);
        CHECK(h != nullptr, "nonce flip open");
        if (!h) continue;
        std::vector<uint8_t> got;
        err = drain_dec(h, got);
        if (pass)
          CHECK(err == RC_EOF && got == std::vector<uint8_t>(plain.size(), 0), "nonce flip pass %zu", p);
        else
          CHECK(err == RC_ERR_BAD_BLOCK && got.empty(), "nonce flip %zu err %d", p, err);
        rc_decrypter_free(h);
        rc_cipher_set_pass_bad_blocks(c, 0);
        continue;
      }
      run_damaged(c, t, plain, bad, pass, "flip", p);
    }
}

static void test_reader_errors(rc_cipher* c, const uint8_t key[32]) {
  const std::vector<uint8_t> plain = rbytes(140000);
  const std::vector<uint8_t> nonce = rbytes(24);
  const std::vector<uint8_t> f = oracle_file(plain, nonce.data(), key);
  // encrypter: an error at plaintext position q = the reference's output for the first q bytes
  for (int64_t q : {0L, 1L, 65535L, 65536L, 65537L, 100000L, 131072L}) {
    Src s;
    s.p = plain.data();
    s.n = plain.size();
    s.fail_at = q;
    int32_t err = 0;
    rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
    if (!e) {
      CHECK(false, "encrypt_data");
      continue;
    }
    std::vector<uint8_t> ct;
    err = drain_enc(e, ct);
    std::vector<uint8_t> head(plain.begin(), plain.begin() + q);
    CHECK(err == s.fail_err && ct == oracle_file(head, nonce.data(), key), "encrypter error at %ld: err %d", (long)q,
          err);
    int32_t err2 = 0;
    uint8_t one;
    CHECK(rc_encrypter_read(e, &one, 1, &err2) == 0 && err2 == s.fail_err, "sticky encrypter error");
    rc_encrypter_free(e);
  }
  // decrypter: pending reader errors win over header / auth errors (cipher.go:874-884)
  for (int64_t q : {0L, 5L, 31L, 32L, 40L, 48L, 32L + 65552, 32L + 65552 + 10, 32L + 65552 + 16, 32L + 65552 + 17,
                    32L + 65552 + 30000}) {
    Src s;
    s.p = f.data();
    s.n = f.size();
    s.fail_at = q;
    int32_t err = 0;
    rc_decrypter* h = rc_decrypt_data(c, mk(&s), &err);
    if (q < 32) {
      CHECK(!h && err == s.fail_err && s.closes == 1, "header error at %ld: %d", (long)q, err);
      if (h) rc_decrypter_free(h);
      continue;
    }
    if (!h) {
      CHECK(false, "open at %ld", (long)q);
      continue;
    }
    std::vector<uint8_t> got;
    err = drain_dec(h, got);
    const size_t full = (size_t)(q - 32) / 65552;  // blocks that arrived whole
    std::vector<uint8_t> want(plain.begin(), plain.begin() + full * 65536);
    CHECK(err == s.fail_err && got == want, "decrypter error at %ld: err %d got %zu want %zu", (long)q, err,
          got.size(), want.size());
    rc_decrypter_free(h);
  }
}

// read-ahead (cipher.go:726-741): one block before the first data byte; then doubling, or full
// batches at once from a fast (memory) source under the default adaptive growth
static void test_readahead(rc_cipher* c) {
  const std::vector<uint8_t> plain = rbytes(40 * 65536);
  const std::vector<uint8_t> nonce = rbytes(24);
  for (uint32_t growth : {2u, 0u}) {
    rc_cipher_set_batch_blocks(c, 16);
    rc_cipher_set_readahead_growth(c, growth);
    Src s;
    s.p = plain.data();
    s.n = plain.size();
    int32_t err = 0;
    rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
    std::vector<uint8_t> buf(65536 + 64);
    rc_encrypter_read(e, buf.data(), 32, &err);
    CHECK(s.reads == 0, "reads before the header is consumed: %d", s.reads);
    rc_encrypter_read(e, buf.data(), 1, &err);
    CHECK(s.pos == 65536, "first data byte read %zu source bytes", s.pos);
    rc_encrypter_read(e, buf.data(), 65535 + 16, &err);
    rc_encrypter_read(e, buf.data(), 1, &err);
    // growth 0 jumps to full batches only after a refill read faster than 2 GB/s: a memory source
    // is that fast, except under ThreadSanitizer's instrumentation, where it may double instead
#if defined(__SANITIZE_THREAD__)
    const bool slow_ok = growth == 0 && s.pos == 3u * 65536;
#else
    const bool slow_ok = false;
#endif
    CHECK(s.pos == (growth == 2 ? 3u : 17u) * 65536 || slow_ok, "growth %u: second refill ends at %zu", growth, s.pos);
    rc_encrypter_free(e);
  }
  rc_cipher_set_batch_blocks(c, 64);
  rc_cipher_set_readahead_growth(c, 0);
}

struct OpenCtx {
  const std::vector<uint8_t>* f;
  std::vector<Src*> srcs;
  std::vector<std::pair<int64_t, int64_t>> calls;
};
static int32_t open_cb(void* u, int64_t off, int64_t lim, rc_reader* out) {
  OpenCtx* o = (OpenCtx*)u;
  o->calls.push_back({off, lim});
  Src* s = new Src();
  const size_t n = o->f->size();
  const size_t a = (size_t)off < n ? (size_t)off : n;
  size_t b = lim < 0 ? n : std::min(n, a + (size_t)lim);
  s->p = o->f->data() + a;
  s->n = b - a;
  s->chunk = 5000;
  o->srcs.push_back(s);
  *out = mk(s);
  return RC_NIL;
}

static void test_seek_grid(rc_cipher* c, const uint8_t key[32]) {
  const std::vector<uint8_t> plain = rbytes(150000);
  const std::vector<uint8_t> nonce = rbytes(24);
  const std::vector<uint8_t> f = oracle_file(plain, nonce.data(), key);
  const int64_t offs[] = {0, 1, 2, 65535, 65536, 65537, 131071, 131072, 131073, 149999, 150000};
  const int64_t lims[] = {-1, 0, 1, 65535, 65536, 65537, 131072, 150000, 1 << 30};
  for (int64_t off : offs)
    for (int64_t lim : lims) {
      OpenCtx o{&f, {}, {}};
      int32_t err = 0;
      rc_decrypter* h = rc_decrypt_data_seek(c, open_cb, &o, off, lim, &err);
      if (lim == 0 && off >= 150000) {
        if (h) rc_decrypter_free(h);
        for (auto* s : o.srcs) delete s;
        continue;
      }
      if (!h) {
        CHECK(off >= (int64_t)plain.size() && err == RC_ERR_BAD_SEEK, "seek %ld/%ld open err %d", (long)off,
              (long)lim, err);
        for (auto* s : o.srcs) delete s;
        continue;
      }
      std::vector<uint8_t> got;
      err = drain_dec(h, got);
      const size_t a = (size_t)std::min<int64_t>(off, (int64_t)plain.size());
      const size_t b = lim < 0 ? plain.size() : std::min(plain.size(), a + (size_t)lim);
      std::vector<uint8_t> want(plain.begin() + a, plain.begin() + b);
      CHECK(err == RC_EOF && got == want, "seek %ld limit %ld: err %d %zu bytes want %zu", (long)off, (long)lim, err,
            got.size(), want.size());
      // RangeSeek back to a random place on the same handle
      const int64_t o2 = (int64_t)(rnd() % 150000), l2 = (int64_t)(rnd() % 70000);
      rc_decrypter_range_seek(h, o2, 0, l2, &err);
      CHECK(err == RC_NIL, "range seek err %d", err);
      got.clear();
      err = drain_dec(h, got);
      const size_t b2 = std::min<size_t>(plain.size(), (size_t)(o2 + l2));
      CHECK(err == RC_EOF && got == std::vector<uint8_t>(plain.begin() + o2, plain.begin() + b2), "range seek %ld/%ld",
            (long)o2, (long)l2);
      rc_decrypter_close(h);
      rc_decrypter_free(h);
      for (auto* s : o.srcs) delete s;
    }
}

// ---------------------------------------------------------------- names
static std::vector<std::string> run_names(rc_cipher* c, int32_t op, const std::vector<std::string>& in,
                                          std::vector<int32_t>* errs) {
  std::vector<const char*> p(in.size());
  std::vector<uint64_t> l(in.size());
  for (size_t i = 0; i < in.size(); i++) {
    p[i] = in[i].data();
    l[i] = in[i].size();
  }
  rc_names* r = nullptr;
  std::vector<std::string> out(in.size());
  if (errs) errs->assign(in.size(), 0);
  int32_t rc = rc_names_run(c, op, in.size(), p.data(), l.data(), &r);
  CHECK(rc == RC_NIL, "rc_names_run %d", rc);
  if (rc != RC_NIL) return out;
  for (size_t i = 0; i < in.size(); i++) {
    const char* s;
    uint64_t n;
    int32_t e;
    int64_t a;
    rc_names_get(r, i, &s, &n, &e, &a);
    out[i].assign(s, n);
    if (errs) (*errs)[i] = e;
  }
  rc_names_free(r);
  return out;
}

static std::string rand_name(size_t maxlen, bool ascii) {
  static const char* uni[] = {"é", "ü", "日本", "😀", "ß", "Ω", "\xe2\x80\x8b"};
  std::string s;
  const size_t n = 1 + rnd() % maxlen;
  while (s.size() < n) {
    if (!ascii && rnd() % 5 == 0) s += uni[rnd() % 7];
    else s += (char)('!' + rnd() % 94);
  }
  for (auto& ch : s)
    if (ch == '/') ch = '_';
  return s;
}

static void test_names(rc_cipher* c) {
  // decoders on random bytes and random strings over each alphabet: no crash, no overrun
  const char* alpha[] = {"0123456789abcdefghijklmnopqrstuv=", "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_="};
  for (int k = 0; k < 3000; k++) {
    const int enc = k % 3;
    std::string s;
    const size_t n = rnd() % 90;
    for (size_t i = 0; i < n; i++) {
      if (enc < 2 && rnd() % 8) s += alpha[enc][rnd() % strlen(alpha[enc])];
      else s += (char)rnd();
    }
    uint8_t out[256];
    uint64_t ol = 0;
    int64_t arg = 0;
    const int32_t e = rc_name_decode(enc, s.data(), s.size(), out, sizeof out, &ol, &arg);
    CHECK(e == RC_NIL || e <= -130, "decode returned %d", e);
    CHECK(arg >= 0 && arg <= (int64_t)s.size() + 8, "decode err arg %ld of %zu", (long)arg, s.size());
  }
  for (int k = 0; k < 500; k++) {  // encode -> decode round trip
    const int enc = k % 3;
    std::vector<uint8_t> b = rbytes(rnd() % 200);
    char buf[1024];
    const int64_t n = rc_name_encode(enc, b.data(), b.size(), buf, sizeof buf);
    uint8_t out[256];
    uint64_t ol = 0;
    int64_t arg = 0;
    CHECK(n < (int64_t)sizeof buf && rc_name_decode(enc, buf, (uint64_t)n, out, sizeof out, &ol, &arg) == RC_NIL &&
              ol == b.size() && (ol == 0 || !memcmp(out, b.data(), ol)),
          "encoding %d round trip of %zu bytes", enc, b.size());
  }
  // every mode / encoding: garbage decrypts give an error or a string, valid names round trip
  for (int32_t mode : {RC_NAME_STANDARD, RC_NAME_OBFUSCATE, RC_NAME_OFF})
    for (int32_t enc : {RC_ENC_BASE32, RC_ENC_BASE64, RC_ENC_BASE32768})
      for (int32_t dir : {1, 0}) {
        rc_cipher_set_name_encryption(c, mode, dir, enc);
        std::vector<std::string> names;
        for (int k = 0; k < 300; k++) {
          std::string s = rand_name(k % 10 == 0 ? 200 : 40, k % 3 == 0);
          if (k % 7 == 0) s = "dir" + std::to_string(k) + "/" + s;
          if (k % 11 == 0) s += "-v2001-02-03-040506-123.txt";
          names.push_back(s);
        }
        std::vector<int32_t> errs;
        const std::vector<std::string> enc_names = run_names(c, RC_OP_ENCRYPT_FILE_NAME, names, &errs);
        for (size_t i = 0; i < names.size(); i++) CHECK(errs[i] == RC_NIL, "encrypt name err %d", errs[i]);
        const std::vector<std::string> back = run_names(c, RC_OP_DECRYPT_FILE_NAME, enc_names, &errs);
        for (size_t i = 0; i < names.size(); i++)
          CHECK(errs[i] == RC_NIL && back[i] == names[i], "mode %d enc %d dir %d: round trip of '%s' -> '%s' err %d",
                mode, enc, dir, names[i].c_str(), back[i].c_str(), errs[i]);
        std::vector<std::string> junk;
        for (size_t i = 0; i < enc_names.size(); i++) {
          std::string s = enc_names[i];
          switch (i % 6) {
            case 0: if (!s.empty()) s[rnd() % s.size()] ^= (char)(1 + rnd() % 255); break;
            case 1: s = s.substr(0, rnd() % (s.size() + 1)); break;
            case 2: s += (char)rnd(); break;
            case 3: s = rand_name(60, false); break;
            case 4: { std::vector<uint8_t> b = rbytes(rnd() % 100); s.assign(b.begin(), b.end()); } break;
            default: s = s + "/" + s.substr(0, s.size() / 2); break;
          }
          junk.push_back(s);
        }
        for (int32_t op : {RC_OP_DECRYPT_FILE_NAME, RC_OP_DECRYPT_DIR_NAME}) run_names(c, op, junk, &errs);
        run_names(c, RC_OP_DEOBFUSCATE_SEGMENT, junk, &errs);
        if (mode == RC_NAME_STANDARD) run_names(c, RC_OP_DECRYPT_SEGMENT, junk, &errs);
      }
  rc_cipher_set_name_encryption(c, RC_NAME_STANDARD, 1, RC_ENC_BASE32);
  // crafted standard-mode errors (cipher.go:293-312): lengths not a multiple of 16 after decode,
  // too long, and bad padding after decryption ("" decrypts to "" without error, :294)
  std::vector<std::string> crafted = {"a", "aaaaaaaa", std::string(3300, 'a'), "0123456789abcdefghijklmnopqrstuv"};
  std::vector<int32_t> errs;
  run_names(c, RC_OP_DECRYPT_SEGMENT, crafted, &errs);
  for (size_t i = 0; i < crafted.size(); i++) CHECK(errs[i] != RC_NIL, "crafted name %zu decrypted", i);
  const std::vector<std::string> empty = run_names(c, RC_OP_DECRYPT_SEGMENT, {""}, &errs);
  CHECK(errs[0] == RC_NIL && empty[0].empty(), "empty segment");
}


// ---------------------------------------------------------------- per-object hashes
// computeHashWithNonce (crypt.go:784-806): MD5 of the crypt file newEncrypter(src, &nonce) would
// produce, the source closed once, reader errors / close errors returned as io.Copy + CheckClose do
static void test_hash_with_nonce(rc_cipher* c, const uint8_t key[32]) {
  const size_t lens[] = {0, 1, 65535, 65536, 65537, 16 * 65536, 16 * 65536 + 1, 48 * 65536 + 3, 3000001};
  for (size_t L : lens)
    for (size_t ch : {(size_t)4096, (size_t)65537, (size_t)1 << 30}) {
      std::vector<uint8_t> plain = rbytes(L), nonce = rbytes(24);
      if (L == 3000001) memset(nonce.data(), 0xFF, 8);
      Src s;
      s.p = plain.data();
      s.n = L;
      s.chunk = ch;
      uint8_t got[16];
      const int32_t err = rc_compute_hash_with_nonce(c, mk(&s), nonce.data(), got);
      const std::vector<uint8_t> f = oracle_file(plain, nonce.data(), key);
      CHECK(err == RC_NIL && md5_of(f.data(), f.size()) == std::vector<uint8_t>(got, got + 16) && s.closes == 1,
            "hash L=%zu chunk=%zu err=%d closes=%d", L, ch, err, s.closes);
    }
  const std::vector<uint8_t> plain = rbytes(3 * 1048576 + 77), nonce = rbytes(24);
  for (int64_t q : {0L, 1L, 65536L, 65537L, 1048576L, 2500000L}) {  // reader error: returned, source closed
    Src s;
    s.p = plain.data();
    s.n = plain.size();
    s.fail_at = q;
    uint8_t got[16];
    const int32_t err = rc_compute_hash_with_nonce(c, mk(&s), nonce.data(), got);
    CHECK(err == s.fail_err && s.closes == 1, "hash reader error at %ld: err %d closes %d", (long)q, err, s.closes);
    Src t = s;  // read error and close error: the read error wins
    t.pos = 0;
    t.closes = 0;
    const int32_t err2 = rc_compute_hash_with_nonce(c, rc_reader{src_read, src_close_fail, nullptr, &t}, nonce.data(), got);
    CHECK(err2 == t.fail_err && t.closes == 1, "hash reader+close error at %ld: %d", (long)q, err2);
  }
  Src s;  // clean read, failing close: the close error, with the digest (hashStr, CheckClose's err)
  s.p = plain.data();
  s.n = plain.size();
  uint8_t got[16];
  const int32_t err = rc_compute_hash_with_nonce(c, rc_reader{src_read, src_close_fail, nullptr, &s}, nonce.data(), got);
  const std::vector<uint8_t> pf = oracle_file(plain, nonce.data(), key);
  CHECK(err == RC_USER_BASE + 9 && s.closes == 1 && std::vector<uint8_t>(got, got + 16) == md5_of(pf.data(), pf.size()),
        "hash close error: %d", err);
  Src n;  // no close function (io.NopCloser)
  n.p = plain.data();
  n.n = 100;
  CHECK(rc_compute_hash_with_nonce(c, rc_reader{src_read, nullptr, nullptr, &n}, nonce.data(), got) == RC_NIL,
        "hash without close");
  CHECK(rc_compute_hash_with_nonce(nullptr, mk(&n), nonce.data(), got) == RC_ERR_INVALID, "hash null cipher");
}

// crypt.put's tee hash taken by the encrypter: MD5 of exactly the bytes read so far
static void test_encrypter_md5(rc_cipher* c, const uint8_t key[32]) {
  for (size_t L : {(size_t)0, (size_t)1, (size_t)65536, (size_t)65537, (size_t)(5 * 1048576 + 3), (size_t)(9 * 1048576)}) {
    std::vector<uint8_t> plain = rbytes(L), nonce = rbytes(24);
    const std::vector<uint8_t> f = oracle_file(plain, nonce.data(), key);
    // stop points: nothing read, inside the header, header only, inside / at the end of a batch, all
    std::vector<size_t> stops = {0, 5, 32, 33, f.size() / 2, f.size()};
    for (size_t stop : stops) {
      if (stop > f.size()) continue;
      Src s;
      s.p = plain.data();
      s.n = L;
      s.chunk = 65537;
      int32_t err = 0;
      rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
      if (!e) {
        CHECK(false, "encrypt_data");
        continue;
      }
      uint8_t d[16];
      CHECK(rc_encrypter_md5(e, d) == RC_ERR_INVALID, "md5 while off");
      CHECK(rc_encrypter_set_md5(e, 1) == RC_NIL, "set_md5");
      std::vector<uint8_t> ct;
      while (ct.size() < stop) {
        uint8_t buf[70000];
        const int64_t want = (int64_t)std::min<size_t>(sizeof buf, stop - ct.size());
        const int64_t k = rc_encrypter_read(e, buf, want, &err);
        ct.insert(ct.end(), buf, buf + k);
        if (err != RC_NIL) break;
      }
      if (stop == f.size()) {  // the consumer also sees EOF (io.ReadAll)
        uint8_t one;
        CHECK(rc_encrypter_read(e, &one, 1, &err) == 0 && err == RC_EOF, "EOF after the stream");
      }
      CHECK(rc_encrypter_md5(e, d) == RC_NIL && ct.size() == stop &&
                std::vector<uint8_t>(d, d + 16) == md5_of(f.data(), stop),
            "encrypter md5 L=%zu stop=%zu got %zu", L, stop, ct.size());
      CHECK(rc_encrypter_set_md5(e, 1) == (stop ? RC_ERR_INVALID : RC_NIL), "set_md5 after a read");
      rc_encrypter_free(e);
    }
  }
}

// ---------------------------------------------------------------- node topology (xs_topo.cpp)
// A fake sysfs tree: the GPU's PCI function on node 1, node 1 = CPU 0 only.  Library threads
// pinned to node 1 may then run on CPU 0 only; the preferred-node memory policy is scoped.
static void put_file(const std::string& path, const char* text) {
  std::string dir;
  for (size_t i = 1; i < path.size(); i++)
    if (path[i] == '/') mkdir(path.substr(0, i).c_str(), 0755);
  FILE* f = fopen(path.c_str(), "w");
  if (f) {
    fputs(text, f);
    fclose(f);
  }
}
static void test_topology() {
  char tmpl[] = "/tmp/rc_sysfs_XXXXXX";
  const char* root = mkdtemp(tmpl);
  CHECK(root != nullptr, "mkdtemp");
  if (!root) return;
  const std::string r(root);
  put_file(r + "/bus/pci/devices/0000:c1:00.0/numa_node", "1\n");
  put_file(r + "/bus/pci/devices/0000:05:00.0/numa_node", "-1\n");
  put_file(r + "/devices/system/node/node1/cpulist", "0\n");
  put_file(r + "/devices/system/node/node2/cpulist", "4-7,12,14-15\n");
  setenv("RCLONE_AMD_SYSFS_ROOT", root, 1);
  CHECK(xs::pci_numa_node("0000:C1:00.0") == 1, "bus id -> node (upper-case id)");
  CHECK(xs::pci_numa_node("0000:05:00.0") == -1 && xs::pci_numa_node("0000:99:00.0") == -1, "unknown node");
  std::vector<int> cpus;
  CHECK(xs::node_cpus(2, &cpus) && cpus == std::vector<int>({4, 5, 6, 7, 12, 14, 15}), "cpulist ranges");
  CHECK(!xs::node_cpus(3, &cpus) && !xs::node_cpus(-1, &cpus), "missing node");
  CHECK(!xs::parse_cpulist("3-1", &cpus) && !xs::parse_cpulist("x", &cpus), "malformed cpulist");
  std::vector<int> devs;
  CHECK(xs::parse_device_list("0,1,1,2", &devs) == 4 && devs == std::vector<int>({0, 1, 1, 2}), "device list repeats");
  CHECK(xs::parse_device_list(" 3, 4", &devs) == 2 && devs == std::vector<int>({3, 4}), "device list spaces");
  CHECK(xs::parse_device_list("0,x", &devs) == 1 && xs::parse_device_list("", &devs) == 0, "device list garbage");
  int on_cpu0 = 0;
  std::thread t([&] {
    xs::pin_thread_to_node(1);
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) on_cpu0 = CPU_COUNT(&set) == 1 && CPU_ISSET(0, &set);
  });
  t.join();
  CHECK(on_cpu0, "thread pinned to the node's CPUs");
  // a process started under a narrowed mask (taskset / numactl --physcpubind): library threads
  // stay inside it -- the node's CPUs intersected with the mask, or left alone when disjoint
  cpu_set_t full;
  CPU_ZERO(&full);
  sched_getaffinity(0, sizeof full, &full);
  if (CPU_ISSET(0, &full) && CPU_ISSET(1, &full) && CPU_ISSET(2, &full)) {
    put_file(r + "/devices/system/node/node3/cpulist", "0-1\n");
    cpu_set_t narrow;
    CPU_ZERO(&narrow);
    CPU_SET(1, &narrow);
    CPU_SET(2, &narrow);
    sched_setaffinity(0, sizeof narrow, &narrow);
    xs::capture_process_affinity();
    int inter_ok = 0, disjoint_ok = 0;
    std::thread t2([&] {
      xs::pin_thread_to_node(3);  // node {0,1} & mask {1,2} = {1}
      cpu_set_t s;
      CPU_ZERO(&s);
      if (sched_getaffinity(0, sizeof s, &s) == 0) inter_ok = CPU_COUNT(&s) == 1 && CPU_ISSET(1, &s);
    });
    t2.join();
    std::thread t3([&] {
      xs::pin_thread_to_node(1);  // node {0} & mask {1,2} = {}: unchanged
      cpu_set_t s;
      CPU_ZERO(&s);
      if (sched_getaffinity(0, sizeof s, &s) == 0) disjoint_ok = CPU_EQUAL(&s, &narrow);
    });
    t3.join();
    const int counted = xs::effective_cpus();
    // the main thread's mask narrows after load, with no capture call (OMP_PROC_BIND binding the
    // host program's initial thread, or taskset -p on its pid): the load-time mask still counts,
    // so pool sizing does not drop to one CPU and pinning still finds the node's CPUs
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(2, &one);
    sched_setaffinity(0, sizeof one, &one);
    const int counted_one = xs::effective_cpus();
    int kept_ok = 0;
    std::thread t4([&] {
      xs::pin_thread_to_node(3);  // node {0,1} & (mask {2} | load {1,2}) = {1}
      cpu_set_t s;
      CPU_ZERO(&s);
      if (sched_getaffinity(0, sizeof s, &s) == 0) kept_ok = CPU_COUNT(&s) == 1 && CPU_ISSET(1, &s);
    });
    t4.join();
    // ... but a cgroup cpuset narrowed to {2} after load is the operator's: honoured
    put_file(r + "/fs/cgroup/cpuset.cpus.effective", "2\n");
    const int counted_cpuset = xs::effective_cpus();
    int moved_ok = 0;
    std::thread t5([&] {
      xs::pin_thread_to_node(3);  // node {0,1} & {2} = {}: left on the process mask
      cpu_set_t s;
      CPU_ZERO(&s);
      if (sched_getaffinity(0, sizeof s, &s) == 0) moved_ok = CPU_COUNT(&s) == 1 && CPU_ISSET(2, &s);
    });
    t5.join();
    remove((r + "/fs/cgroup/cpuset.cpus.effective").c_str());
    sched_setaffinity(0, sizeof full, &full);
    const int counted_full = xs::effective_cpus();
    xs::capture_process_affinity();
    CHECK(counted_one == 2 || getenv("RCLONE_AMD_CPUS"), "a main thread narrowed after load keeps the load mask (%d)",
          counted_one);
    CHECK(kept_ok, "pinning uses the load-time mask while only the main thread is narrowed");
    CHECK(counted_cpuset == 1 || getenv("RCLONE_AMD_CPUS"), "effective_cpus follows a cpuset narrowed after load (%d)",
          counted_cpuset);
    CHECK(counted_full >= counted || getenv("RCLONE_AMD_CPUS"), "effective_cpus follows a mask widened again (%d)", counted_full);
    CHECK(moved_ok, "library threads stay inside the cgroup cpuset as it is now");
    CHECK(inter_ok, "pinning intersects the node with the process mask");
    CHECK(disjoint_ok, "no pinning outside the process mask when the node is disjoint from it");
    CHECK(counted == 2 || getenv("RCLONE_AMD_CPUS"), "effective_cpus counts the process mask (%d)", counted);
  }
  int mode_before = -1, mode_in = -1, mode_after = -1;
  unsigned long mask[16] = {0};
  syscall(SYS_get_mempolicy, &mode_before, mask, 1024ul, nullptr, 0ul);
  {
    xs::ScopedMemPolicy pol(0);  // node 0 exists on any Linux machine
    memset(mask, 0, sizeof mask);
    syscall(SYS_get_mempolicy, &mode_in, mask, 1024ul, nullptr, 0ul);
    CHECK(mode_in == 1 && (mask[0] & 1ul), "preferred node 0 inside the scope (mode %d)", mode_in);
  }
  syscall(SYS_get_mempolicy, &mode_after, mask, 1024ul, nullptr, 0ul);
  CHECK(mode_after == mode_before, "policy restored (%d vs %d)", mode_after, mode_before);
  unsetenv("RCLONE_AMD_SYSFS_ROOT");
  (void)!system(("rm -rf " + r).c_str());
}

// ---------------------------------------------------------------- host MD5 tiers (md5_workers.h)
// Many streams through one worker, a CPU budget of 1 and the 16-lane engine: jobs of odd sizes
// (partial blocks on both ends), each stream's digest equal to the scalar MD5 of its bytes.
static void test_md5_tiers() {
  static xs::Md5Workers* w = new xs::Md5Workers(1, -1, 1, true, 2);  // never destroyed (parked threads)
  const uint64_t lanes0 = xs::md5_tier_stats().lanes.load();
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 24; t++)
    th.emplace_back([&, t] {
      uint64_t r = 0x9E37u * (t + 1);
      auto rnd32 = [&] {
        r = r * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(r >> 33);
      };
      std::vector<uint8_t> data(3 * 1048576 + 4096 * t + 7);
      for (auto& b : data) b = (uint8_t)rnd32();
      xs::HostMd5 got, want;
      xs::Md5Job job;
      job.st = &got;
      size_t pos = 0;
      while (pos < data.size()) {
        const size_t n = std::min<size_t>(data.size() - pos, 1 + rnd32() % 300000);
        md5_wait(&job);
        job.p = data.data() + pos;
        job.n = n;
        w->submit(&job, (rnd32() & 1) != 0);
        pos += n;
      }
      md5_wait(&job);
      want.update(data.data(), data.size());
      uint8_t a[16], b[16];
      got.final(a);
      want.final(b);
      if (memcmp(a, b, 16)) bad++;
    });
  for (auto& x : th) x.join();
  CHECK(bad == 0, "%d streams hashed wrongly through the tiers", bad.load());
  CHECK(!xs::md5_x16_supported() || xs::md5_tier_stats().lanes.load() > lanes0, "engine lanes used");
}

// ---------------------------------------------------------------- a failing GPU engine
// A GPU submission that fails (stub_engine_fail: XS_ERR_HIP, as a HIP error in xs_api.cpp would be)
// must surface as RC_ERR_GPU at the refill that made it, exactly as the reference surfaces any
// error there: no byte of the failed batch is served, the error is sticky through later Reads and
// RangeSeek (encrypter/decrypter finish, cipher.go:748-758, :1042-1052), Close still closes the
// source once and then reports ErrorFileClosed (:1069-1087), and other handles on the same cipher
// keep working.  Refills ramp 1, 2, 4, 8, 8, ... blocks (growth 2, batch 8), so failing refill k
// leaves exactly the first 2^k - 1 blocks served.
static void test_engine_failure(rc_cipher* c, const uint8_t key[32]) {
  const std::vector<uint8_t> plain = rbytes(40 * 65536 + 123);
  const std::vector<uint8_t> nonce = rbytes(24);
  const std::vector<uint8_t> want = oracle_file(plain, nonce.data(), key);
  rc_cipher_set_batch_blocks(c, 8);
  rc_cipher_set_readahead_growth(c, 2);
  const long failed0 = stub_engine_failed();
  for (int k = 0; k < 5; k++) {
    const size_t blocks_before = k < 4 ? (1u << k) - 1 : 15;  // refills 1, 2, 4, 8 then 8
    const size_t wire_before = 32 + blocks_before * 65552, plain_before = blocks_before * 65536;
    // encrypter
    Src s;
    s.p = plain.data();
    s.n = plain.size();
    int32_t err = 0;
    rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
    stub_engine_fail(stub_engine_submissions() + k, 1);
    std::vector<uint8_t> ct;
    err = drain_enc(e, ct);
    stub_engine_fail(-1, 0);
    CHECK(err == RC_ERR_GPU, "encrypter: refill %d failed with %d", k, err);
    CHECK(ct.size() == wire_before && std::equal(ct.begin(), ct.end(), want.begin()),
          "encrypter: refill %d failed after %zu bytes (want the %zu before it)", k, ct.size(), wire_before);
    uint8_t b[64];
    CHECK(rc_encrypter_read(e, b, 64, &err) == 0 && err == RC_ERR_GPU, "encrypter: sticky error %d", err);
    CHECK(rc_encrypter_read(e, b, 1, &err) == 0 && err == RC_ERR_GPU, "encrypter: sticky error again %d", err);
    // another handle on the same cipher while this one is failed: unaffected
    {
      Src s2;
      s2.p = plain.data();
      s2.n = 3 * 65536 + 5;
      rc_encrypter* e2 = rc_encrypt_data(c, mk(&s2), nonce.data(), &err);
      std::vector<uint8_t> ct2;
      std::vector<uint8_t> p2(plain.begin(), plain.begin() + (long)s2.n);
      CHECK(drain_enc(e2, ct2) == RC_EOF && ct2 == oracle_file(p2, nonce.data(), key), "other encrypter");
      rc_encrypter_free(e2);
    }
    rc_encrypter_free(e);
    // decrypter (DecryptData): the header read makes no submission
    Src d;
    d.p = want.data();
    d.n = want.size();
    rc_decrypter* h = rc_decrypt_data(c, mk(&d), &err);
    CHECK(h && err == RC_NIL, "decrypt_data %d", err);
    if (!h) continue;
    stub_engine_fail(stub_engine_submissions() + k, 1);
    std::vector<uint8_t> pt;
    err = drain_dec(h, pt);
    stub_engine_fail(-1, 0);
    CHECK(err == RC_ERR_GPU, "decrypter: refill %d failed with %d", k, err);
    CHECK(pt.size() == plain_before && std::equal(pt.begin(), pt.end(), plain.begin()),
          "decrypter: refill %d failed after %zu bytes (want the %zu before it)", k, pt.size(), plain_before);
    CHECK(rc_decrypter_read(h, b, 64, &err) == 0 && err == RC_ERR_GPU, "decrypter: sticky error %d", err);
    rc_decrypter_range_seek(h, 0, 0, -1, &err);  // not opened with a seek callback: finish() returns the set error
    CHECK(err == RC_ERR_GPU, "decrypter: RangeSeek after the failure returned %d", err);
    CHECK(rc_decrypter_close(h) == RC_NIL && d.closes == 1, "decrypter close after the failure");
    CHECK(rc_decrypter_read(h, b, 64, &err) == 0 && err == RC_ERR_FILE_CLOSED, "read after close %d", err);
    CHECK(rc_decrypter_close(h) == RC_ERR_FILE_CLOSED && d.closes == 1, "second close");
    rc_decrypter_free(h);
  }
  // DecryptDataSeek: its RangeSeek fills the first block itself (cipher.go:1027-1031), so a failure
  // there fails the open -- no handle, RC_ERR_GPU, every source it opened closed
  // (newDecrypterSeek, :826-832); a failure at the next refill serves the rest of the first block,
  // then RC_ERR_GPU, and a RangeSeek after it returns that sticky error (finished with an error
  // other than EOF, :976-980)
  for (int at = 0; at < 2; at++) {
    OpenCtx o{&want, {}, {}};
    int32_t err = 0;
    stub_engine_fail(stub_engine_submissions() + at, 1);
    rc_decrypter* h = rc_decrypt_data_seek(c, open_cb, &o, 70000, -1, &err);
    if (at == 0) {
      stub_engine_fail(-1, 0);
      CHECK(!h && err == RC_ERR_GPU, "seek open with a failed first fill: %d", err);
      bool closed = !o.srcs.empty();
      for (auto* x : o.srcs) closed = closed && x->closes == 1;
      CHECK(closed, "seek open: sources closed after the failure");
    } else {
      CHECK(h && err == RC_NIL, "decrypt_data_seek %d", err);
      if (h) {
        std::vector<uint8_t> pt;
        err = drain_dec(h, pt);
        stub_engine_fail(-1, 0);
        CHECK(err == RC_ERR_GPU && pt.size() == 131072 - 70000 &&
                  std::equal(pt.begin(), pt.end(), plain.begin() + 70000),
              "seek decrypter: %d after %zu bytes", err, pt.size());
        rc_decrypter_range_seek(h, 0, 0, -1, &err);
        CHECK(err == RC_ERR_GPU, "seek decrypter RangeSeek %d", err);
        CHECK(rc_decrypter_close(h) == RC_NIL, "seek decrypter close");
        rc_decrypter_free(h);
      }
    }
    stub_engine_fail(-1, 0);
    for (auto* x : o.srcs) delete x;
  }
  // computeHashWithNonce: the failed seal is the call's error, no digest; the next call succeeds
  {
    Src s;
    s.p = plain.data();
    s.n = plain.size();
    uint8_t md5[16] = {0}, zero[16] = {0};
    stub_engine_fail(stub_engine_submissions() + 2, 1);
    const int32_t e1 = rc_compute_hash_with_nonce(c, mk(&s), nonce.data(), md5);
    stub_engine_fail(-1, 0);
    CHECK(e1 == RC_ERR_GPU && !memcmp(md5, zero, 16) && s.closes == 1, "hash with a failed seal: %d", e1);
    Src s2;
    s2.p = plain.data();
    s2.n = plain.size();
    CHECK(rc_compute_hash_with_nonce(c, mk(&s2), nonce.data(), md5) == RC_NIL &&
              std::vector<uint8_t>(md5, md5 + 16) == md5_of(want.data(), want.size()),
          "hash after the failure");
  }
  // concurrent streams (TSan): 8 writers of 20 blocks, 5 refills each; three consecutive
  // submissions fail, so exactly three streams end with RC_ERR_GPU after a correct prefix and
  // the other five complete bit-exact
  {
    std::atomic<int> failed{0}, bad{0};
    std::vector<std::vector<uint8_t>> outs(8);
    const long base = stub_engine_submissions();
    stub_engine_fail(base + 10, 3);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; t++)
      th.emplace_back([&, t] {
        Src s;
        s.p = plain.data();
        s.n = 20 * 65536;
        int32_t err = 0;
        rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce.data(), &err);
        std::vector<uint8_t> ct;
        err = drain_enc(e, ct);
        const size_t full = 32 + 20 * 65552;
        if (err == RC_ERR_GPU) {
          failed++;
          if (ct.size() >= full || !std::equal(ct.begin(), ct.end(), want.begin())) bad++;
        } else if (err != RC_EOF || ct.size() != full || !std::equal(ct.begin(), ct.end(), want.begin())) {
          bad++;
        }
        rc_encrypter_free(e);
      });
    for (auto& x : th) x.join();
    stub_engine_fail(-1, 0);
    CHECK(failed == 3 && bad == 0, "concurrent: %d streams failed (want 3), %d bad", failed.load(), bad.load());
  }
  CHECK(stub_engine_failed() - failed0 == 5 * 2 + 2 + 1 + 3, "injected failures %ld", stub_engine_failed() - failed0);
  rc_cipher_set_batch_blocks(c, 64);
  rc_cipher_set_readahead_growth(c, 0);
}

// ---------------------------------------------------------------- concurrency (TSan)
static void test_concurrency(rc_cipher* c, const uint8_t key[32]) {
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++)
    th.emplace_back([&, t] {
      for (int k = 0; k < 6; k++) {
        std::vector<uint8_t> plain((size_t)(t * 37000 + k * 9000 + 1), (uint8_t)(t * 7 + k));
        uint8_t nonce[24];
        for (int i = 0; i < 24; i++) nonce[i] = (uint8_t)(t + 3 * k + i);
        Src s;
        s.p = plain.data();
        s.n = plain.size();
        s.chunk = 30000;
        int32_t err = 0;
        rc_encrypter* e = rc_encrypt_data(c, mk(&s), nonce, &err);
        if (!e) {
          bad++;
          continue;
        }
        std::vector<uint8_t> ct;
        if (drain_enc(e, ct) != RC_EOF || ct != oracle_file(plain, nonce, key)) bad++;
        rc_encrypter_free(e);
        Src d;
        d.p = ct.data();
        d.n = ct.size();
        rc_decrypter* h = rc_decrypt_data(c, mk(&d), &err);
        if (!h) {
          bad++;
          continue;
        }
        std::vector<uint8_t> pt;
        if (drain_dec(h, pt) != RC_EOF || pt != plain) bad++;
        rc_decrypter_free(h);
        // per-object hash (cryptcheck's checkers) and the encrypter's own tee hash (put's transfers),
        // objects large enough to go through the MD5 workers
        std::vector<uint8_t> big((size_t)(2 * 1048576 + t * 65536 + k * 1000 + 5), (uint8_t)(k + t));
        const std::vector<uint8_t> bf = oracle_file(big, nonce, key), want = md5_of(bf.data(), bf.size());
        Src b;
        b.p = big.data();
        b.n = big.size();
        uint8_t hd[16];
        if (rc_compute_hash_with_nonce(c, mk(&b), nonce, hd) != RC_NIL || std::vector<uint8_t>(hd, hd + 16) != want) bad++;
        Src b2;
        b2.p = big.data();
        b2.n = big.size();
        rc_encrypter* e2 = rc_encrypt_data(c, mk(&b2), nonce, &err);
        if (!e2 || rc_encrypter_set_md5(e2, 1) != RC_NIL) {
          bad++;
          if (e2) rc_encrypter_free(e2);
          continue;
        }
        std::vector<uint8_t> ct2;
        if (drain_enc(e2, ct2) != RC_EOF || ct2 != bf || rc_encrypter_md5(e2, hd) != RC_NIL ||
            std::vector<uint8_t>(hd, hd + 16) != want)
          bad++;
        rc_encrypter_free(e2);
      }
    });
  for (auto& t : th) t.join();
  CHECK(bad == 0, "%d concurrent stream failures", bad.load());
  // one batch large enough for 16 host threads (> 2 chunks of 8192 names), first decode of the
  // process: the base32/base64 tables are built concurrently
  for (int32_t enc : {RC_ENC_BASE64, RC_ENC_BASE32}) {
    rc_cipher_set_name_encryption(c, RC_NAME_STANDARD, 1, enc);
    std::vector<std::string> names;
    for (int k = 0; k < 20000; k++) names.push_back("file" + std::to_string(k) + ".txt");
    std::vector<int32_t> errs;
    const std::vector<std::string> e = run_names(c, RC_OP_ENCRYPT_FILE_NAME, names, &errs);
    const std::vector<std::string> d = run_names(c, RC_OP_DECRYPT_FILE_NAME, e, &errs);
    int nbad = 0;
    for (size_t i = 0; i < names.size(); i++) nbad += d[i] != names[i] || errs[i] != RC_NIL;
    CHECK(nbad == 0, "%d names failed the concurrent round trip (enc %d)", nbad, enc);
  }
  rc_cipher_set_name_encryption(c, RC_NAME_STANDARD, 1, RC_ENC_BASE32);
}

int main(int argc, char** argv) {
  const bool only_concurrency = argc > 1 && !strcmp(argv[1], "--concurrency");
  setenv("RCLONE_AMD_NAME_THREADS", "16", 1);
  int32_t err = 0;
  rc_cipher* c = rc_cipher_new("potato", "", &err);
  if (!c) {
    fprintf(stderr, "rc_cipher_new: %d\n", err);
    return 1;
  }
  uint8_t key[32];
  rc_cipher_keys(c, key, nullptr, nullptr);
  if (only_concurrency) {
    test_concurrency(c, key);
    test_engine_failure(c, key);
    test_md5_tiers();
  } else {
    test_md5_tiers();
    test_concurrency(c, key);  // first: the decode tables are still unbuilt
    test_readahead(c);
    test_round_trips(c, key);
    test_damaged(c, key);
    test_reader_errors(c, key);
    test_hash_with_nonce(c, key);
    test_topology();
    test_encrypter_md5(c, key);
    test_seek_grid(c, key);
    test_engine_failure(c, key);
    test_names(c);
  }
  rc_cipher_free(c);
  if (g_fail) {
    fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  printf("sanitize ok (%ld checks)\n", g_checks.load());
  return 0;
}
