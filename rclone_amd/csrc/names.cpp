// names.cpp -- host mirror of the file-name half of rclone's backend/crypt/cipher.go (v1.76.0)
// behind the rc_* C ABI, with the EME-AES-256 segment cipher on the GPU (xs_eme.hip).
//
//   NewNameEncryptionMode / String        cipher.go:92-118   rc_new_name_encryption_mode
//   caseInsensitiveBase32Encoding         cipher.go:127-152  enc_base32 / dec_base32
//   NewNameEncoding (base64, base32768)   cipher.go:155-169  rc_new_name_encoding
//   encryptSegment / decryptSegment       cipher.go:264-312  batched: host pkcs7 + encoding,
//                                                            one GPU EME launch per batch
//   obfuscateSegment / deobfuscateSegment cipher.go:315-479  obfuscate / deobfuscate
//   encryptFileName / EncryptFileName / EncryptDirName / decryptFileName / DecryptFileName /
//   DecryptDirName                        cipher.go:482-618  run_path
//   lib/version Match / Remove / Add      lib/version/version.go
//   pkcs7 Pad / Unpad                     backend/crypt/pkcs7/pkcs7.go:20-63
//
// Host code only: the GPU side (name engines, the EME launch, xs_eme_batch_dev) is in
// names_gpu.cpp, so this file also builds into the CPU sanitizer harness (tests/native/).
//
// The reference encrypts one path segment per call; here a batch of names (a directory
// listing, a sync's worth of object names) is split into segments on the host, every segment
// that needs the block cipher is packed into one pinned buffer and transformed by a single
// kernel launch, then the results are encoded and reassembled.  Outputs and errors (values
// and which segment's error wins) are the reference's.
#include <algorithm>
#include <condition_variable>
#include <functional>
#include <array>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rc_internal.h"

namespace {

constexpr int kNameBlock = 16;         // nameCipherBlockSize = aes.BlockSize (cipher.go:33)
constexpr size_t kMaxCipherName = 2048;  // decryptSegment's limit (cipher.go:303); EME's 128 blocks

// ------------------------------------------------------------------ UTF-8 (Go unicode/utf8)
constexpr int32_t kRuneError = 0xFFFD;

// utf8.DecodeRuneInString: (RuneError, 1) for an invalid or short sequence.
int32_t decode_rune(const uint8_t* s, size_t n, size_t* size) {
  uint8_t b0 = s[0];
  if (b0 < 0x80) {
    *size = 1;
    return b0;
  }
  *size = 1;
  int need;
  int32_t r;
  uint8_t lo = 0x80, hi = 0xBF;
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    need = 1;
    r = b0 & 0x1F;
  } else if (b0 >= 0xE0 && b0 <= 0xEF) {
    need = 2;
    r = b0 & 0x0F;
    if (b0 == 0xE0) lo = 0xA0;
    if (b0 == 0xED) hi = 0x9F;
  } else if (b0 >= 0xF0 && b0 <= 0xF4) {
    need = 3;
    r = b0 & 0x07;
    if (b0 == 0xF0) lo = 0x90;
    if (b0 == 0xF4) hi = 0x8F;
  } else {
    return kRuneError;
  }
  if (n < (size_t)need + 1) return kRuneError;
  for (int i = 1; i <= need; i++) {
    uint8_t b = s[i];
    if (i == 1 ? (b < lo || b > hi) : (b < 0x80 || b > 0xBF)) return kRuneError;
    r = (r << 6) | (b & 0x3F);
  }
  *size = need + 1;
  return r;
}

bool valid_utf8(const std::string& s) {
  const uint8_t* p = (const uint8_t*)s.data();
  size_t i = 0;
  while (i < s.size()) {
    size_t sz;
    int32_t r = decode_rune(p + i, s.size() - i, &sz);
    if (r == kRuneError && sz == 1) return false;
    i += sz;
  }
  return true;
}

bool valid_rune(int64_t r) { return (r >= 0 && r < 0xD800) || (r > 0xDFFF && r <= 0x10FFFF); }

// strings.Builder.WriteRune: invalid runes are written as U+FFFD.
void put_rune(std::string& o, int64_t r) {
  if (!valid_rune(r)) r = kRuneError;
  if (r < 0x80) {
    o += (char)r;
  } else if (r < 0x800) {
    o += (char)(0xC0 | (r >> 6));
    o += (char)(0x80 | (r & 0x3F));
  } else if (r < 0x10000) {
    o += (char)(0xE0 | (r >> 12));
    o += (char)(0x80 | ((r >> 6) & 0x3F));
    o += (char)(0x80 | (r & 0x3F));
  } else {
    o += (char)(0xF0 | (r >> 18));
    o += (char)(0x80 | ((r >> 12) & 0x3F));
    o += (char)(0x80 | ((r >> 6) & 0x3F));
    o += (char)(0x80 | (r & 0x3F));
  }
}

template <class F>
void for_runes(const std::string& s, F f) {
  const uint8_t* p = (const uint8_t*)s.data();
  size_t i = 0;
  while (i < s.size()) {
    size_t sz;
    int32_t r = decode_rune(p + i, s.size() - i, &sz);
    f(r);
    i += sz;
  }
}

// ------------------------------------------------------------------ encodings
struct Err {
  int32_t code = RC_NIL;
  int64_t arg = 0;
};

const char kB32Hex[] = "0123456789ABCDEFGHIJKLMNOPQRSTUV";
const char kB64Url[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

const char kB32HexLower[] = "0123456789abcdefghijklmnopqrstuv";

// base32.HexEncoding.EncodeToString, '=' trimmed, lower-cased (cipher.go:136-140): five bytes
// to eight characters per step, written in place.
void enc_base32(const uint8_t* p, size_t n, std::string& o) {
  const size_t at = o.size();
  o.resize(at + (n * 8 + 4) / 5);  // unpadded length: 2, 4, 5, 7 characters for a 1..4-byte tail
  char* d = &o[at];
  size_t i = 0;
  for (; i + 5 <= n; i += 5, d += 8) {
    const uint64_t v = (uint64_t)p[i] << 32 | (uint64_t)p[i + 1] << 24 | (uint64_t)p[i + 2] << 16 |
                       (uint64_t)p[i + 3] << 8 | p[i + 4];
    for (int k = 0; k < 8; k++) d[k] = kB32HexLower[(v >> (35 - 5 * k)) & 31];
  }
  uint64_t acc = 0;
  int bits = 0;
  for (; i < n; i++) {
    acc = (acc << 8) | p[i];
    bits += 8;
    while (bits >= 5) {
      bits -= 5;
      *d++ = kB32HexLower[(acc >> bits) & 31];
    }
  }
  if (bits) *d++ = kB32HexLower[(acc << (5 - bits)) & 31];
}

// Value of a base32hex character after strings.ToUpper (either case accepted), or -1.
const std::array<int8_t, 256>& b32_values() {
  static const std::array<int8_t, 256> m = [] {
    std::array<int8_t, 256> t;
    t.fill(-1);
    for (int i = 0; i < 32; i++) {
      t[(uint8_t)kB32Hex[i]] = (int8_t)i;
      t[(uint8_t)kB32HexLower[i]] = (int8_t)i;
    }
    return t;
  }();
  return m;
}

// dec_base32 for the inputs EncodeToString produces: every byte a base32hex character in
// either case and a length whose unpadded tail is 0, 2, 4, 5 or 7 characters.  Then padding,
// upper-casing and newline stripping change nothing and encoding/base32 decodes quantum by
// quantum, ignoring a tail's unused low bits (non-strict).  False: take the exact path.
bool dec_base32_fast(const char* s, size_t n, std::vector<uint8_t>& out) {
  const size_t r = n & 7;
  if (r == 1 || r == 3 || r == 6) return false;
  const auto& v = b32_values();
  const uint8_t* p = (const uint8_t*)s;
  out.resize(n / 8 * 5 + (r * 5) / 8);
  uint8_t* d = out.data();
  size_t i = 0;
  for (; i + 8 <= n; i += 8, d += 5) {
    uint64_t acc = 0;
    int bad = 0;
    for (int k = 0; k < 8; k++) {
      const int8_t x = v[p[i + k]];
      bad |= x;
      acc = acc << 5 | (uint8_t)x;
    }
    if (bad < 0) return false;
    for (int k = 0; k < 5; k++) d[k] = (uint8_t)(acc >> (32 - 8 * k));
  }
  if (r) {
    uint64_t acc = 0;
    for (size_t k = 0; k < r; k++) {
      const int8_t x = v[p[i + k]];
      if (x < 0) return false;
      acc = acc << 5 | (uint8_t)x;
    }
    acc <<= 5 * (8 - r);
    for (size_t k = 0; k < (r * 5) / 8; k++) d[k] = (uint8_t)(acc >> (32 - 8 * k));
  }
  return true;
}

// caseInsensitiveBase32Encoding.DecodeString (cipher.go:143-152) over encoding/base32's
// decoder: '=' suffix rejected, padding re-added, upper-cased, newlines stripped, then the
// quantum decoder with Go's CorruptInputError offsets.
Err dec_base32(const char* s0, size_t n0, std::vector<uint8_t>& out) {
  out.clear();
  if (n0 && s0[n0 - 1] == '=') return {RC_ERR_BAD_BASE32_ENCODING, 0};
  if (dec_base32_fast(s0, n0, out)) return {};
  out.clear();
  size_t equals = ((n0 + 7) & ~(size_t)7) - n0;  // from the length before ToUpper, as in Go
  thread_local std::string s;
  s.clear();
  s.reserve(n0 + equals);
  for (size_t q = 0; q < n0; q++) {
    char ch = s0[q];
    if (ch == '\r' || ch == '\n') continue;  // stripNewlines
    // strings.ToUpper maps two non-ASCII runes onto the alphabet: U+0131 'ı' -> 'I' and U+017F
    // 'ſ' -> 'S' (two bytes become one, so the padding computed above no longer fits).  Every
    // other non-ASCII rune stays outside the alphabet and fails at the same offset.
    if (q + 1 < n0 && (uint8_t)ch == 0xC4 && (uint8_t)s0[q + 1] == 0xB1) {
      s += 'I';
      q++;
      continue;
    }
    if (q + 1 < n0 && (uint8_t)ch == 0xC5 && (uint8_t)s0[q + 1] == 0xBF) {
      s += 'S';
      q++;
      continue;
    }
    s += (ch >= 'a' && ch <= 'z') ? (char)(ch - 32) : ch;
  }
  s.append(equals, '=');
  // built once, thread-safely (C++11 magic static): rc_names_run decodes from many threads
  static const std::array<int8_t, 256> map = [] {
    std::array<int8_t, 256> m;
    m.fill(-1);
    for (int i = 0; i < 32; i++) m[(uint8_t)kB32Hex[i]] = (int8_t)i;
    return m;
  }();
  const int64_t olen = (int64_t)s.size();
  size_t pos = 0;
  bool end = false;
  while (pos < s.size() && !end) {
    uint8_t d[8] = {0};
    int dlen = 8;
    int j = 0;
    while (j < 8) {
      int64_t rem = (int64_t)s.size() - (int64_t)pos;
      if (rem == 0) return {RC_ERR_BASE32_CORRUPT, olen - rem - j};
      uint8_t in = (uint8_t)s[pos++];
      rem--;
      if (in == '=' && j >= 2 && rem < 8) {
        if (rem + j < 8 - 1) return {RC_ERR_BASE32_CORRUPT, olen};
        for (int k = 0; k < 8 - 1 - j; k++)
          if (rem > k && s[pos + k] != '=') return {RC_ERR_BASE32_CORRUPT, olen - rem + k - 1};
        dlen = j;
        end = true;
        if (dlen == 1 || dlen == 3 || dlen == 6) return {RC_ERR_BASE32_CORRUPT, olen - rem - 1};
        break;
      }
      int8_t v = map[in];
      if (v < 0) return {RC_ERR_BASE32_CORRUPT, olen - rem - 1};
      d[j++] = (uint8_t)v;
    }
    uint8_t b[5] = {(uint8_t)(d[0] << 3 | d[1] >> 2), (uint8_t)(d[1] << 6 | d[2] << 1 | d[3] >> 4),
                    (uint8_t)(d[3] << 4 | d[4] >> 1), (uint8_t)(d[4] << 7 | d[5] << 2 | d[6] >> 3),
                    (uint8_t)(d[6] << 5 | d[7])};
    int nb = dlen == 8 ? 5 : dlen == 7 ? 4 : dlen == 5 ? 3 : dlen == 4 ? 2 : dlen == 2 ? 1 : 0;
    out.insert(out.end(), b, b + nb);
  }
  return {};
}

// base64.RawURLEncoding.EncodeToString
void enc_base64(const uint8_t* p, size_t n, std::string& o) {
  const size_t at = o.size();
  o.resize(at + n / 3 * 4);
  char* d = &o[at];
  size_t i = 0;
  for (; i + 3 <= n; i += 3, d += 4) {  // three bytes to four characters per step
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    d[0] = kB64Url[v >> 18];
    d[1] = kB64Url[(v >> 12) & 63];
    d[2] = kB64Url[(v >> 6) & 63];
    d[3] = kB64Url[v & 63];
  }
  uint32_t acc = 0;
  int bits = 0;
  for (; i < n; i++) {
    acc = (acc << 8) | p[i];
    bits += 8;
    while (bits >= 6) {
      bits -= 6;
      o += kB64Url[(acc >> bits) & 63];
    }
  }
  if (bits) o += kB64Url[(acc << (6 - bits)) & 63];
}

// base64.RawURLEncoding.DecodeString: encoding/base64 decodeQuantum semantics (newlines skipped,
// no padding, non-strict), CorruptInputError at the offending input byte.
Err dec_base64(const char* s, size_t sn, std::vector<uint8_t>& out) {
  out.clear();
  static const std::array<int8_t, 256> map = [] {
    std::array<int8_t, 256> m;
    m.fill(-1);
    for (int i = 0; i < 64; i++) m[(uint8_t)kB64Url[i]] = (int8_t)i;
    return m;
  }();
  // Inputs EncodeToString produces (every byte in the alphabet, no 1-character tail) decode
  // four characters to three bytes per step; anything else takes the exact quantum decoder.
  if (sn % 4 != 1) {
    const uint8_t* p = (const uint8_t*)s;
    const size_t r = sn % 4;
    out.resize(sn / 4 * 3 + (r ? r - 1 : 0));
    uint8_t* d = out.data();
    size_t i = 0;
    int bad = 0;
    for (; i + 4 <= sn; i += 4, d += 3) {
      const int8_t a = map[p[i]], b = map[p[i + 1]], c = map[p[i + 2]], e = map[p[i + 3]];
      bad |= a | b | c | e;
      const uint32_t v = (uint32_t)(uint8_t)a << 18 | (uint32_t)(uint8_t)b << 12 | (uint32_t)(uint8_t)c << 6 | (uint8_t)e;
      d[0] = (uint8_t)(v >> 16);
      d[1] = (uint8_t)(v >> 8);
      d[2] = (uint8_t)v;
    }
    uint32_t v = 0;
    for (size_t k = 0; k < r; k++) {
      const int8_t a = map[p[i + k]];
      bad |= a;
      v |= (uint32_t)(uint8_t)a << (18 - 6 * k);
    }
    for (size_t k = 0; k + 1 < r; k++) d[k] = (uint8_t)(v >> (16 - 8 * k));
    if (bad >= 0) return {};
    out.clear();
  }
  size_t si = 0;
  while (si < sn) {
    uint8_t d[4] = {0};
    int dlen = 4;
    for (int j = 0; j < 4; j++) {
      if (si == sn) {
        if (j == 0) return {};
        if (j == 1) return {RC_ERR_BASE64_CORRUPT, (int64_t)si - j};
        dlen = j;
        break;
      }
      uint8_t in = (uint8_t)s[si++];
      int8_t v = map[in];
      if (v >= 0) {
        d[j] = (uint8_t)v;
        continue;
      }
      if (in == '\n' || in == '\r') {
        j--;
        continue;
      }
      return {RC_ERR_BASE64_CORRUPT, (int64_t)si - 1};
    }
    uint32_t val = (uint32_t)d[0] << 18 | (uint32_t)d[1] << 12 | (uint32_t)d[2] << 6 | d[3];
    uint8_t b[3] = {(uint8_t)(val >> 16), (uint8_t)(val >> 8), (uint8_t)val};
    out.insert(out.end(), b, b + (dlen - 1));
  }
  return {};
}

// base32768.SafeEncoding (github.com/Max-Sum/base32768, qntm's base32768): 15 bits per
// character from a 32768-character repertoire, a final group of <= 7 bits from a
// 128-character one; bits big-endian, the last group padded with 1s.  The repertoires are
// ranges of 32 code points given as (first, last) pairs.
const char32_t kB32768Pairs15[] =
    U"ҠҿԀԟڀڿݠޟ߀ߟကဟႠႿᄀᅟᆀᆟᇠሿበቿዠዿጠጿᎠᏟᐠᙟᚠᛟកសᠠᡟᣀᣟᦀᦟ᧠᧿ᨠᨿᯀᯟᰀᰟᴀᴟ⇠⇿⋀⋟⍀⏟␀␟─❟➀➿⠀⥿⦠⦿⨠⩟⪀⪿⫠⭟ⰀⰟⲀⳟⴀⴟⵀⵟ⺠⻟㇀㇟㐀䶟䷀龿ꀀꑿ꒠꒿ꔀꗿꙀꙟꚠꛟ꜀ꝟꞀꞟꡀꡟ";
const char32_t kB32768Pairs7[] = U"ƀƟɀʟ";

struct B32768 {
  std::vector<char32_t> enc15, enc7;
  std::vector<int32_t> dec;  // code point (< 0x10000) -> value | (15 or 7) << 16, or -1
  B32768() {
    for (size_t i = 0; kB32768Pairs15[i]; i += 2)
      for (char32_t c = kB32768Pairs15[i]; c <= kB32768Pairs15[i + 1]; c++) enc15.push_back(c);
    for (size_t i = 0; kB32768Pairs7[i]; i += 2)
      for (char32_t c = kB32768Pairs7[i]; c <= kB32768Pairs7[i + 1]; c++) enc7.push_back(c);
    dec.assign(0x10000, -1);
    for (size_t v = 0; v < enc15.size(); v++) dec[enc15[v]] = (int32_t)v | 15 << 16;
    for (size_t v = 0; v < enc7.size(); v++) dec[enc7[v]] = (int32_t)v | 7 << 16;
  }
};
const B32768& b32768() {
  static B32768 t;
  return t;
}

void enc_base32768(const uint8_t* p, size_t n, std::string& o) {
  const B32768& t = b32768();
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; i++) {
    acc = (acc << 8) | p[i];
    bits += 8;
    if (bits >= 15) {
      bits -= 15;
      put_rune(o, t.enc15[(acc >> bits) & 0x7FFF]);
    }
  }
  if (bits > 7) {
    put_rune(o, t.enc15[((acc << (15 - bits)) | ((1u << (15 - bits)) - 1)) & 0x7FFF]);
  } else if (bits > 0) {
    put_rune(o, t.enc7[((acc << (7 - bits)) | ((1u << (7 - bits)) - 1)) & 0x7F]);
  }
}

// Decoder: a character outside the repertoire, or a 7-bit character before the end, is a
// CorruptInputError at its character index (cipher_test.go:172-186 pins the index for
// "㼿c", "!", "㻙ⲿ=㻙ⲿ"); trailing pad bits are dropped.
Err dec_base32768(const char* s, size_t sn, std::vector<uint8_t>& out) {
  out.clear();
  const B32768& t = b32768();
  const uint8_t* p = (const uint8_t*)s;
  size_t i = 0;
  int64_t idx = 0;
  uint32_t acc = 0;
  int bits = 0;
  bool ended = false;
  while (i < sn) {
    size_t sz;
    int32_t r = decode_rune(p + i, sn - i, &sz);
    i += sz;
    int32_t v = (r >= 0 && r < 0x10000 && !(r == kRuneError && sz == 1)) ? t.dec[r] : -1;
    if (v < 0 || ended) return {RC_ERR_BASE32768_CORRUPT, idx};
    int nb = v >> 16;
    if (nb == 7) ended = true;
    acc = (acc << nb) | (uint32_t)(v & 0x7FFF);
    bits += nb;
    while (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
    }
    acc &= (1u << bits) - 1;
    idx++;
  }
  return {};
}

void encode_append(int32_t enc, const uint8_t* p, size_t n, std::string& o) {
  switch (enc) {
    case RC_ENC_BASE64: return enc_base64(p, n, o);
    case RC_ENC_BASE32768: return enc_base32768(p, n, o);
    default: return enc_base32(p, n, o);
  }
}

std::string encode(int32_t enc, const uint8_t* p, size_t n) {
  std::string o;
  encode_append(enc, p, n, o);
  return o;
}

Err decode(int32_t enc, const char* p, size_t n, std::vector<uint8_t>& out) {
  switch (enc) {
    case RC_ENC_BASE64: return dec_base64(p, n, out);
    case RC_ENC_BASE32768: return dec_base32768(p, n, out);
    default: return dec_base32(p, n, out);
  }
}

// ------------------------------------------------------------------ lib/version
const size_t kVersionLen = 23;  // len("-v2006-01-02-150405.000")

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// version.Match: regexp `-v\d{4}-\d{2}-\d{2}-\d{6}-\d{3}` anywhere in the name.
const char kVersionPat[] = "-vdddd-dd-dd-dddddd-ddd";

bool version_at(const char* p) {
  for (size_t k = 0; k < kVersionLen; k++)
    if (kVersionPat[k] == 'd' ? !is_digit(p[k]) : p[k] != kVersionPat[k]) return false;
  return true;
}

bool version_match(const char* p, size_t n) {
  if (n < kVersionLen) return false;
  const char* const last = p + (n - kVersionLen);  // the latest start a version fits at
  for (const char* q = p; q <= last; q++) {
    q = (const char*)memchr(q, '-', (size_t)(last - q) + 1);
    if (!q) return false;
    if (version_at(q)) return true;
  }
  return false;
}

// path.Ext with splitExt's ".file" rule (version.go:15-25): the base length of name.
size_t base_len(const char* p, size_t n) {
  for (size_t i = n; i-- > 0 && p[i] != '/';)
    if (p[i] == '.') return i == 0 ? n : i;  // ".file": base = ".file", ext = ""
  return n;
}

int days_in(int month, int year) {
  static const int d[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (month == 2 && (year % 4 == 0 && (year % 100 != 0 || year % 400 == 0))) return 29;
  return d[month - 1];
}

int num(const char* s, size_t n) {
  int v = 0;
  for (size_t i = 0; i < n; i++) v = v * 10 + (s[i] - '0');
  return v;
}

// version.Remove (version.go:38-56): if name's base ends in a version time.Parse accepts,
// returns its position; the stripped name is name[:at] + name[at+23:].  The version string is
// then kept verbatim (time.Format of the parsed time reproduces it), so version.Add(name, t)
// == insert it before name's extension.
bool version_remove(const char* p, size_t n, size_t* at) {
  size_t bl = base_len(p, n);
  if (bl < kVersionLen) return false;
  size_t st = bl - kVersionLen;
  if (p[bl - 4] != '-') return false;
  const char* v = p + st;  // time.Parse("-v2006-01-02-150405.000", ...)
  if (!version_at(v)) return false;
  int year = num(v + 2, 4), month = num(v + 7, 2), day = num(v + 10, 2);
  int hh = num(v + 13, 2), mm = num(v + 15, 2), ss = num(v + 17, 2);
  if (month < 1 || month > 12 || day < 1 || day > days_in(month, year) || hh > 23 || mm > 59 || ss > 59) return false;
  *at = st;
  return true;
}

// version.Add for the piece of `o` starting at `from`: insert ver before the piece's extension.
void version_add_at(std::string& o, size_t from, const char* ver) {
  size_t bl = base_len(o.data() + from, o.size() - from);
  o.insert(from + bl, ver, kVersionLen);
}

// ------------------------------------------------------------------ obfuscation
std::string obfuscate(const rc_cipher* c, const std::string& pt) {
  if (pt.empty()) return "";
  if (!valid_utf8(pt)) return "!." + pt;
  int64_t dir = 0;
  for_runes(pt, [&](int32_t r) { dir += r; });
  dir %= 256;
  std::string o = std::to_string(dir) + ".";
  for (int i = 0; i < 32; i++) dir += c->name_key[i];
  for_runes(pt, [&](int32_t r) {
    if (r == '!') {
      o += "!!";
    } else if (r >= '0' && r <= '9') {
      int64_t thisdir = (dir % 9) + 1;
      put_rune(o, '0' + (r - '0' + thisdir) % 10);
    } else if ((r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z')) {
      int64_t thisdir = dir % 25 + 1;
      int64_t pos = r - 'A';
      if (pos >= 26) pos -= 6;
      pos = (pos + thisdir) % 52;
      if (pos >= 26) pos += 6;
      put_rune(o, 'A' + pos);
    } else if (r >= 0xA0 && r <= 0xFF) {
      int64_t thisdir = (dir % 95) + 1;
      put_rune(o, 0xA0 + (r - 0xA0 + thisdir) % 96);
    } else if (r >= 0x100) {
      int64_t thisdir = (dir % 127) + 1;
      int64_t base = r - r % 256;
      int64_t nr = base + (r - base + thisdir) % 256;
      if (!valid_rune(nr)) {
        o += '!';
        put_rune(o, r);
      } else {
        put_rune(o, nr);
      }
    } else {
      put_rune(o, r);
    }
  });
  return o;
}

// strconv.Atoi (64-bit int)
bool atoi64(const std::string& s, int64_t* v) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i == s.size()) return false;
  uint64_t x = 0;
  for (; i < s.size(); i++) {
    if (!is_digit(s[i])) return false;
    uint64_t d = (uint64_t)(s[i] - '0');
    if (x > (UINT64_MAX - d) / 10) return false;
    x = x * 10 + d;
    if (x > (uint64_t)INT64_MAX + (neg ? 1 : 0)) return false;
  }
  *v = neg ? (int64_t)(0 - x) : (int64_t)x;
  return true;
}

Err deobfuscate(const rc_cipher* c, const std::string& ct, std::string* out) {
  out->clear();
  if (ct.empty()) return {};
  size_t dot = ct.find('.');
  if (dot == std::string::npos) return {RC_ERR_NOT_AN_ENCRYPTED_FILE, 0};
  std::string numstr = ct.substr(0, dot), after = ct.substr(dot + 1);
  if (numstr == "!") {
    *out = after;
    return {};
  }
  int64_t dir;
  if (!atoi64(numstr, &dir)) return {RC_ERR_NOT_AN_ENCRYPTED_FILE, 0};
  uint64_t udir = (uint64_t)dir;  // Go int arithmetic wraps
  for (int i = 0; i < 32; i++) udir += c->name_key[i];
  dir = (int64_t)udir;
  std::string& o = *out;
  bool in_quote = false;
  for_runes(after, [&](int32_t r) {
    if (in_quote) {
      put_rune(o, r);
      in_quote = false;
    } else if (r == '!') {
      in_quote = true;
    } else if (r >= '0' && r <= '9') {
      int64_t thisdir = (dir % 9) + 1;
      int64_t nr = '0' + (int64_t)r - '0' - thisdir;
      if (nr < '0') nr += 10;
      put_rune(o, nr);
    } else if ((r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z')) {
      int64_t thisdir = dir % 25 + 1;
      int64_t pos = r - 'A';
      if (pos >= 26) pos -= 6;
      pos -= thisdir;
      if (pos < 0) pos += 52;
      if (pos >= 26) pos += 6;
      put_rune(o, 'A' + pos);
    } else if (r >= 0xA0 && r <= 0xFF) {
      int64_t thisdir = (dir % 95) + 1;
      int64_t nr = 0xA0 + (int64_t)r - 0xA0 - thisdir;
      if (nr < 0xA0) nr += 96;
      put_rune(o, nr);
    } else if (r >= 0x100) {
      int64_t thisdir = (dir % 127) + 1;
      int64_t base = r - r % 256;
      int64_t nr = (int32_t)(base + ((int64_t)r - base - thisdir));
      if (nr < base) nr += 256;
      put_rune(o, nr);
    } else {
      put_rune(o, r);
    }
  });
  return {};
}

// A batch of segments for the block cipher: padded/decoded bytes packed at 16-aligned
// offsets, then one H2D, one EME launch (in place), one D2H.
struct SegBatch {
  std::vector<uint8_t> data;
  std::vector<xs_name_desc> desc;
  uint64_t add(const uint8_t* p, size_t n) {  // n multiple of 16, 16..2048
    xs_name_desc d{data.size(), (uint32_t)(n / kNameBlock), 0};
    data.insert(data.end(), p, p + n);
    desc.push_back(d);
    return desc.size() - 1;
  }
  const uint8_t* get(uint64_t i) const { return data.data() + desc[i].off; }
};

// Host stages of a large batch run on up to kHostThreads threads, one chunk of names each.
constexpr size_t kChunkNames = 8192;
constexpr unsigned kHostThreads = 16;

// A batch's host stages call parallel_for three or four times; spawning 16 threads each time
// costs milliseconds per call.  One process-wide set of helpers stays parked between calls (never
// destroyed) and serves one parallel_for at a time, whichever batch or stage it belongs to; a
// parallel_for that finds it busy (another batch's stage in flight) spawns its own threads.
class NamePool {
 public:
  explicit NamePool(unsigned helpers) {
    for (unsigned t = 0; t < helpers; t++) th_.emplace_back([this] { run(); });
  }
  bool try_run(size_t n, const std::function<void(size_t)>& f) {
    std::unique_lock<std::mutex> busy(use_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(mu_);
      f_ = &f;
      n_ = n;
      next_.store(0);
      active_ = (unsigned)th_.size();
      gen_++;
    }
    cv_.notify_all();
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);  // the caller works too
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return active_ == 0; });
    f_ = nullptr;
    return true;
  }
  unsigned helpers() const { return (unsigned)th_.size(); }

 private:
  void run() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return gen_ != seen; });
      seen = gen_;
      const std::function<void(size_t)>* f = f_;
      const size_t n = n_;
      g.unlock();
      for (size_t i; (i = next_.fetch_add(1)) < n;) (*f)(i);
      g.lock();
      if (--active_ == 0) done_.notify_one();
    }
  }
  std::mutex use_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(size_t)>* f_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  unsigned active_ = 0;
  uint64_t gen_ = 0;
};

unsigned name_threads() {
  static const unsigned nt = [] {
    unsigned v = (unsigned)xs::effective_cpus();
    if (const char* e = getenv("RCLONE_AMD_NAME_THREADS")) v = (unsigned)atoi(e);
    return std::max(1u, std::min(v, kHostThreads));
  }();
  return nt;
}

// the one helper pool of the process (a template-local static would give every call site's
// lambda type a pool of its own)
NamePool& name_pool() {
  static NamePool* pool = new NamePool(name_threads() - 1);
  return *pool;
}

void parallel_for_fn(size_t n, const std::function<void(size_t)>& f) {
  const unsigned nt = std::max(1u, std::min(name_threads(), (unsigned)n));
  if (nt <= 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  NamePool& pool = name_pool();
  if (pool.helpers() + 1 >= nt && pool.try_run(n, f)) return;
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++)
    th.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : th) t.join();
}

template <class F>
void parallel_for(size_t n, F f) {
  parallel_for_fn(n, std::function<void(size_t)>(f));
}

// All parts' segments in one pinned buffer -> one H2D, one EME launch (in place), one D2H
// (names_gpu.cpp).
int32_t run_eme(const rc_cipher* c, bool encrypt, std::vector<SegBatch*>& parts, double* ms) {
  *ms = 0;
  size_t nparts = parts.size();
  std::vector<size_t> base(nparts + 1, 0), dbase(nparts + 1, 0);
  for (size_t i = 0; i < nparts; i++) {
    base[i + 1] = base[i] + parts[i]->data.size();
    dbase[i + 1] = dbase[i] + parts[i]->desc.size();
  }
  const size_t data_bytes = base[nparts], ndesc = dbase[nparts];
  if (ndesc == 0) return RC_NIL;
  size_t desc_off = (data_bytes + 255) & ~(size_t)255;
  size_t total = desc_off + ndesc * sizeof(xs_name_desc);
  uint8_t* h = nullptr;
  rcn::EmeDev* dev = rcn::eme_acquire(total, &h);
  if (!dev) return RC_ERR_GPU;
  xs_name_desc* hd = (xs_name_desc*)(h + desc_off);
  parallel_for(nparts, [&](size_t i) {
    const SegBatch& b = *parts[i];
    memcpy(h + base[i], b.data.data(), b.data.size());
    for (size_t k = 0; k < b.desc.size(); k++) {
      hd[dbase[i] + k] = b.desc[k];
      hd[dbase[i] + k].off += base[i];
    }
  });
  int32_t rc = rcn::eme_run(dev, encrypt, c, desc_off, ndesc, data_bytes, total, ms);
  if (rc == RC_NIL)
    parallel_for(nparts, [&](size_t i) { memcpy(parts[i]->data.data(), h + base[i], parts[i]->data.size()); });
  rcn::eme_release(dev);
  return rc;
}

// ------------------------------------------------------------------ paths (flat, per chunk)
// A chunk holds up to kChunkNames consecutive inputs of one rc_names_run call: their segments
// in one vector, owned texts / host-mode outputs / results in a few strings, so a name costs
// no heap allocations of its own.
struct Seg {
  uint32_t off = 0, len = 0;          // text: [off, off+len) of the input, or of Chunk::own if owned
  uint32_t ver = 0;                   // version string (23 bytes) at input offset ver when has_ver
  uint32_t slot = 0;                  // descriptor index in the chunk's SegBatch when gpu
  uint32_t out_off = 0, out_len = 0;  // obfuscate / deobfuscate output in Chunk::segout
  bool owned = false, process = false, gpu = false, has_ver = false;
  Err err;
};

struct Chunk {
  std::vector<Seg> segs;
  std::vector<uint32_t> seg0;  // input k owns segs[seg0[k] .. seg0[k+1])
  std::vector<uint8_t> direct; // input k was resolved without segments (result already in res)
  std::string own, segout;
  SegBatch batch;
  std::string res;             // every result of the chunk, back to back
  std::vector<uint64_t> roff;
  std::vector<uint32_t> rlen;
  std::vector<Err> err;
};

struct Ctx {
  const rc_cipher* c;
  int32_t op;
  bool enc_dir, standard;
};

// pkcs7.Pad(16) straight into the batch (encryptSegment's host half before the kernel).
void seg_encrypt_prepare(Seg& g, const char* text, SegBatch& b) {
  size_t n = g.len;
  size_t padded = n + (kNameBlock - n % kNameBlock);
  if (padded > kMaxCipherName) {  // eme.Transform panics on > 128 blocks
    g.err = {RC_ERR_NAME_TOO_LONG, 0};
    return;
  }
  size_t off = b.data.size();
  b.data.resize(off + padded);
  memcpy(b.data.data() + off, text, n);
  memset(b.data.data() + off + n, (int)(padded - n), padded - n);
  b.desc.push_back(xs_name_desc{off, (uint32_t)(padded / kNameBlock), 0});
  g.slot = (uint32_t)(b.desc.size() - 1);
  g.gpu = true;
}

// decryptSegment's host half before the kernel (cipher.go:293-307): decode, length checks.
void seg_decrypt_prepare(const rc_cipher* c, Seg& g, const char* text, SegBatch& b) {
  thread_local std::vector<uint8_t> raw;
  g.err = decode(c->name_enc, text, g.len, raw);
  if (g.err.code != RC_NIL) return;
  if (raw.size() % kNameBlock) {
    g.err = {RC_ERR_NOT_A_MULTIPLE_OF_BLOCKSIZE, 0};
    return;
  }
  if (raw.empty()) {
    g.err = {RC_ERR_TOO_SHORT_AFTER_DECODE, 0};
    return;
  }
  if (raw.size() > kMaxCipherName) {
    g.err = {RC_ERR_TOO_LONG_AFTER_DECODE, 0};
    return;
  }
  g.slot = (uint32_t)b.add(raw.data(), raw.size());
  g.gpu = true;
}

// Phase A for input k of the chunk: resolve directly (mode "off", directory names left alone)
// or split into segments, strip the last segment's version, and prepare every segment.
void prepare_input(const Ctx& x, Chunk& ch, const char* s, size_t n) {
  const rc_cipher* c = x.c;
  ch.seg0.push_back((uint32_t)ch.segs.size());
  uint8_t direct = 0;
  Err derr;
  size_t res_at = ch.res.size();
  switch (x.op) {
    case RC_OP_ENCRYPT_FILE_NAME:
      if (c->mode == RC_NAME_OFF) {  // EncryptFileName :542-547
        direct = 1;
        ch.res.append(s, n);
        ch.res += c->encrypted_suffix;
      }
      break;
    case RC_OP_ENCRYPT_DIR_NAME:
    case RC_OP_DECRYPT_DIR_NAME:
      if (c->mode == RC_NAME_OFF || !c->dir_name_encrypt) {  // :550-555, :613-618
        direct = 1;
        ch.res.append(s, n);
      }
      break;
    case RC_OP_DECRYPT_FILE_NAME:
      if (c->mode == RC_NAME_OFF) {  // DecryptFileName :600-611
        direct = 1;
        const std::string& suf = c->encrypted_suffix;
        size_t sl = suf.size();
        bool has = n >= sl && memcmp(s + n - sl, suf.data(), sl) == 0;
        if (n == sl || !has) {
          derr = {RC_ERR_NOT_AN_ENCRYPTED_FILE, 0};
        } else {
          size_t dn = n - sl, at;
          if (version_match(s, dn) && version_remove(s, dn, &at) && dn - kVersionLen == 0)
            derr = {RC_ERR_NOT_AN_ENCRYPTED_FILE, 0};  // only a version left
          else
            ch.res.append(s, dn);
        }
      }
      break;
    default:
      break;
  }
  if (direct) {
    ch.direct.push_back(1);
    ch.roff.push_back(res_at);
    ch.rlen.push_back((uint32_t)(ch.res.size() - res_at));
    ch.err.push_back(derr);
    return;
  }
  ch.direct.push_back(0);
  ch.roff.push_back(0);
  ch.rlen.push_back(0);
  ch.err.push_back(Err{});
  const bool whole = x.op >= RC_OP_ENCRYPT_SEGMENT;  // segment-level ops: the input is one segment
  size_t st = 0;
  for (;;) {
    size_t e = whole ? n : st;
    if (!whole)
      while (e < n && s[e] != '/') e++;
    Seg g;
    g.off = (uint32_t)st;
    g.len = (uint32_t)(e - st);
    bool last = e >= n;
    g.process = whole || c->dir_name_encrypt || last;
    const char* text = s + st;
    if (g.process && last && !whole) {  // encryptFileName / decryptFileName strip the version (:496-507)
      size_t at;
      if (version_match(text, g.len) && version_remove(text, g.len, &at)) {
        g.has_ver = true;
        g.ver = (uint32_t)(st + at);
        size_t o = ch.own.size();
        ch.own.append(text, at);
        ch.own.append(text + at + kVersionLen, g.len - at - kVersionLen);
        g.owned = true;
        g.off = (uint32_t)o;
        g.len -= (uint32_t)kVersionLen;
      }
    }
    if (g.process) {
      const char* t = g.owned ? ch.own.data() + g.off : s + g.off;
      if (x.standard) {
        if (g.len == 0) {
          // encryptSegment("") == decryptSegment("") == "" (cipher.go:281, :294)
        } else if (x.enc_dir)
          seg_encrypt_prepare(g, t, ch.batch);
        else
          seg_decrypt_prepare(c, g, t, ch.batch);
      } else {
        std::string in(t, g.len), out;
        if (x.enc_dir)
          out = obfuscate(c, in);
        else
          g.err = deobfuscate(c, in, &out);
        g.out_off = (uint32_t)ch.segout.size();
        g.out_len = (uint32_t)out.size();
        ch.segout += out;
      }
    }
    ch.segs.push_back(g);
    if (last) break;
    st = e + 1;
  }
}

// Phase C for input k: encode / unpad each segment, first error wins, reassemble with '/'.
void finish_input(const Ctx& x, Chunk& ch, size_t k, const char* s) {
  if (ch.direct[k]) return;
  const rc_cipher* c = x.c;
  size_t start = ch.res.size();
  Err first;
  uint32_t e = k + 1 < ch.seg0.size() ? ch.seg0[k + 1] : (uint32_t)ch.segs.size();
  for (uint32_t q = ch.seg0[k]; q < e; q++) {
    Seg& g = ch.segs[q];
    if (q != ch.seg0[k]) ch.res += '/';
    size_t at = ch.res.size();
    if (!g.process) {
      ch.res.append(s + g.off, g.len);
      continue;
    }
    if (g.err.code == RC_NIL && g.gpu) {
      const uint8_t* p = ch.batch.get(g.slot);
      size_t len = (size_t)ch.batch.desc[g.slot].nblk * kNameBlock;
      if (x.enc_dir) {
        encode_append(c->name_enc, p, len, ch.res);
      } else {  // pkcs7.Unpad(16)
        int pad = p[len - 1];
        if (pad > kNameBlock) {
          g.err = {RC_ERR_PKCS7_TOO_LONG, 0};
        } else if (pad == 0) {
          g.err = {RC_ERR_PKCS7_TOO_SHORT, 0};
        } else {
          for (int i = 0; i < pad; i++)
            if (p[len - 1 - i] != pad) {
              g.err = {RC_ERR_PKCS7_NOT_ALL_THE_SAME, 0};
              break;
            }
        }
        if (g.err.code == RC_NIL) ch.res.append((const char*)p, len - pad);
      }
    } else if (g.err.code == RC_NIL) {
      ch.res.append(ch.segout, g.out_off, g.out_len);
    }
    if (g.err.code != RC_NIL) {  // decryptFileName returns at the first failing segment
      first = g.err;
      break;
    }
    if (g.has_ver) version_add_at(ch.res, at, s + g.ver);
  }
  if (first.code != RC_NIL) ch.res.resize(start);
  ch.roff[k] = start;
  ch.rlen[k] = (uint32_t)(ch.res.size() - start);
  ch.err[k] = first;
}

}  // namespace

struct rc_names {
  std::vector<Chunk> chunks;
  double kernel_ms = 0;
};

extern "C" {

int32_t rc_new_name_encryption_mode(const char* s, int32_t* mode) {
  std::string v = s ? s : "";
  for (auto& ch : v) ch = (char)tolower((unsigned char)ch);
  if (v == "off") *mode = RC_NAME_OFF;
  else if (v == "standard") *mode = RC_NAME_STANDARD;
  else if (v == "obfuscate") *mode = RC_NAME_OBFUSCATE;
  else return RC_ERR_UNKNOWN_MODE;
  return RC_NIL;
}

int32_t rc_new_name_encoding(const char* s, int32_t* enc) {
  std::string v = s ? s : "";
  for (auto& ch : v) ch = (char)tolower((unsigned char)ch);
  if (v == "base32") *enc = RC_ENC_BASE32;
  else if (v == "base64") *enc = RC_ENC_BASE64;
  else if (v == "base32768") *enc = RC_ENC_BASE32768;
  else return RC_ERR_UNKNOWN_ENCODING;
  return RC_NIL;
}

void rc_cipher_set_name_encryption(rc_cipher* c, int32_t mode, int32_t dir_name_encrypt, int32_t enc) {
  c->mode = mode;
  c->dir_name_encrypt = dir_name_encrypt != 0;
  c->name_enc = enc;
}

// setEncryptedSuffix (cipher.go:207-217)
void rc_cipher_set_encrypted_suffix(rc_cipher* c, const char* suffix) {
  std::string s = suffix ? suffix : "";
  std::string low = s;
  for (auto& ch : low) ch = (char)tolower((unsigned char)ch);
  if (low == "none") {
    c->encrypted_suffix.clear();
    return;
  }
  if (s.empty() || s[0] != '.') s = "." + s;  // the reference logs ErrorSuffixMissingDot
  c->encrypted_suffix = s;
}

int64_t rc_name_encode(int32_t enc, const uint8_t* src, uint64_t n, char* out, uint64_t cap) {
  std::string s = encode(enc, src, n);
  if (out) memcpy(out, s.data(), s.size() < cap ? s.size() : cap);
  return (int64_t)s.size();
}

int32_t rc_name_decode(int32_t enc, const char* s, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len,
                       int64_t* err_arg) {
  std::vector<uint8_t> v;
  Err e = decode(enc, s ? s : "", s ? n : 0, v);
  if (out && !v.empty()) memcpy(out, v.data(), v.size() < cap ? v.size() : cap);
  if (out_len) *out_len = v.size();
  if (err_arg) *err_arg = e.arg;
  return e.code;
}

int32_t rc_names_run(rc_cipher* c, int32_t op, uint64_t n, const char* const* in, const uint64_t* in_len,
                     rc_names** out) {
  if (!c || !out || (n && (!in || !in_len)) || op < 0 || op > RC_OP_DEOBFUSCATE_SEGMENT) return RC_ERR_INVALID;
  *out = nullptr;
  for (uint64_t i = 0; i < n; i++)
    if (in_len[i] > 0xFFFFFFF0u || (in_len[i] && !in[i])) return RC_ERR_INVALID;
  Ctx x;
  x.c = c;
  x.op = op;
  x.enc_dir = op == RC_OP_ENCRYPT_FILE_NAME || op == RC_OP_ENCRYPT_DIR_NAME || op == RC_OP_ENCRYPT_SEGMENT ||
              op == RC_OP_OBFUSCATE_SEGMENT;
  x.standard = op == RC_OP_ENCRYPT_SEGMENT || op == RC_OP_DECRYPT_SEGMENT ||
               (op <= RC_OP_DECRYPT_DIR_NAME && c->mode == RC_NAME_STANDARD);
  // RCLONE_AMD_NAME_TIMING=1: per-phase wall times of each call on stderr (measurement aid)
  static const bool timing = [] {
    const char* v = getenv("RCLONE_AMD_NAME_TIMING");
    return v && atoi(v) != 0;
  }();
  const auto t_start = std::chrono::steady_clock::now();
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  rc_names* r = new rc_names();
  const size_t nchunks = (n + kChunkNames - 1) / kChunkNames;
  r->chunks.resize(nchunks);
  // host half before the kernel: split, strip versions, pad / decode, pack
  parallel_for(nchunks, [&](size_t ci) {
    Chunk& ch = r->chunks[ci];
    uint64_t i0 = ci * kChunkNames, i1 = std::min<uint64_t>(n, i0 + kChunkNames);
    ch.segs.reserve(i1 - i0);
    ch.seg0.reserve(i1 - i0);
    ch.direct.reserve(i1 - i0);
    ch.roff.reserve(i1 - i0);
    ch.rlen.reserve(i1 - i0);
    ch.err.reserve(i1 - i0);
    ch.batch.desc.reserve(i1 - i0);
    ch.batch.data.reserve((i1 - i0) * 48);
    for (uint64_t i = i0; i < i1; i++) prepare_input(x, ch, in[i], in_len[i]);
  });
  const double t_prep = ms_since(t_start);
  std::vector<SegBatch*> parts(nchunks);
  for (size_t ci = 0; ci < nchunks; ci++) parts[ci] = &r->chunks[ci].batch;
  const auto t_eme0 = std::chrono::steady_clock::now();
  int32_t rc = run_eme(c, x.enc_dir, parts, &r->kernel_ms);
  const double t_eme = ms_since(t_eme0);
  if (rc != RC_NIL) {
    delete r;
    return rc;
  }
  // host half after the kernel: encode / unpad, first error per name, reassemble
  parallel_for(nchunks, [&](size_t ci) {
    Chunk& ch = r->chunks[ci];
    uint64_t i0 = ci * kChunkNames, i1 = std::min<uint64_t>(n, i0 + kChunkNames);
    ch.res.reserve(ch.res.size() + ch.batch.data.size() * 2 + (i1 - i0) * 8);
    for (uint64_t i = i0; i < i1; i++) finish_input(x, ch, i - i0, in[i]);
    std::vector<Seg>().swap(ch.segs);
    std::vector<uint32_t>().swap(ch.seg0);
    std::string().swap(ch.own);
    std::string().swap(ch.segout);
    ch.batch = SegBatch();
  });
  if (timing)
    fprintf(stderr, "rc_names_run op %d n %llu: prepare %.2f ms, eme (pack + copies + kernel %.2f + unpack) %.2f ms, "
            "finish %.2f ms\n", (int)op, (unsigned long long)n, t_prep, r->kernel_ms, t_eme,
            ms_since(t_start) - t_prep - t_eme);
  *out = r;
  return RC_NIL;
}

void rc_names_get(const rc_names* r, uint64_t i, const char** s, uint64_t* len, int32_t* err, int64_t* err_arg) {
  const Chunk& ch = r->chunks[i / kChunkNames];
  uint64_t k = i % kChunkNames;
  if (s) *s = ch.res.data() + ch.roff[k];
  if (len) *len = ch.rlen[k];
  if (err) *err = ch.err[k].code;
  if (err_arg) *err_arg = ch.err[k].arg;
}

double rc_names_kernel_ms(const rc_names* r) { return r->kernel_ms; }

void rc_names_free(rc_names* r) { delete r; }

}  // extern "C"
