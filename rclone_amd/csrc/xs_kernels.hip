// xs_kernels.hip -- CDNA4 (gfx950) kernels for rclone's crypt data path.
//
// What is computed: NaCl secretbox (XSalsa20 + Poly1305) of every <=64 KiB crypt block,
// exactly as backend/crypt/cipher.go:737 (secretbox.Seal) and :880 (secretbox.Open) apply
// it, with block i of an object using nonce0 + i (cipher.go:665-678).
//
// Structure (see DESIGN.md "Kernels"):
//   xs_keygen  one lane per crypt block: per-block nonce, HSalsa20 subkey, keystream
//              block 0 (Poly1305 key r||s), keystream block 1024 words 0..7 (the last
//              two 16-byte chunks of a full block) and the Poly1305 power tables the
//              main kernel needs (r, r^253, r^0..31, r^(32a)).  ~2% of the work.
//   xs_seal / xs_open   one 64 KiB block per wave64 (four per 256-lane workgroup).  Lane l owns the
//              Salsa20 keystream blocks K = l + 64*s (s = 0..15), i.e. message chunks
//              4K-2 .. 4K+1 (16 bytes each, offset by the 32-byte Poly1305 key).  A lane
//              keeps the whole 16-word Salsa20 state in VGPRs; key/nonce words are
//              wave-uniform and live in SGPRs.  Each 4 KiB group is staged through LDS with
//              1 KiB-contiguous loads and stores.  Poly1305 of a full block runs on the
//              matrix cores (crypt_block_mfma): the chunk sums against the powers r^(64k)
//              are an i8 GEMM on v_mfma_i32_16x16x64_i8 whose B operand is each lane's own
//              ciphertext; one transpose at the end gives each lane one column to fold and
//              multiply by r^(66-g).  Partial blocks run a strided VALU Horner (uniform
//              multipliers r inside a group, r^253 between groups, final r^e from the
//              tables; the 64 partial sums added with wave shuffles).  Lane 0 adds s and
//              writes (seal) or checks (open) the tag.
//   xs_crypt_fused2  tiny batches (ranged reads): one workgroup per block, key schedule and crypt
//              in one launch.  A ranged read's open (a group window) computes its tag on the VALU
//              from a 64-entry power table, with the key setup of one- and two-block launches
//              derived on the host; whole blocks keep the matrix-core tag.
//   Poly1305 arithmetic is radix 2^26 (5 limbs): the product columns are
//   v_mad_u64_u32 chains, which measured as fast as v_alignbit on gfx950.
//
// The bound is the VALU issue rate (Salsa20 add/rotate/xor, ~90% of the instructions) at the
// power-limited clock, plus one HBM read and one HBM write per byte.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "xs_internal.h"
#include "xs_salsa_lazy.h"

// Tuning parameters (launch thresholds and occupancy targets; runtime env overrides where
// noted).  Designs that measured slower (double-buffered staging, permlane output transpose,
// XCD-remapped workgroup order, VALU data XOR, VALU Poly1305 for full blocks, the one- and
// four-crypt-wave fused kernels) are not in this file: DESIGN.md section 3 records their A/Bs.
// XS_SEAL_WPE / XS_OPEN_WPE: minimum waves per SIMD the register allocator must allow
// (amdgpu_waves_per_eu) for the seal / open kernels.
#ifndef XS_FUSED_MAX  // single-request descriptor batches up to this many blocks: keygen + crypt in one launch
#define XS_FUSED_MAX 16
#endif
#ifndef XS_KEYGEN_WIDE_MAX  // batches up to this many blocks get one keygen wave per block (latency)
#define XS_KEYGEN_WIDE_MAX 16
#endif
#ifndef XS_SPLIT_MAX  // batches up to this many blocks run four waves per block (latency)
#define XS_SPLIT_MAX 256
#endif
#ifndef XS_SEAL_WPE  // 5 waves per SIMD (<= 96 VGPRs): hides the LDS atomics' latency; paired
#define XS_SEAL_WPE 5  // -0.7% seal / -1.1% open against 4
#endif
#ifndef XS_OPEN_WPE
#define XS_OPEN_WPE 5
#endif


namespace xs {

constexpr uint32_t M26 = 0x3ffffffu;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct P5 {
  uint32_t v[5];
};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, int s) {
  return __builtin_amdgcn_alignbit(hi, lo, s);
}

#define XS_QR(a, b, c, d)        \
  b ^= rotl(a + d, 7);           \
  c ^= rotl(b + a, 9);           \
  d ^= rotl(c + b, 13);          \
  a ^= rotl(d + c, 18);

// The double-round loop is deliberately not unrolled: fully unrolled, the scheduler hoists
// across rounds and the kernel needs ~90 VGPRs; rolled it needs ~20 and measured faster.
__device__ __forceinline__ void salsa_rounds_n(uint32_t (&x)[16], int nd) {
#pragma unroll 1
  for (int i = 0; i < nd; i++) {
    XS_QR(x[0], x[4], x[8], x[12]);
    XS_QR(x[5], x[9], x[13], x[1]);
    XS_QR(x[10], x[14], x[2], x[6]);
    XS_QR(x[15], x[3], x[7], x[11]);
    XS_QR(x[0], x[1], x[2], x[3]);
    XS_QR(x[5], x[6], x[7], x[4]);
    XS_QR(x[10], x[11], x[8], x[9]);
    XS_QR(x[15], x[12], x[13], x[14]);
  }
}

__device__ __forceinline__ void salsa_rounds(uint32_t (&x)[16]) { salsa_rounds_n(x, 10); }

// The same 20 rounds through the deferred-XOR double rounds of xs_salsa_lazy.h.  For one state in
// one wave (latency, not throughput: HSalsa20 and the keystream blocks of keygen_wave) the plain
// form is compiled into a single dependent chain (~4 us); this one schedules as ~2 us.
__device__ __forceinline__ void salsa_rounds_lazy(uint32_t (&x)[16]) {
  uint32_t t[16];
  xs_salsa_dr_lazy_enter(x, t);
#pragma unroll 1
  for (int i = 0; i < 9; i++) xs_salsa_dr_lazy(x, t);
#pragma unroll
  for (int i = 0; i < 16; i++)
    if ((XS_LAZY_MASK >> i) & 1u) x[i] ^= t[i];
}

constexpr uint32_t SIG0 = 0x61707865u, SIG1 = 0x3320646eu, SIG2 = 0x79622d32u, SIG3 = 0x6b206574u;

// A wave-uniform value handed to the compiler as lane-varying: the computation that follows runs
// on the VALU instead of the scalar unit.  For a latency-bound single state (HSalsa20 of a ranged
// read's block) the SALU is ~3x slower: no one-instruction rotate, one scalar op in flight per
// wave (measured 6.8 us vs ~2 us for the 20 rounds with phase marks, round 2).
__device__ __forceinline__ uint32_t as_varying(uint32_t x) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(x));
  return v;
}

// Salsa20/20 keystream block `ctr` for a 32-byte key (k[8]) and 8-byte nonce (n0, n1).
// Salsa20/20 keystream block `ctr` for a 32-byte key (k[8]) and 8-byte nonce (n0, n1).
__device__ __forceinline__ void salsa20_block(const uint32_t (&k)[8], uint32_t n0, uint32_t n1,
                                              uint32_t ctr, uint32_t (&out)[16]) {
  uint32_t x[16] = {SIG0, k[0], k[1], k[2], k[3], SIG1, n0, n1,
                    ctr,  0u,   SIG2, k[4], k[5], k[6], k[7], SIG3};
  salsa_rounds(x);
  out[0] = x[0] + SIG0;
  out[1] = x[1] + k[0];
  out[2] = x[2] + k[1];
  out[3] = x[3] + k[2];
  out[4] = x[4] + k[3];
  out[5] = x[5] + SIG1;
  out[6] = x[6] + n0;
  out[7] = x[7] + n1;
  out[8] = x[8] + ctr;
  out[9] = x[9];
  out[10] = x[10] + SIG2;
  out[11] = x[11] + k[4];
  out[12] = x[12] + k[5];
  out[13] = x[13] + k[6];
  out[14] = x[14] + k[7];
  out[15] = x[15] + SIG3;
}

// salsa20_block with the rounds of salsa_rounds_lazy (latency-bound single states).
__device__ __forceinline__ void salsa20_block_lazy(const uint32_t (&k)[8], uint32_t n0, uint32_t n1, uint32_t ctr,
                                                   uint32_t (&out)[16]) {
  const uint32_t in[16] = {SIG0, k[0], k[1], k[2], k[3], SIG1, n0, n1, ctr, 0u, SIG2, k[4], k[5], k[6], k[7], SIG3};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = in[i];
  salsa_rounds_lazy(x);
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

// First double round, partially evaluated.  With key and nonce wave-uniform only the block
// counter (word 8) differs between lanes; 60 of the round's 96 add/rotate/xor steps do not
// depend on it and are computed once per workgroup (SalsaPre), the other 36 per block.
struct SalsaPre {
  uint32_t k[8], n0, n1;
  uint32_t x4, u9;                 // column QR(0,4,8,12): x4 final, rotl(x4 + x0, 9)
  uint32_t x1, x2, x3;             // column-round outputs feeding row QR(0,1,2,3)
  uint32_t x4r, x5r, x6r, x7r;     // row QR(5,6,7,4): fully uniform
  uint32_t x9, x10, x11r, v9;      // row QR(10,11,8,9): first step uniform; v9 = rotl(x11r + x10, 9)
  uint32_t x13, x14, x15, w7;      // row QR(15,12,13,14): w7 = rotl(x15 + x14, 7)
};

__device__ __forceinline__ uint32_t rotl_u(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

__device__ __forceinline__ SalsaPre salsa_pre(const uint32_t (&k)[8], uint32_t n0, uint32_t n1) {
  SalsaPre p;
#pragma unroll
  for (int i = 0; i < 8; i++) p.k[i] = k[i];
  p.n0 = n0;
  p.n1 = n1;
  // column round
  uint32_t x0 = SIG0, x4 = k[3], x12 = k[5];
  x4 ^= rotl_u(x0 + x12, 7);
  p.x4 = x4;
  p.u9 = rotl_u(x4 + x0, 9);
  uint32_t x5 = SIG1, x9 = 0, x13 = k[6], x1 = k[0];
  x9 ^= rotl_u(x5 + x1, 7); x13 ^= rotl_u(x9 + x5, 9); x1 ^= rotl_u(x13 + x9, 13); x5 ^= rotl_u(x1 + x13, 18);
  uint32_t x10 = SIG2, x14 = k[7], x2 = k[1], x6 = n0;
  x14 ^= rotl_u(x10 + x6, 7); x2 ^= rotl_u(x14 + x10, 9); x6 ^= rotl_u(x2 + x14, 13); x10 ^= rotl_u(x6 + x2, 18);
  uint32_t x15 = SIG3, x3 = k[2], x7 = n1, x11 = k[4];
  x3 ^= rotl_u(x15 + x11, 7); x7 ^= rotl_u(x3 + x15, 9); x11 ^= rotl_u(x7 + x3, 13); x15 ^= rotl_u(x11 + x7, 18);
  p.x1 = x1; p.x2 = x2; p.x3 = x3;
  // row round, uniform parts
  x6 ^= rotl_u(x5 + x4, 7); x7 ^= rotl_u(x6 + x5, 9); x4 ^= rotl_u(x7 + x6, 13); x5 ^= rotl_u(x4 + x7, 18);
  p.x4r = x4; p.x5r = x5; p.x6r = x6; p.x7r = x7;
  x11 ^= rotl_u(x10 + x9, 7);
  p.x9 = x9; p.x10 = x10; p.x11r = x11; p.v9 = rotl_u(x11 + x10, 9);
  p.x13 = x13; p.x14 = x14; p.x15 = x15; p.w7 = rotl_u(x15 + x14, 7);
  return p;
}

// Keystream block `ctr` from the precomputed first-round values (bit-identical to
// salsa20_block).
__device__ __forceinline__ void salsa20_block_pre(const SalsaPre& p, uint32_t ctr, uint32_t (&out)[16]) {
  uint32_t x[16];
  // column QR(0,4,8,12) lane part
  x[8] = ctr ^ p.u9;
  x[12] = p.k[5] ^ rotl(x[8] + p.x4, 13);
  x[0] = SIG0 ^ rotl(x[12] + x[8], 18);
  // row QR(0,1,2,3)
  x[1] = p.x1; x[2] = p.x2; x[3] = p.x3;
  XS_QR(x[0], x[1], x[2], x[3]);
  x[4] = p.x4r; x[5] = p.x5r; x[6] = p.x6r; x[7] = p.x7r;
  // row QR(10,11,8,9)
  x[11] = p.x11r;
  x[8] ^= p.v9;
  x[9] = p.x9 ^ rotl(x[8] + x[11], 13);
  x[10] = p.x10 ^ rotl(x[9] + x[8], 18);
  // row QR(15,12,13,14)
  x[12] ^= p.w7;
  x[13] = p.x13 ^ rotl(x[12] + p.x15, 9);
  x[14] = p.x14 ^ rotl(x[13] + x[12], 13);
  x[15] = p.x15 ^ rotl(x[14] + x[13], 18);
  // double rounds 2..10 with deferred XORs (xs_salsa_lazy.h): word i is b[i] ^ t[i] when bit
  // i of XS_LAZY_MASK is set, else b[i]; the feed-forward absorbs the pending XOR (v_xad_u32)
  uint32_t t[16];
  xs_salsa_dr_lazy_enter(x, t);
#pragma unroll 1
  for (int i = 0; i < 8; i++) xs_salsa_dr_lazy(x, t);
  const uint32_t in[16] = {SIG0, p.k[0], p.k[1], p.k[2], p.k[3], SIG1, p.n0, p.n1,
                           ctr,  0u,     SIG2,   p.k[4], p.k[5], p.k[6], p.k[7], SIG3};
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if ((XS_LAZY_MASK >> i) & 1u) out[i] = xs_xad(x[i], t[i], in[i]);
    else out[i] = x[i] + in[i];
  }
}

// ---------------------------------------------------------------- Poly1305, radix 2^26
// h * m mod 2^130-5.  Limbs of h < 2^27, limbs of m < 2^26 + 2^6 (bounds keep every
// column sum < 2^58 and every carry*5 < 2^32).  Carries are folded into the next column's
// mad chain.
__device__ __forceinline__ P5 pmul(const P5& h, const P5& m) {
  const uint32_t s1 = m.v[1] * 5, s2 = m.v[2] * 5, s3 = m.v[3] * 5, s4 = m.v[4] * 5;
  uint64_t d0 = (uint64_t)h.v[0] * m.v[0] + (uint64_t)h.v[1] * s4 + (uint64_t)h.v[2] * s3 +
                (uint64_t)h.v[3] * s2 + (uint64_t)h.v[4] * s1;
  P5 o;
  o.v[0] = (uint32_t)d0 & M26;
  uint64_t d1 = (d0 >> 26) + (uint64_t)h.v[0] * m.v[1] + (uint64_t)h.v[1] * m.v[0] +
                (uint64_t)h.v[2] * s4 + (uint64_t)h.v[3] * s3 + (uint64_t)h.v[4] * s2;
  o.v[1] = (uint32_t)d1 & M26;
  uint64_t d2 = (d1 >> 26) + (uint64_t)h.v[0] * m.v[2] + (uint64_t)h.v[1] * m.v[1] +
                (uint64_t)h.v[2] * m.v[0] + (uint64_t)h.v[3] * s4 + (uint64_t)h.v[4] * s3;
  o.v[2] = (uint32_t)d2 & M26;
  uint64_t d3 = (d2 >> 26) + (uint64_t)h.v[0] * m.v[3] + (uint64_t)h.v[1] * m.v[2] +
                (uint64_t)h.v[2] * m.v[1] + (uint64_t)h.v[3] * m.v[0] + (uint64_t)h.v[4] * s4;
  o.v[3] = (uint32_t)d3 & M26;
  uint64_t d4 = (d3 >> 26) + (uint64_t)h.v[0] * m.v[4] + (uint64_t)h.v[1] * m.v[3] +
                (uint64_t)h.v[2] * m.v[2] + (uint64_t)h.v[3] * m.v[1] + (uint64_t)h.v[4] * m.v[0];
  o.v[4] = (uint32_t)d4 & M26;
  uint32_t c = (uint32_t)(d4 >> 26);
  o.v[0] += c * 5;
  c = o.v[0] >> 26;
  o.v[0] &= M26;
  o.v[1] += c;
  return o;
}

// Same product when the multiplier is wave-uniform and its 5*m limbs are precomputed.
struct PMul {
  uint32_t m[5], s[5];
};

__device__ __forceinline__ PMul pmul_prep(const P5& m) {
  PMul p;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    p.m[i] = m.v[i];
    p.s[i] = m.v[i] * 5;
  }
  return p;
}

__device__ __forceinline__ P5 pmul_u(const P5& h, const PMul& M) {
  uint64_t d0 = (uint64_t)h.v[0] * M.m[0] + (uint64_t)h.v[1] * M.s[4] + (uint64_t)h.v[2] * M.s[3] +
                (uint64_t)h.v[3] * M.s[2] + (uint64_t)h.v[4] * M.s[1];
  P5 o;
  o.v[0] = (uint32_t)d0 & M26;
  uint64_t d1 = (d0 >> 26) + (uint64_t)h.v[0] * M.m[1] + (uint64_t)h.v[1] * M.m[0] +
                (uint64_t)h.v[2] * M.s[4] + (uint64_t)h.v[3] * M.s[3] + (uint64_t)h.v[4] * M.s[2];
  o.v[1] = (uint32_t)d1 & M26;
  uint64_t d2 = (d1 >> 26) + (uint64_t)h.v[0] * M.m[2] + (uint64_t)h.v[1] * M.m[1] +
                (uint64_t)h.v[2] * M.m[0] + (uint64_t)h.v[3] * M.s[4] + (uint64_t)h.v[4] * M.s[3];
  o.v[2] = (uint32_t)d2 & M26;
  uint64_t d3 = (d2 >> 26) + (uint64_t)h.v[0] * M.m[3] + (uint64_t)h.v[1] * M.m[2] +
                (uint64_t)h.v[2] * M.m[1] + (uint64_t)h.v[3] * M.m[0] + (uint64_t)h.v[4] * M.s[4];
  o.v[3] = (uint32_t)d3 & M26;
  uint64_t d4 = (d3 >> 26) + (uint64_t)h.v[0] * M.m[4] + (uint64_t)h.v[1] * M.m[3] +
                (uint64_t)h.v[2] * M.m[2] + (uint64_t)h.v[3] * M.m[1] + (uint64_t)h.v[4] * M.m[0];
  o.v[4] = (uint32_t)d4 & M26;
  uint32_t c = (uint32_t)(d4 >> 26);
  o.v[0] += c * 5;
  c = o.v[0] >> 26;
  o.v[0] &= M26;
  o.v[1] += c;
  return o;
}

// h += 16-byte chunk (LE words w0..w3) with the 2^128 pad bit (full chunks).
__device__ __forceinline__ void padd_full(P5& h, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  h.v[0] += w0 & M26;
  h.v[1] += alignbit(w1, w0, 26) & M26;
  h.v[2] += alignbit(w2, w1, 20) & M26;
  h.v[3] += alignbit(w3, w2, 14) & M26;
  h.v[4] += (w3 >> 8) | (1u << 24);
}

// h += partial chunk already padded with 0x01 at byte L (no 2^128 bit).
__device__ __forceinline__ void padd_part(P5& h, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  h.v[0] += w0 & M26;
  h.v[1] += alignbit(w1, w0, 26) & M26;
  h.v[2] += alignbit(w2, w1, 20) & M26;
  h.v[3] += alignbit(w3, w2, 14) & M26;
  h.v[4] += (w3 >> 8);
}

// ---------------------------------------------------------------- Poly1305, radix 2^32 words
struct P32 {
  uint32_t w0, w1, w2, w3, w4;
};

// radix 2^26 limbs (each < 2^27) -> radix 2^32, exact (additive repacking with carries)
__device__ __forceinline__ P32 to32(const P5& o) {
  P32 h;
  uint64_t v = (uint64_t)o.v[0] + ((uint64_t)o.v[1] << 26);
  h.w0 = (uint32_t)v;
  v = (v >> 32) + ((uint64_t)o.v[2] << 20);
  h.w1 = (uint32_t)v;
  v = (v >> 32) + ((uint64_t)o.v[3] << 14);
  h.w2 = (uint32_t)v;
  v = (v >> 32) + ((uint64_t)o.v[4] << 8);
  h.w3 = (uint32_t)v;
  h.w4 = (uint32_t)(v >> 32);
  return h;
}

// Carry-normalise limbs < 2^32 into limbs < 2^26 (+2^6 on limb 1), value mod p preserved.
__device__ __forceinline__ void pnorm(P5& h) {
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[0] += c * 5;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
}

// Fully reduce mod p = 2^130-5 (canonical limbs).
__device__ __forceinline__ P5 pcanon(P5 h) {
  pnorm(h);
  pnorm(h);
  uint32_t c;
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[0] += c * 5;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  uint32_t g0 = h.v[0] + 5; c = g0 >> 26; g0 &= M26;
  uint32_t g1 = h.v[1] + c; c = g1 >> 26; g1 &= M26;
  uint32_t g2 = h.v[2] + c; c = g2 >> 26; g2 &= M26;
  uint32_t g3 = h.v[3] + c; c = g3 >> 26; g3 &= M26;
  uint32_t g4 = h.v[4] + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1u;
  P5 o;
  o.v[0] = (h.v[0] & ~mask) | (g0 & mask);
  o.v[1] = (h.v[1] & ~mask) | (g1 & mask);
  o.v[2] = (h.v[2] & ~mask) | (g2 & mask);
  o.v[3] = (h.v[3] & ~mask) | (g3 & mask);
  o.v[4] = (h.v[4] & ~mask) | (g4 & mask);
  return o;
}

__device__ __forceinline__ void ptag(const P5& hc, const uint32_t (&s)[4], uint32_t (&tag)[4]) {
  const uint32_t w0 = hc.v[0] | (hc.v[1] << 26), w1 = (hc.v[1] >> 6) | (hc.v[2] << 20),
                 w2 = (hc.v[2] >> 12) | (hc.v[3] << 14), w3 = (hc.v[3] >> 18) | (hc.v[4] << 8);
  uint64_t f = (uint64_t)w0 + s[0];
  tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + s[1] + (f >> 32);
  tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + s[2] + (f >> 32);
  tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + s[3] + (f >> 32);
  tag[3] = (uint32_t)f;
}

// ---------------------------------------------------------------- matrix-core Poly1305 tables
// Full-block tag as h = sum_g r^(66-g) T_g (+ chunks 4094, 4095), column g = (c+2) mod 64,
// row p = (c+2) / 64, T_g = sum_p (c_{p,g} + 2^128) W_{63-p}, W_k = r^(64k).  The kernel gets
// sum_p c_{p,g} W_{63-p} from i8 MFMAs over the ciphertext bytes biased to signed (c - 128),
// accumulators started at 2^24; corr collects every key-only term:
//   corr = S * (E * sum_k W_k - B) - 2^128 (r^66 + r^65) W_63,   S = sum_{e=3..66} r^e,
// E = 128*(1 + 256 + ... + 256^15) + 2^128 (byte bias and pad bit of every row),
// B = 2^24 * (1 + 256 + ... + 256^31) (accumulator bias).  The key slots (row 0, columns 0
// and 1) are fed as zero bytes; only their pad bits need removing.
__device__ __constant__ uint32_t kE[5] = {0x808080u, 0x202020u, 0x80808u, 0x2020202u, 0x1808080u};
__device__ __constant__ uint32_t kB[5] = {0x242d2d0u, 0x909090u, 0x242424u, 0x1090909u, 0x2424242u};

// a - b mod p (b canonical): a + 4p - b, limbs < 2^29, then normalised
__device__ __forceinline__ P5 psub(const P5& a, const P5& b) {
  P5 o;
  o.v[0] = a.v[0] + 0xFFFFFECu - b.v[0];
#pragma unroll
  for (int i = 1; i < 5; i++) o.v[i] = a.v[i] + 0xFFFFFFCu - b.v[i];
  pnorm(o);
  return o;
}

// radix-2^26 limbs of a 16-byte little-endian chunk without the pad bit
__device__ __forceinline__ P5 chunk26(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  P5 o;
  o.v[0] = w0 & M26;
  o.v[1] = alignbit(w1, w0, 26) & M26;
  o.v[2] = alignbit(w2, w1, 20) & M26;
  o.v[3] = alignbit(w3, w2, 14) & M26;
  o.v[4] = w3 >> 8;
  return o;
}

// Full-block tables and correction.  The Toeplitz weights W_k = r^(64k) (k = 0..63) are
// A[k&7] B[k>>3] and the column exponents r^e (e = 3..66) are C[e&7] D[e>>3]; the kernel forms
// the one product each lane needs.  S = sum_{e=3..66} r^e = r^3 (1 + r^32) (sum C)(D0+..+D3),
// sum_k W_k = (sum A)(sum B).  SEAL: the key slots hash the keystream words that the
// kernel's zeroed staging slot XORs into them (chunk -2 = ks[0..3] at exponent 4098, chunk -1 =
// ks[4..7] at 4097), so corr also removes W_63 (ks_lo r^66 + ks_hi r^65); OPEN hashes zero
// bytes there (the staged wire data of those slots is zero).
__device__ __forceinline__ void put5(uint32_t (&dst)[5], const P5& v) {
#pragma unroll
  for (int i = 0; i < 5; i++) dst[i] = v.v[i];
}

__device__ __forceinline__ void add5(P5& a, const P5& b) {
#pragma unroll
  for (int i = 0; i < 5; i++) a.v[i] += b.v[i];
}

__device__ void full_corr(bool seal, P5 sumA, P5 sumB, P5 sumC, P5 sumD4, const P5& r3, const P5& r32,
                          const P5& r65, const P5& r66, const P5& W63, const uint32_t (&ks)[16], BlockKey* __restrict__ o);

__device__ void full_tables(bool seal, const P5& r, const uint32_t (&ks)[16], BlockKey* __restrict__ o) {
  P5 one;
  one.v[0] = 1; one.v[1] = one.v[2] = one.v[3] = one.v[4] = 0;
  // C_b = r^b
  P5 p = one, sumC = one;
  put5(o->full.C[0], one);
  for (int b = 1; b < 8; b++) {
    p = pmul(p, r);
    put5(o->full.C[b], p);
    add5(sumC, p);
  }
  const P5 r3 = pmul(pmul(r, r), r);
  const P5 r8 = pmul(p, r);
  // D_a = r^(8a), a = 0..8
  P5 q = one, sumD4 = one, r32 = one;
  put5(o->full.D[0], one);
  for (int a = 1; a <= 8; a++) {
    q = pmul(q, r8);
    put5(o->full.D[a], q);
    if (a < 4) add5(sumD4, q);
    if (a == 4) r32 = q;
  }
  const P5 r64 = q;
  // A_i = r^(64i), B_j = r^(512j)
  P5 w = one, sumA = one;
  put5(o->full.A[0], one);
  for (int i = 1; i < 8; i++) {
    w = pmul(w, r64);
    put5(o->full.A[i], w);
    add5(sumA, w);
  }
  const P5 r512 = pmul(w, r64);
  P5 v = one, sumB = one;
  put5(o->full.B[0], one);
  for (int j = 1; j < 8; j++) {
    v = pmul(v, r512);
    put5(o->full.B[j], v);
    add5(sumB, v);
  }
  const P5 W63 = pmul(w, v);
  const P5 r65 = pmul(r64, r);
  full_corr(seal, sumA, sumB, sumC, sumD4, r3, r32, r65, pmul(r65, r), W63, ks, o);
}

// corr from the table sums (sumA = sum A_i, sumB = sum B_j, sumC = sum C_b, sumD4 = D0+..+D3)
// and r^3, r^32, r^65, r^66, r^4032 = W_63 (any pmul-bounded representatives).
__device__ void full_corr(bool seal, P5 sumA, P5 sumB, P5 sumC, P5 sumD4, const P5& r3, const P5& r32,
                          const P5& r65, const P5& r66, const P5& W63, const uint32_t (&ks)[16], BlockKey* __restrict__ o) {
  pnorm(sumA);
  pnorm(sumB);
  const P5 SW = pcanon(pmul(sumA, sumB));
  pnorm(sumC);
  pnorm(sumD4);
  P5 one_r32 = r32;
  one_r32.v[0] += 1;
  const P5 S = pcanon(pmul(pmul(pmul(r3, sumC), sumD4), one_r32));
  P5 E, B, two128;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    E.v[i] = kE[i];
    B.v[i] = kB[i];
    two128.v[i] = 0;
  }
  two128.v[4] = 1u << 24;  // 2^128 = 2^(104 + 24)
  const P5 es_b = pcanon(psub(pcanon(pmul(E, SW)), B));
  const P5 a = pcanon(pmul(S, es_b));
  P5 kk = r65;
  add5(kk, r66);
  pnorm(kk);
  kk = pmul(two128, kk);
  if (seal) {  // + ks_lo r^66 + ks_hi r^65 (the key-slot bytes; their pad bits are the 2^128 term)
    add5(kk, pmul(chunk26(ks[0], ks[1], ks[2], ks[3]), r66));
    add5(kk, pmul(chunk26(ks[4], ks[5], ks[6], ks[7]), r65));
    pnorm(kk);
  }
  const P5 b = pcanon(pmul(kk, W63));
  const P5 c = pcanon(psub(a, b));
  put5(o->corr, c);
}

// ---------------------------------------------------------------- keygen
// One lane per crypt block.  MODE: 0 object seal, 1 object open, 2 descriptor seal,
// 3 descriptor open.  Object mode derives nonce, offsets and length from the block
// index (cipher.go:665-678 nonce.add; :1121 EncryptedSize layout).
// A descriptor's nonce, offsets and length (MODE 2 seal, 3 open); false when it fails validation
// (bounds + 16-byte payload alignment).  bounds carries {src_len, dst_len, src base misalignment,
// dst base misalignment}.
template <int MODE>
__device__ __forceinline__ bool desc_params(const xs_block_desc& d, const NonceArg& bounds, uint32_t (&n)[6],
                                            uint64_t& src, uint64_t& dst, uint32_t& len) {
#pragma unroll
  for (int i = 0; i < 6; i++) {
    n[i] = (uint32_t)d.nonce[4 * i] | ((uint32_t)d.nonce[4 * i + 1] << 8) | ((uint32_t)d.nonce[4 * i + 2] << 16) |
           ((uint32_t)d.nonce[4 * i + 3] << 24);
  }
  src = d.src_off;
  dst = d.dst_off;
  len = d.len;
  const uint64_t src_len = ((uint64_t)bounds.n[1] << 32) | bounds.n[0];
  const uint64_t dst_len = ((uint64_t)bounds.n[3] << 32) | bounds.n[2];
  const uint64_t in_need = (uint64_t)len + (MODE == 3 ? XS_BLOCK_HDR : 0u);
  const uint64_t out_need = (uint64_t)len + (MODE == 2 ? XS_BLOCK_HDR : 0u);
  const uint64_t in_pay = src + (MODE == 3 ? XS_BLOCK_HDR : 0u) + bounds.n[4];
  const uint64_t out_pay = dst + (MODE == 2 ? XS_BLOCK_HDR : 0u) + bounds.n[5];
  const bool bad = len == 0 || len > XS_BLOCK_DATA || src > src_len || in_need > src_len - src || dst > dst_len ||
                   out_need > dst_len - dst || (in_pay & 15u) || (out_pay & 15u);
  return !bad;
}

// Block b's nonce, offsets and length; false for a descriptor that fails validation.
template <int MODE>
__device__ __forceinline__ bool block_params(const NonceArg& nonce0, uint64_t first_block, uint64_t total_len,
                                             const xs_block_desc* __restrict__ desc, uint64_t b, uint32_t (&n)[6],
                                             uint64_t& src, uint64_t& dst, uint32_t& len) {
  if constexpr (MODE < 2) {
    // 192-bit little-endian nonce0 + (first_block + b) == nonce.add (cipher.go:665)
    uint64_t add = first_block + b;
    uint64_t lo = ((uint64_t)nonce0.n[1] << 32) | nonce0.n[0];
    uint64_t sum = lo + add;
    uint32_t carry = sum < lo ? 1u : 0u;
    n[0] = (uint32_t)sum;
    n[1] = (uint32_t)(sum >> 32);
#pragma unroll
    for (int i = 2; i < 6; i++) {
      uint32_t v = nonce0.n[i] + carry;
      carry = (carry && v == 0) ? 1u : 0u;
      n[i] = v;
    }
    if constexpr (MODE == 0) {
      src = b * XS_BLOCK_DATA;
      dst = b * XS_BLOCK_SIZE;
      uint64_t rem = total_len - src;
      len = (uint32_t)(rem < XS_BLOCK_DATA ? rem : XS_BLOCK_DATA);
    } else {
      src = b * XS_BLOCK_SIZE;
      dst = b * XS_BLOCK_DATA;
      uint64_t rem = total_len - src;
      len = (uint32_t)(rem < XS_BLOCK_SIZE ? rem : XS_BLOCK_SIZE) - XS_BLOCK_HDR;
    }
  } else {
    return desc_params<MODE>(desc[b], nonce0, n, src, dst, len);
  }
  return true;
}

template <int MODE>
__global__ void __launch_bounds__(64) xs_keygen(KeyArg key, NonceArg nonce0, uint64_t first_block,
                                                uint64_t total_len, uint64_t nblocks,
                                                const xs_block_desc* __restrict__ desc,
                                                BlockKey* __restrict__ out) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  uint32_t n[6];
  uint64_t src, dst;
  uint32_t len;
  if (!block_params<MODE>(nonce0, first_block, total_len, desc, b, n, src, dst, len)) {
    out[b].flags = 1;
    out[b].len = 0;
    return;
  }
  // HSalsa20(key, nonce[0:16]) -> subkey
  uint32_t x[16] = {SIG0, key.k[0], key.k[1], key.k[2], key.k[3], SIG1, n[0], n[1],
                    n[2], n[3],     SIG2,     key.k[4], key.k[5], key.k[6], key.k[7], SIG3};
  salsa_rounds(x);
  uint32_t sk[8] = {x[0], x[5], x[10], x[15], x[6], x[7], x[8], x[9]};
  uint32_t ks[16];
  salsa20_block(sk, n[4], n[5], 0u, ks);
  BlockKey* o = out + b;
#pragma unroll
  for (int i = 0; i < 8; i++) o->subkey[i] = sk[i];
  o->n2[0] = n[4];
  o->n2[1] = n[5];
  o->len = len;
  o->flags = 0;
  o->src = src;
  o->dst = dst;
#pragma unroll
  for (int i = 0; i < 4; i++) o->s[i] = ks[4 + i];
  // clamp r (bytes 0..15 of keystream block 0) into radix-2^26 limbs
  P5 r;
  r.v[0] = ks[0] & 0x3ffffffu;
  r.v[1] = alignbit(ks[1], ks[0], 26) & 0x3ffff03u;
  r.v[2] = alignbit(ks[2], ks[1], 20) & 0x3ffc0ffu;
  r.v[3] = alignbit(ks[3], ks[2], 14) & 0x3f03fffu;
  r.v[4] = (ks[3] >> 8) & 0x00fffffu;
  if (len > XS_BLOCK_DATA - 32) {
    uint32_t ks2[16];
    salsa20_block(sk, n[4], n[5], 1024u, ks2);
#pragma unroll
    for (int i = 0; i < 8; i++) o->ks1024[i] = ks2[i];
  }
#pragma unroll
  for (int i = 0; i < 5; i++) o->r[i] = r.v[i];
  if (len == XS_BLOCK_DATA) {
    full_tables(MODE == 0 || MODE == 2, r, ks, o);
    return;
  }
  // partial block: power tables for the VALU Horner.  pmul outputs (limbs < 2^26, limb 1 <
  // 2^26 + 2^6) are valid multipliers, so the chains stay uncanonicalised.
  P5 p, r29;
  p.v[0] = 1; p.v[1] = 0; p.v[2] = 0; p.v[3] = 0; p.v[4] = 0;
  r29 = p;
  for (int i = 0; i < 32; i++) {
    put5(o->part.T1[i], p);
    if (i == 29) r29 = p;
    if (i < 31) p = pmul(p, r);
  }
  const P5 r32 = pmul(p, r);
  p.v[0] = 1; p.v[1] = 0; p.v[2] = 0; p.v[3] = 0; p.v[4] = 0;
  P5 r224 = p;
  for (int a = 0; a < 8; a++) {
    put5(o->part.T2[a], p);
    if (a == 7) r224 = p;
    if (a < 7) p = pmul(p, r32);
  }
  // r^253 = r^224 * r^29: the Horner gap between a lane's consecutive chunk groups
  // (64 lanes per block, 4 chunks per group: 4*64 - 3)
  put5(o->R, pmul(r224, r29));
}

// ---------------------------------------------------------------- keygen, one wave per block
// For small batches (ranged reads, a decrypter's last blocks) the one-lane-per-block keygen is a
// single lane's dependent chain (~50 field multiplies after three Salsa20 cores).  Here the 64
// lanes of a wave share one block: lanes < 32 make keystream block 0 while lanes >= 32 make
// block 1024 (one Salsa20 latency instead of two), and the table entries are built across
// lanes (a wave issues one pmul for all lanes at once): full blocks in 13 pmul steps (levels
// of base^0..base^8 for the bases r, r^8, r^64, r^512, three steps each, spare lanes building
// the correction term's products in the same instructions, then one step for r^3 and r^4096)
// instead of the ~45 of full_tables' chains; partial blocks (lane 0..31 T1[i] = r^i, 32..39
// T2[a] = r^(32a), 40 R = r^253) by square-and-multiply per lane, 8 steps.  The entries are
// other representatives of the same residues (pmul-bounded, as the crypt kernels accept); corr
// is canonical, so tags and ciphertext equal the narrow keygen's.
// The body: one wave (lanes l = threadIdx.x & 63) builds block b's key schedule into *o (global
// memory, or LDS in the fused kernels).

typedef __attribute__((address_space(3))) uint32_t lds_u32;
// Wait until another wave of the workgroup raised *flag (LDS), then read the 8-word subkey it
// published at sk (LDS).  Plain LDS reads here would make the compiler first wait for this wave's
// outstanding LDS-DMA loads (vmcnt), since they could alias: inline ds_reads, lgkmcnt only.
__device__ __forceinline__ void lds_wait_flag(const uint32_t* flag) {
  const uint32_t fa = (uint32_t)(uintptr_t)(const lds_u32*)flag;
  for (;;) {
    uint32_t f;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(f) : "v"(fa) : "memory");
    if (__builtin_amdgcn_readfirstlane(f) != 0u) break;
    __builtin_amdgcn_s_sleep(1);
  }
}
// Raise *flag (LDS) once this wave's earlier LDS writes have completed.  Not a release: that would
// also wait for the wave's outstanding global loads (vmcnt), the PCIe round trip here.  Inline
// ds_write for the same reason as the reads above: a compiler-visible store to LDS (even a relaxed
// atomic) gets a vmcnt(0) first, since the wave's LDS-DMA loads might target the same word.
__device__ __forceinline__ void lds_raise_flag(uint32_t* flag) {
  const uint32_t fa = (uint32_t)(uintptr_t)(lds_u32*)flag;
  asm volatile("s_waitcnt lgkmcnt(0)\n\tds_write_b32 %0, %1" : : "v"(fa), "v"(1u) : "memory");
}
__device__ __forceinline__ void lds_wait_subkey(const uint32_t* flag, const uint32_t* sk, uint32_t out[8]) {
  const uint32_t ka = (uint32_t)(uintptr_t)(const lds_u32*)sk;
  lds_wait_flag(flag);
  uint4 a, b;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(a), "=&v"(b) : "v"(ka) : "memory");
  out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
  out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
}

struct KgNoMid {
  __device__ void operator()() const {}
};
template <int MODE, class Mid = KgNoMid>
__device__ __forceinline__ void keygen_wave_body(const KeyArg& key, const uint32_t n[6], uint64_t src, uint64_t dst,
                                                 uint32_t len, BlockKey* o, const uint32_t* sk_lds,
                                                 const uint32_t* sk_flag, const Mid& mid = Mid(),
                                                 uint32_t* cd_flag = nullptr, bool use_kp = false,
                                                 const XsKeyPre& kp = XsKeyPre{});

// sk_lds / sk_flag (LDS, optional): take the HSalsa20 subkey another wave of the workgroup derives
// for the same block (its LDS writes completed, then *sk_flag raised) instead of computing it
// again on a shared SIMD.
template <int MODE>
__device__ __forceinline__ void keygen_wave(const KeyArg& key, const NonceArg& nonce0, uint64_t first_block,
                                            uint64_t total_len, const xs_block_desc* __restrict__ desc,
                                            uint64_t b, BlockKey* o,
                                            const uint32_t* sk_lds = nullptr, const uint32_t* sk_flag = nullptr) {
  const uint32_t l = threadIdx.x & 63u;
  uint32_t n[6];
  uint64_t src, dst;
  uint32_t len;
  if (!block_params<MODE>(nonce0, first_block, total_len, desc, b, n, src, dst, len)) {
    if (l == 0) {
      o->flags = 1;
      o->len = 0;
    }
    return;
  }
  keygen_wave_body<MODE>(key, n, src, dst, len, o, sk_lds, sk_flag);
}

// The key schedule of one block whose descriptor fields are already known (and valid).  For a
// full block, mid() runs once the A and B power tables are in *o (before C, D and the correction
// term): the fused kernel builds its Toeplitz table there and lets the crypt waves go on.  With
// use_kp, kp is the block's key setup derived on the host (XsKeyPre): no Salsa20 core here then.
template <int MODE, class Mid>
__device__ __forceinline__ void keygen_wave_body(const KeyArg& key, const uint32_t n[6], uint64_t src, uint64_t dst,
                                                 uint32_t len, BlockKey* o, const uint32_t* sk_lds,
                                                 const uint32_t* sk_flag, const Mid& mid, uint32_t* cd_flag,
                                                 bool use_kp, const XsKeyPre& kp) {
  const uint32_t l = threadIdx.x & 63u;
  uint32_t sk[8];
  if (use_kp) {
#pragma unroll
    for (int i = 0; i < 8; i++) sk[i] = kp.sk[i];
  } else if (sk_lds) {
    lds_wait_subkey(sk_flag, sk_lds, sk);
  } else {
    uint32_t x[16] = {SIG0, key.k[0], key.k[1], key.k[2], key.k[3], SIG1, n[0], n[1],
                      n[2], n[3],     SIG2,     key.k[4], key.k[5], key.k[6], key.k[7], SIG3};
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = as_varying(x[i]);  // HSalsa20 on the VALU (latency)
    salsa_rounds_lazy(x);
    sk[0] = x[0]; sk[1] = x[5]; sk[2] = x[10]; sk[3] = x[15];
    sk[4] = x[6]; sk[5] = x[7]; sk[6] = x[8]; sk[7] = x[9];
  }
  uint32_t ks[16];
  if (use_kp) {  // words 0..7 of keystream blocks 0 (lanes < 32) and 1024 (lanes >= 32), as below
    // Both words are read as wave-uniform (scalar) loads and selected per lane afterwards: a per-lane
    // choice of address would make them vector loads of the kernel arguments (microseconds)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t a = __builtin_amdgcn_readfirstlane(kp.k0[i]), b = __builtin_amdgcn_readfirstlane(kp.k1024[i]);
      ks[i] = as_varying(l < 32 ? a : b);
    }
  } else {
    salsa20_block_lazy(sk, n[4], n[5], l < 32 ? 0u : 1024u, ks);
  }
  if (l == 32 && len > XS_BLOCK_DATA - 32) {
#pragma unroll
    for (int i = 0; i < 8; i++) o->ks1024[i] = ks[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) ks[i] = __shfl(ks[i], 0);  // block 0 words 0..7 (r, s) everywhere
  P5 r;
  r.v[0] = ks[0] & 0x3ffffffu;
  r.v[1] = alignbit(ks[1], ks[0], 26) & 0x3ffff03u;
  r.v[2] = alignbit(ks[2], ks[1], 20) & 0x3ffc0ffu;
  r.v[3] = alignbit(ks[3], ks[2], 14) & 0x3f03fffu;
  r.v[4] = (ks[3] >> 8) & 0x00fffffu;
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) o->subkey[i] = sk[i];
    o->n2[0] = n[4];
    o->n2[1] = n[5];
    o->len = len;
    o->flags = 0;
    o->src = src;
    o->dst = dst;
#pragma unroll
    for (int i = 0; i < 4; i++) o->s[i] = ks[4 + i];
#pragma unroll
    for (int i = 0; i < 5; i++) o->r[i] = r.v[i];
  }
  P5 p;
  p.v[0] = 1; p.v[1] = 0; p.v[2] = 0; p.v[3] = 0; p.v[4] = 0;
  if (len == XS_BLOCK_DATA) {
    // Level m = 0..3 (bases r, r^8, r^64, r^512) lives in lanes 9m + b holding base^b,
    // b = 0..8; three pmul steps per level (b = 2; 3, 4; 5..8), lane 9m + 8 = the next base.
    // Step st of level m multiplies by base^(2^st) = r^(2^(3m + st)): over the 12 steps these are
    // r^1, r^2, ..., r^2048, the factors of the correction term's product forms (full_corr):
    //   sum C (1 + r^32) sum D4 = prod_{i<6} (1 + r^(2^i)),  sum A sum B = prod_{6<=i<12} (1 + r^(2^i)),
    // so  corr = E r^3 prod_{i<12} (1 + r^(2^i)) - B r^3 prod_{i<6} (1 + r^(2^i)) - K,
    //   K = 2^128 (r^65 + r^66) W_63 [+ SEAL key slots] = r^4096 ((2^128 [+ ks_lo]) r^2 + (2^128 [+ ks_hi]) r).
    // Spare lanes ride along in the same pmul instructions: lane 40 accumulates the E product
    // (all 12 steps), lane 41 the B product (steps 0..5), lanes 42 / 43 the two K terms (steps
    // 1 / 0).  One more step after the levels multiplies in r^3 (lanes 40, 41) and r^4096 (lane 42);
    // then corr is two subtractions and one canonicalisation instead of a chain of products.
    constexpr uint32_t kLaneE = 40u, kLaneB = 41u, kLaneKlo = 42u, kLaneKhi = 43u;
    const bool seal = MODE == 0 || MODE == 2;
    P5 two128;
#pragma unroll
    for (int i = 0; i < 5; i++) two128.v[i] = 0;
    two128.v[4] = 1u << 24;  // 2^128 = 2^(104 + 24)
    if (l == 1) p = r;
    if (l == kLaneE) {
#pragma unroll
      for (int i = 0; i < 5; i++) p.v[i] = kE[i];
    } else if (l == kLaneB) {
#pragma unroll
      for (int i = 0; i < 5; i++) p.v[i] = kB[i];
    } else if (l == kLaneKlo || l == kLaneKhi) {
      p = two128;
      if (seal) {  // the key-slot words (chunk -2 = ks[0..3], chunk -1 = ks[4..7])
        add5(p, l == kLaneKlo ? chunk26(ks[0], ks[1], ks[2], ks[3]) : chunk26(ks[4], ks[5], ks[6], ks[7]));
      }
    }
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const uint32_t b = l - 9u * m;  // wraps for lanes below the level: not in 2..8
#pragma unroll
      for (int st = 0; st < 3; st++) {
        // operands: st 0: b=2 <- 1*1; st 1: b=3 <- 2*1, b=4 <- 2*2; st 2: b=5..8 <- 4*(b-4)
        const uint32_t lo = st == 0 ? 2u : st == 1 ? 3u : 5u, hi = st == 0 ? 2u : st == 1 ? 4u : 8u;
        const bool act = b >= lo && b <= hi;
        const int step = 3 * m + st;
        // spare lanes multiply their own value by the step's factor: (1 + a) or a
        const bool plus1 = l == kLaneE || (l == kLaneB && step < 6);
        const bool own = plus1 || (l == kLaneKlo && step == 1) || (l == kLaneKhi && step == 0);
        const uint32_t ia = 9u * m + (st == 0 ? 1u : st == 1 ? 2u : 4u);
        const uint32_t ib = own ? l : 9u * m + (act ? (st == 0 ? 1u : st == 1 ? b - 2u : b - 4u) : 0u);
        P5 a, c;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          a.v[i] = (uint32_t)__shfl((int)p.v[i], (int)ia);
          c.v[i] = (uint32_t)__shfl((int)p.v[i], (int)ib);
        }
        a.v[0] += plus1 ? 1u : 0u;
        const P5 q = pmul(a, c);
        if (act || own) p = q;
      }
      if (m == 1) {  // C[b] = lane b, D[a] = lane 9 + a are final: out now (cd_flag: LDS, raised after)
        if (l < 8) put5(o->full.C[l], p);
        else if (l >= 9 && l < 18) put5(o->full.D[l - 9], p);
        if (cd_flag) lds_raise_flag(cd_flag);
      }
      if (m == 0) {  // K = r^4096 (lane 42 + lane 43), summed in lane 42
        P5 khi;
#pragma unroll
        for (int i = 0; i < 5; i++) khi.v[i] = (uint32_t)__shfl((int)p.v[i], (int)kLaneKhi);
        if (l == kLaneKlo) {
          add5(p, khi);
          pnorm(p);
        }
      }
      if (m < 3) {  // next level: base^0 = 1, base^1 = this level's base^8
        P5 nb;
#pragma unroll
        for (int i = 0; i < 5; i++) nb.v[i] = (uint32_t)__shfl((int)p.v[i], (int)(9u * m + 8u));
        if (l == 9u * (m + 1) + 1u) p = nb;
      }
    }
    // A[i] = lane 18 + i, B[j] = lane 27 + j
    if (l >= 18 && l < 26) put5(o->full.A[l - 18], p);
    else if (l >= 27 && l < 35) put5(o->full.B[l - 27], p);
    mid();
    {  // r^3 (lane 3) into lanes 40, 41; r^4096 (lane 35) into lane 42
      const uint32_t ia = l == kLaneKlo ? 35u : 3u;
      P5 a;
#pragma unroll
      for (int i = 0; i < 5; i++) a.v[i] = (uint32_t)__shfl((int)p.v[i], (int)ia);
      const P5 q = pmul(a, p);
      if (l >= kLaneE && l <= kLaneKlo) p = q;
    }
    P5 e, bq, k;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      e.v[i] = as_varying(__builtin_amdgcn_readlane(p.v[i], kLaneE));
      bq.v[i] = as_varying(__builtin_amdgcn_readlane(p.v[i], kLaneB));
      k.v[i] = as_varying(__builtin_amdgcn_readlane(p.v[i], kLaneKlo));
    }
    // pmul outputs (limbs < 2^26 + 2^6) are valid subtrahends for psub; corr is canonical, the
    // same value full_corr gives
    const P5 cr = pcanon(psub(psub(e, bq), k));
    if (l == 0) put5(o->corr, cr);
    return;
  }
  // partial blocks (one per object at most): lane e's entry by square-and-multiply
  const uint32_t e = l < 32 ? l : l < 40 ? 32u * (l - 32u) : l == 40 ? 253u : 0u;
  P5 sq = r;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const P5 q = pmul(p, sq);
    if ((e >> j) & 1u) p = q;
    if (j < 7) sq = pmul(sq, sq);
  }
  if (l < 32) put5(o->part.T1[l], p);
  else if (l < 40) put5(o->part.T2[l - 32], p);
  else if (l == 40) put5(o->R, p);
}

template <int MODE>
__global__ void __launch_bounds__(64) xs_keygen_wide(KeyArg key, NonceArg nonce0, uint64_t first_block,
                                                     uint64_t total_len, uint64_t nblocks,
                                                     const xs_block_desc* __restrict__ desc,
                                                     BlockKey* __restrict__ out) {
  if (blockIdx.x >= nblocks) return;  // uniform per workgroup
  keygen_wave<MODE>(key, nonce0, first_block, total_len, desc, blockIdx.x, out + blockIdx.x);
}

// ---------------------------------------------------------------- main block kernel
// SEAL: in = plaintext block, out = tag(16) || ct.   OPEN: in = tag || ct, out = plaintext,
// ok[blk] = 1 if the tag verified (else the plaintext is zero-filled, the
// pass_bad_blocks contract of cipher.go:885-893).
//
// One 64 KiB block per wave64 (a 256-thread workgroup carries four blocks; no barriers).
// Group s (s = 0..15): lane l owns keystream block K = l + 64 s and message chunks
// 4K-2 .. 4K+1.  The wave's 4 KiB of input for the group is staged into its LDS slot by
// global_load_lds_dwordx4 (no VGPRs held across the 20 Salsa20 rounds), read back after the
// keystream is ready, XORed and stored.  Lane 63 also owns chunks 4094, 4095 (keystream block
// 1024, precomputed by keygen), so every lane's Horner multipliers are uniform: r inside a
// group, r^253 between groups.
// Full blocks run Poly1305 on the matrix cores (crypt_block_mfma); crypt_block below is the
// partial-block path (VALU Horner).
constexpr int STAGE_WORDS = 1024;
constexpr int WAVE_LDS_WORDS = STAGE_WORDS + 768;  // 4 KiB staging + 3 KiB Toeplitz table
constexpr int LDS_WORDS = 4 * WAVE_LDS_WORDS;
constexpr uint32_t LANES = 64, GROUPS = 16;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ uint32_t keep_mask(uint32_t L, uint32_t i) {
  // mask of the bytes of word i (bytes 4i..4i+3) that lie below L
  return (L >= 4u * i + 4u) ? 0xffffffffu : (L <= 4u * i ? 0u : ((1u << (8u * (L - 4u * i))) - 1u));
}

// A partial block (n < 65536 bytes): VALU Horner per lane over its chunks, uniform multipliers
// r inside a group and r^253 between groups, final r^e from the key schedule's T1/T2 tables.
template <bool SEAL>
__device__ __forceinline__ void crypt_block(const BlockKey* __restrict__ bk, const uint8_t* __restrict__ pin,
                                            uint8_t* __restrict__ pout, uint32_t n, uint32_t* wb, P5& h) {
  const uint32_t l = threadIdx.x & 63u;
  const int nc = (int)((n + 15u) >> 4);
  const int nfull = (int)(n >> 4);  // chunks that are whole 16-byte chunks
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = bk->subkey[i];
  const SalsaPre pre = salsa_pre(k, bk->n2[0], bk->n2[1]);
  P5 rr, RR;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    rr.v[i] = bk->r[i];
    RR.v[i] = bk->R[i];
  }
  const PMul Mr = pmul_prep(rr), MR = pmul_prep(RR);
  int c_last = -1;
  P5 t1, t2;

#pragma unroll 1
  for (int s = 0; s < (int)GROUPS; s++) {
    const uint32_t K = l + LANES * (uint32_t)s;
    const int cfirst = 4 * (int)K - 2;
    if (cfirst >= nc) break;
    // stage this group's input (whole chunks only) into the wave's LDS slot
    const uint8_t* src = pin + 64u * K - 32u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int c = cfirst + j;
      if (c >= 0 && c < nfull) __builtin_amdgcn_global_load_lds(src + 16 * j, (lds_void*)(wb + 256 * j), 16, 0, 0);
    }
    uint32_t ks[16];
    salsa20_block_pre(pre, K, ks);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t d[16];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint4 v = *reinterpret_cast<const uint4*>(wb + 256 * j + 4 * l);
      d[4 * j] = v.x; d[4 * j + 1] = v.y; d[4 * j + 2] = v.z; d[4 * j + 3] = v.w;
    }
    uint32_t plen[4];  // bytes of each chunk (16 whole, 0 absent, else partial)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int c = cfirst + j;
      plen[j] = (c < 0 || c >= nc) ? 0u : ((c < nfull) ? 16u : (n & 15u));
    }
    // the block's last chunk may be partial: byte loads by its owner
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (plen[j] != 0u && plen[j] != 16u) {
        const uint32_t off = 16u * (uint32_t)(cfirst + j);
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; i < plen[j]; i++) w[i >> 2] |= (uint32_t)pin[off + i] << (8u * (i & 3u));
        d[4 * j] = w[0]; d[4 * j + 1] = w[1]; d[4 * j + 2] = w[2]; d[4 * j + 3] = w[3];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (plen[j] == 0u) { d[4 * j] = 0; d[4 * j + 1] = 0; d[4 * j + 2] = 0; d[4 * j + 3] = 0; }
    }
    uint32_t o[16];
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = d[i] ^ ks[i];
#pragma unroll
    for (int j = 0; j < 4; j++) {  // absent chunks hash as zero; partial chunks keep L bytes
      if (plen[j] == 0u) { o[4 * j] = 0; o[4 * j + 1] = 0; o[4 * j + 2] = 0; o[4 * j + 3] = 0; }
      if (plen[j] != 16u) {
#pragma unroll
        for (int i = 0; i < 4; i++) o[4 * j + i] &= keep_mask(plen[j], (uint32_t)i);
      }
    }
    uint8_t* dst = pout + 64u * K - 32u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (plen[j] == 16u) {
        *reinterpret_cast<uint4*>(dst + 16 * j) = make_uint4(o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]);
      } else if (plen[j] != 0u) {
        for (uint32_t i = 0; i < plen[j]; i++) dst[16 * j + i] = (uint8_t)(o[4 * j + (i >> 2)] >> (8u * (i & 3u)));
      }
    }
    // Poly1305 over the ciphertext: (h + c) * r within the group, * r^253 (or r) at its end
    const uint32_t* cw = SEAL ? o : d;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (plen[j] != 0u) {
        uint32_t w0 = cw[4 * j], w1 = cw[4 * j + 1], w2 = cw[4 * j + 2], w3 = cw[4 * j + 3];
        uint32_t pad = 1u << 24;
        if (plen[j] != 16u) {  // 0x01 after the last byte, no 2^128 bit
          const uint32_t L = plen[j];
          const uint32_t bit = 1u << (8u * (L & 3u));
          w0 |= (L >> 2) == 0u ? bit : 0u;
          w1 |= (L >> 2) == 1u ? bit : 0u;
          w2 |= (L >> 2) == 2u ? bit : 0u;
          w3 |= (L >> 2) == 3u ? bit : 0u;
          pad = 0u;
        }
        h.v[0] += w0 & M26;
        h.v[1] += alignbit(w1, w0, 26) & M26;
        h.v[2] += alignbit(w2, w1, 20) & M26;
        h.v[3] += alignbit(w3, w2, 14) & M26;
        h.v[4] += (w3 >> 8) | pad;
        const bool use_R = (j == 3) && (s < (int)GROUPS - 1) && (cfirst + 4 * (int)LANES < nc);
        PMul M;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          M.m[i] = use_R ? MR.m[i] : Mr.m[i];
          M.s[i] = use_R ? MR.s[i] : Mr.s[i];
        }
        h = pmul_u(h, M);
        c_last = cfirst + j;
      }
    }
  }
  // lane 63 owns chunks 4094, 4095 (keystream block 1024 words 0..7)
  if (l == 63u && nc > 4094) {
#pragma unroll 1
    for (int j = 0; j < 2; j++) {
      const int c = 4094 + j;
      if (c >= nc) break;
      const uint32_t off = 16u * (uint32_t)c;
      const uint32_t L = (n - off) < 16u ? (n - off) : 16u;
      uint32_t w[4], o4[4];
      if (L == 16u) {
        const uint4 v = *reinterpret_cast<const uint4*>(pin + off);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
      } else {
        w[0] = w[1] = w[2] = w[3] = 0;
        for (uint32_t i = 0; i < L; i++) w[i >> 2] |= (uint32_t)pin[off + i] << (8u * (i & 3u));
      }
#pragma unroll
      for (int i = 0; i < 4; i++) o4[i] = (w[i] ^ bk->ks1024[4 * j + i]) & keep_mask(L, (uint32_t)i);
      if (L == 16u) {
        *reinterpret_cast<uint4*>(pout + off) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      } else {
        for (uint32_t i = 0; i < L; i++) pout[off + i] = (uint8_t)(o4[i >> 2] >> (8u * (i & 3u)));
      }
      uint32_t cw[4];
#pragma unroll
      for (int i = 0; i < 4; i++) cw[i] = SEAL ? o4[i] : w[i];
      if (L == 16u) {
        padd_full(h, cw[0], cw[1], cw[2], cw[3]);
      } else {
        cw[L >> 2] |= 1u << (8u * (L & 3u));
        padd_part(h, cw[0], cw[1], cw[2], cw[3]);
      }
      h = pmul_u(h, Mr);
      c_last = c;
    }
  }
  // bring the lane's partial sum to exponent 0: * r^(nc-1-c_last)
  if (c_last >= 0) {
    const uint32_t e = (uint32_t)(nc - 1 - c_last);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      t1.v[i] = bk->part.T1[e & 31u][i];
      t2.v[i] = bk->part.T2[e >> 5][i];
    }
    h = pmul(h, pmul(t1, t2));
  }
}

// ---------------------------------------------------------------- full blocks on the matrix cores
// Poly1305 of a full 64 KiB block as i8 GEMMs (algebra: mfma_tables).  Index the
// message chunks c = -2 .. 4093 by x = c + 2 = 64 p + g: row p (0..63) = one KiB of the
// keystream, column g (0..63).  Chunk c's Horner exponent is 4096 - c = 64(63-p) + (66-g), so
//   h = sum_g r^(66-g) * sum_p (c_{p,g} + 2^128) r^(64(63-p))   (+ chunks 4094, 4095).
// In super-iteration u lane l runs keystream block K = 64u + l (4 KiB contiguous per wave),
// whose chunks j = 0..3 are row 4u + (l>>4), columns 4(l&15) + j.  That is exactly the
// B-operand layout of v_mfma_i32_16x16x64_i8 (lane l: column l&15, K-group l>>4), so with
// one accumulator per (chunk j, output half mt)
//   acc[j][mt][q][n] = 2^24 + sum_p sum_a Wd_p[16mt + q - a] * (byte_a(c_{p, 4n+j}) - 128)
// the ciphertext never leaves the lane; Wd_p = the 17 signed base-256 digits of r^(64(63-p))
// (A operand: a Toeplitz window of the wave's LDS table Z, K-group kg <-> row 4u + kg).  Key
// slots (x = 0, 1) are fed as zero bytes; the key-only terms are in BlockKey::corr.
typedef int xs_v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Column value from its eight 64-bit partial words X[w] (weight 2^(32w), each < 2^50),
// reduced mod 2^130-5 (limbs < 2^26 + 2^6).
__device__ __forceinline__ P5 column_value(const uint64_t (&x)[8]) {
  uint32_t L[9];
  uint64_t c = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const uint64_t tt = x[w] + c;
    L[w] = (uint32_t)tt;
    c = tt >> 32;
  }
  L[8] = (uint32_t)c;  // < 2^19: the value is < 2^275
  uint32_t v[11];
  v[0] = L[0] & M26;
  v[1] = alignbit(L[1], L[0], 26) & M26;
  v[2] = alignbit(L[2], L[1], 20) & M26;
  v[3] = alignbit(L[3], L[2], 14) & M26;
  v[4] = alignbit(L[4], L[3], 8) & M26;
  v[5] = (L[4] >> 2) & M26;
  v[6] = alignbit(L[5], L[4], 28) & M26;
  v[7] = alignbit(L[6], L[5], 22) & M26;
  v[8] = alignbit(L[7], L[6], 16) & M26;
  v[9] = alignbit(L[8], L[7], 10) & M26;
  v[10] = L[8] >> 4;
  v[5] += 5u * v[10];  // 2^260 = 2^130 * 2^130 -> 5 * 2^130
  P5 V;
#pragma unroll
  for (int i = 0; i < 5; i++) V.v[i] = v[i] + 5u * v[i + 5];
  pnorm(V);
  return V;
}

// NSPLIT = 1: the wave does all 16 super-iterations of its block.  NSPLIT = 4 (small batches,
// latency): the block's four waves take four super-iterations each, their (linear) MFMA
// accumulators are added through LDS and wave 0 finalises; returns whether this wave finalises.
template <bool SEAL, int NSPLIT>
__device__ __forceinline__ bool crypt_block_mfma(const BlockKey* __restrict__ bk, const uint8_t* __restrict__ pin,
                                                 uint8_t* __restrict__ pout, uint32_t* wb, uint32_t* zb, P5& h,
                                                 uint32_t wave, uint32_t* lds_all) {
  static_assert(NSPLIT == 1 || NSPLIT == 4, "split factor");
  const uint32_t l = threadIdx.x & 63u, n = l & 15u, kg = l >> 4;
  const int u_begin = NSPLIT == 1 ? 0 : 4 * (int)wave, u_end = u_begin + 16 / NSPLIT;
  const bool lead = NSPLIT == 1 || wave == 0u;
  // ---- Z table: row p = l holds the signed digits D_0..D_16 of r^(64(63-p)) reversed,
  // Z[u] = D_{31-u} for 15 <= u <= 31, zero elsewhere (12 words per row).  W is stored
  // uncanonicalised (< 2^131): repack the limbs with carries, any representative works.
  {
    P5 qa, qb;
    const uint32_t k = 63u - l;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      qa.v[i] = bk->full.A[k & 7u][i];
      qb.v[i] = bk->full.B[k >> 3][i];
    }
    const P32 wq = to32(pmul(qa, qb));
    uint32_t w0 = wq.w0, w1 = wq.w1, w2 = wq.w2, w3 = wq.w3, w4 = wq.w4;
    unsigned cy;  // +0x80 in every byte, carried; flipping each byte's top bit then gives digits in [-128, 127]
    w0 = __builtin_addc(w0, 0x80808080u, 0u, &cy);
    w1 = __builtin_addc(w1, 0x80808080u, cy, &cy);
    w2 = __builtin_addc(w2, 0x80808080u, cy, &cy);
    w3 = __builtin_addc(w3, 0x80808080u, cy, &cy);
    w4 = (w4 + 0x80u + cy) ^ 0x80u;
    w0 ^= 0x80808080u;
    w1 ^= 0x80808080u;
    w2 ^= 0x80808080u;
    w3 ^= 0x80808080u;
    uint4* row = reinterpret_cast<uint4*>(zb + 12u * l);
    row[0] = make_uint4(0u, 0u, 0u, w4 << 24);
    row[1] = make_uint4(__builtin_bswap32(w3), __builtin_bswap32(w2), __builtin_bswap32(w1), __builtin_bswap32(w0));
    row[2] = make_uint4(0u, 0u, 0u, 0u);
  }
  // Staging layout (per 4 KiB group, one slot of 4 x 1 KiB): load j fetches KiB j of the group
  // contiguously, lane λ taking 16-byte chunk 64j + perm(λ), perm(λ) = 4(λ&15) + (λ>>4), which
  // lands at slot position λ; lane L then finds its own chunks 4L+i at KiB L>>4, positions
  // (L&15) + 16i (conflict-free ds_read_b128).  Outputs go back through the same positions and
  // leave in the load order, so every load and store wave-instruction covers 1 KiB.
  // The key slots (chunks -2, -1 of the block = chunks 0, 1 of group 0 = lanes 0 and 16 of
  // load 0) are never loaded or stored: zeroed here, OPEN hashes zero bytes there and SEAL the
  // keystream (keygen's corr accounts for both).
  if (l == 0u) {
    *reinterpret_cast<uint4*>(wb) = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(wb + 64) = make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = bk->subkey[i];
  const SalsaPre pre = salsa_pre(k, bk->n2[0], bk->n2[1]);
  // A window for output q = 16mt + n starts at Z byte 31 - q: words zlo .. zlo + 8 cover both
  // halves (mt = 1 at word zlo, mt = 0 at word zlo + 4), byte shift zsh
  const uint32_t zlo = (15u - n) >> 2, zsh = (31u - n) & 3u;
  // input and output addressed from 32 bytes before the block (uniform base + 32-bit offset;
  // raw buffer loads/stores measured 3-4% slower for seal, neutral for open)
  const uint8_t* pin_m32 = pin - 32;
  uint8_t* pout_m32 = pout - 32;
  const uint32_t lane_off = 16u * (4u * (l & 15u) + (l >> 4));  // perm(l) chunk, bytes
  const bool not_key = (l & 47u) != 0u;                        // not lane 0 or 16
  // this lane's Z window in row kg, as an opaque LDS address so the per-row reads below use
  // one base register and ds_read2 offsets (otherwise the compiler splits off the slot offset)
  uint32_t zaddr = (uint32_t)(uintptr_t)((const lds_u32*)zb + 12u * kg + zlo);
  asm volatile("" : "+v"(zaddr));
  const lds_u32* zl = (const lds_u32*)(uintptr_t)zaddr;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own Z / zero writes are visible
  xs_v4i acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
      for (int i = 0; i < 4; i++) acc[j][mt][i] = lead ? 1 << 24 : 0;  // the bias once per block
#pragma unroll 1
  for (int u = u_begin; u < u_end; u++) {
    const uint32_t K = 64u * u + l;
    const uint32_t goff = 4096u * (uint32_t)u + lane_off;
    uint32_t* sb = wb;
    // one 64-bit address per group: the four 1 KiB loads differ only in the instruction's
    // immediate offset (no address VALU per load).  The hardware adds that offset to the LDS
    // destination (M0) as well, so all four name the slot base and land 1 KiB apart.
    const uint8_t* gsrc = pin_m32 + goff;
    if (u > 0 || not_key) __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)sb, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)sb, 16, 1024, 0);
    __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)sb, 16, 2048, 0);
    __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)sb, 16, 3072, 0);
    uint32_t ks[16];
    salsa20_block_pre(pre, K, ks);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4* mine = reinterpret_cast<uint4*>(sb + 256 * (l >> 4) + 4 * (l & 15u));
    // The data XOR and the MFMA operand's sign bias (C = 0x80 in every byte) run on the LDS's own
    // ALU: 64-bit atomic XORs on this lane's staged words, so the VALU issues no XOR for either
    // (512 fewer VALU instructions per block; paired A/B in DESIGN.md section 3).  Chunk j, half h
    // of the lane sits at mine + 256 j + 8 h bytes.
    //   seal: ^C, ^ks, then ^C returning d^ks^C = B (the LDS ends as the ciphertext d^ks)
    //   open: ^C, ^ks returning d^C = B, then ^C (the LDS ends as the plaintext d^ks)
    // The group-0 key slots hold zeros, as with the VALU form.
    typedef __attribute__((address_space(3))) uint64_t lds_u64;
    lds_u64* m64 = (lds_u64*)mine;
    uint64_t k64[8], r64[8];
#pragma unroll
    for (int q = 0; q < 8; q++) k64[q] = (uint64_t)ks[2 * q] | ((uint64_t)ks[2 * q + 1] << 32);
    const uint64_t C64 = 0x8080808080808080ull;
#define XS_AX(q, v) __hip_atomic_fetch_xor(m64 + 32 * ((q) >> 1) + ((q) & 1), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#pragma unroll
    for (int q = 0; q < 8; q++) (void)XS_AX(q, C64);
    if (SEAL) {
#pragma unroll
      for (int q = 0; q < 8; q++) (void)XS_AX(q, k64[q]);
#pragma unroll
      for (int q = 0; q < 8; q++) r64[q] = XS_AX(q, C64);
    } else {
#pragma unroll
      for (int q = 0; q < 8; q++) r64[q] = XS_AX(q, k64[q]);
#pragma unroll
      for (int q = 0; q < 8; q++) (void)XS_AX(q, C64);
    }
#undef XS_AX
    asm volatile("" ::: "memory");  // LDS ops of one wave execute in order
    {  // the staged words are now the output: out in load order
      uint4 w[4];
#pragma unroll
      for (int j = 0; j < 4; j++) w[j] = *reinterpret_cast<const uint4*>(sb + 256 * j + 4 * l);
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (j > 0 || u > 0 || not_key) *reinterpret_cast<uint4*>(pout_m32 + goff + 1024 * j) = w[j];
    }
    uint32_t bw[16];  // the MFMA B words (biased ciphertext)
#pragma unroll
    for (int q = 0; q < 8; q++) {
      bw[2 * q] = (uint32_t)r64[q];
      bw[2 * q + 1] = (uint32_t)(r64[q] >> 32);
    }
    // A operands of row 4u + kg for both output halves
    const lds_u32* zr = zl + 48u * u;
    uint32_t z[9];
#pragma unroll
    for (int i = 0; i < 9; i++) z[i] = zr[i];
    xs_v4i A[2];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      A[1][i] = (int)__builtin_amdgcn_alignbyte(z[i + 1], z[i], zsh);
      A[0][i] = (int)__builtin_amdgcn_alignbyte(z[i + 5], z[i + 4], zsh);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      xs_v4i B;
#pragma unroll
      for (int i = 0; i < 4; i++) B[i] = (int)bw[4 * j + i];
#pragma unroll
      for (int mt = 0; mt < 2; mt++) {
        acc[j][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[mt], B, acc[j][mt], 0, 0, 0);
      }
    }
  }
  if (NSPLIT > 1) {  // add the other waves' accumulators into wave 0's
    if (!SEAL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // plaintext stores done before a zero-fill
    __syncthreads();  // every wave is past its staging and Toeplitz reads
    if (!lead) {
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
          for (int i = 0; i < 4; i++) lds_all[(wave - 1u) * 2048u + (uint32_t)(8 * j + 4 * mt + i) * 64u + l] = acc[j][mt][i];
    }
    __syncthreads();
    if (!lead) return false;
#pragma unroll
    for (int w = 0; w < NSPLIT - 1; w++)
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
          for (int i = 0; i < 4; i++) acc[j][mt][i] += (int)lds_all[(uint32_t)w * 2048u + (uint32_t)(8 * j + 4 * mt + i) * 64u + l];
  }
  // ---- transpose the partial words through the (now free) staging slot: lane (n, kg) holds,
  // for column 4n + j, the words at 2^(32(4mt + kg)); lane λ finalises column 4(λ&15) + (λ>>4).
  // (ne, kge) = (n, kg) recomputed from an opaque copy of the lane id: kept live across the group
  // loop instead, at five waves per SIMD the compiler spilled them to scratch.
  uint32_t lid = threadIdx.x & 63u;
  asm volatile("" : "+v"(lid));
  const uint32_t ne = lid & 15u, kge = lid >> 4;
  uint64_t* t64 = reinterpret_cast<uint64_t*>(wb);
  // the byte weights as opaque wave-uniform values: each term is then one v_mad_u64_u32 (a shift
  // would be a zero-extend + 64-bit shift + 64-bit add)
  uint32_t w8 = 1u << 8, w16 = 1u << 16, w24 = 1u << 24;
  asm("" : "+s"(w8), "+s"(w16), "+s"(w24));
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t sx[2];
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
      sx[mt] = (uint64_t)(uint32_t)acc[j][mt][3] * w24 +
               ((uint64_t)(uint32_t)acc[j][mt][2] * w16 +
                ((uint64_t)(uint32_t)acc[j][mt][1] * w8 + (uint64_t)(uint32_t)acc[j][mt][0]));
    *reinterpret_cast<ulonglong2*>(t64 + (((ne * 4u + j) * 4u + kge) * 2u)) = make_ulonglong2(sx[0], sx[1]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint64_t x[8];
  {
    const uint64_t* rd = t64 + (ne * 4u + kge) * 8u;  // column 4n + kg: (kg', mt) pairs for kg' = 0..3
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(rd + 2 * kk);
      x[kk] = v.x;      // mt = 0: word kk
      x[4 + kk] = v.y;  // mt = 1: word 4 + kk
    }
  }
  P5 hs;
  {
    const P5 V = column_value(x);
    const uint32_t e = 66u - (4u * ne + kge);  // column g = 4n + kg (this lane's column)
    P5 t1, t2;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      t1.v[i] = bk->full.C[e & 7u][i];
      t2.v[i] = bk->full.D[e >> 3][i];
    }
    hs = pmul(V, pmul(t2, t1));
  }
  if (l == 0u) {
#pragma unroll
    for (int i = 0; i < 5; i++) hs.v[i] += bk->corr[i];
  }
  // chunks 4094, 4095 (keystream block 1024 words 0..7): exponents 2 and 1
  if (l == 63u) {
    P5 rr, tl;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      rr.v[i] = bk->r[i];
      tl.v[i] = 0;
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t off = 16u * (4094u + j);
      const uint4 v = *reinterpret_cast<const uint4*>(pin + off);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t o4[4];
#pragma unroll
      for (int i = 0; i < 4; i++) o4[i] = w[i] ^ bk->ks1024[4 * j + i];
      *reinterpret_cast<uint4*>(pout + off) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      const uint32_t* cw = SEAL ? o4 : w;
      padd_full(tl, cw[0], cw[1], cw[2], cw[3]);
      tl = pmul(tl, rr);
    }
#pragma unroll
    for (int i = 0; i < 5; i++) hs.v[i] += tl.v[i];
  }
  pnorm(hs);
  h = hs;
  return true;
}

// FUSED: keys is the workgroup's own key schedule (LDS, built by keygen_wave), blk = workgroup.
template <bool SEAL, int NSPLIT, bool FUSED = false>
__device__ __forceinline__ void crypt_wave(const BlockKey* __restrict__ keys, uint64_t nblocks,
                                           const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           uint8_t* __restrict__ ok, uint32_t* lds) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63u;
  // wave-uniform block index
  // blocks in workgroup order: a contiguous-range-per-XCD remap measured no gain
  const uint32_t wg = blockIdx.x;
  const uint64_t blk = FUSED ? (uint64_t)blockIdx.x
                     : NSPLIT == 1 ? (uint64_t)wg * 4u + (uint64_t)__builtin_amdgcn_readfirstlane(wave) : (uint64_t)wg;
  if (blk >= nblocks) return;
  const BlockKey* bk = FUSED ? keys : keys + blk;
  if (bk->flags) {  // rejected descriptor: write nothing
    if (!SEAL && l == 0 && (NSPLIT == 1 || wave == 0u)) ok[blk] = 0;
    return;
  }
  const uint32_t n = bk->len;
  if (NSPLIT > 1 && n != XS_BLOCK_DATA && wave != 0u) return;  // a partial block: wave 0 alone
  const uint8_t* in = src + bk->src;
  uint8_t* out = dst + bk->dst;
  const uint8_t* pin = SEAL ? in : in + XS_BLOCK_HDR;
  uint8_t* pout = SEAL ? out + XS_BLOCK_HDR : out;
  uint32_t* wb = lds + wave * WAVE_LDS_WORDS;

  P5 h;
  h.v[0] = h.v[1] = h.v[2] = h.v[3] = h.v[4] = 0;
  if (n == XS_BLOCK_DATA) {
    if (!crypt_block_mfma<SEAL, NSPLIT>(bk, pin, pout, wb, wb + STAGE_WORDS, h, wave, lds)) return;
  } else {
    crypt_block<SEAL>(bk, pin, pout, n, wb, h);
  }

  // sum the 64 partials with wave shuffles (limbs < 2^26+2^6 -> < 2^32 after 5 levels)
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int i = 0; i < 5; i++) h.v[i] += (uint32_t)__shfl_xor((int)h.v[i], off, 64);
    if (off == 2) pnorm(h);
  }
  uint32_t verdict = 1;
  if (l == 0) {
    P5 hc = pcanon(h);
    uint32_t s4[4] = {bk->s[0], bk->s[1], bk->s[2], bk->s[3]};
    uint32_t tag[4];
    ptag(hc, s4, tag);
    if (SEAL) {
      *reinterpret_cast<uint4*>(out) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    } else {
      const uint4 want = *reinterpret_cast<const uint4*>(in);
      const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) | (want.w ^ tag[3]);
      verdict = diff == 0 ? 1u : 0u;
      ok[blk] = diff == 0 ? 1 : 0;
    }
  }
  if (!SEAL) {
    verdict = (uint32_t)__shfl((int)verdict, 0, 64);
    if (verdict == 0) {
      // authentication failed: zero the block's plaintext, after our own stores completed
      __builtin_amdgcn_s_waitcnt(0);
      for (uint32_t off = 16u * l; off < n; off += 16u * LANES) {
        const uint32_t L = (n - off) < 16u ? (n - off) : 16u;
        if (L == 16u) *reinterpret_cast<uint4*>(pout + off) = make_uint4(0, 0, 0, 0);
        else for (uint32_t i = 0; i < L; i++) pout[off + i] = 0;
      }
    }
  }
}


__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(XS_SEAL_WPE)))
xs_seal(const BlockKey* __restrict__ keys, uint64_t nblocks, const uint8_t* __restrict__ src,
        uint8_t* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_WORDS];
  crypt_wave<true, 1>(keys, nblocks, src, dst, nullptr, lds);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(XS_OPEN_WPE)))
xs_open(const BlockKey* __restrict__ keys, uint64_t nblocks, const uint8_t* __restrict__ src,
        uint8_t* __restrict__ dst, uint8_t* __restrict__ ok) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_WORDS];
  crypt_wave<false, 1>(keys, nblocks, src, dst, ok, lds);
}

// Completion word of a fused batch (every wave of every workgroup reaches it).  Each wave waits for
// its own stores to complete (vmcnt: they have reached the L2 or the fabric), then after the
// barrier thread 0 alone fences the workgroup's outputs at system scope: one L2 write-back per
// workgroup instead of one per wave (nine of them cost ~2.8 us of a ranged read).
// A one-block batch has no other workgroup to count: the system-scope release of the word is that
// fence.  Otherwise thread 0 fences before the acq_rel counter, and the last workgroup to arrive
// signals, ordered after every other workgroup's fenced outputs.
__device__ __forceinline__ void xs_fused_complete(uint32_t* ctr, uint32_t* flag, uint32_t seq, uint64_t nblocks) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (nblocks != 1u) __threadfence_system();
    const bool last = nblocks == 1u ||
                      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nblocks - 1u;
    if (last) {
      if (nblocks != 1u) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Tiny descriptor batches (ranged reads, a few coalesced handles), latency-first: one workgroup
// per block, keygen and crypt in one launch.  Descriptors of batches of <= 16 blocks arrive in the kernel arguments.
// For a full block the crypt waves start at once on the data: each stages its 4 KiB groups with
// LDS-DMA (one PCIe round trip for all of them), derives the HSalsa20 subkey (or takes it from the
// wave on its SIMD that did) and runs its keystream blocks, writing the output and keeping the
// ciphertext in LDS.  The key wave meanwhile builds the block's key schedule (keygen_wave_body,
// taking wave 0's subkey) at raised issue priority; as soon as the power tables the Toeplitz
// digit table needs exist it builds that table and raises the Z flag, then finishes C, D and the
// correction term.  Each crypt wave runs the matrix-core Poly1305 over its own LDS-resident
// ciphertext once the Z flag is up; after one barrier (B2) their accumulators are summed through
// LDS and wave 0 finalises as crypt_block_mfma does (the two tail chunks' terms were computed
// while it waited).  The key schedule thus leaves the critical path.  Cross-wave hand-offs are
// LDS flags raised after lgkmcnt(0) and polled with inline ds_reads, never release / acquire
// (those would wait for the waves' outstanding PCIe loads).  Partial blocks (and rejected
// descriptors) take the plain order: key schedule, then wave 0's VALU path.
// NCW = 8 crypt waves, two per SIMD so that each SIMD interleaves two dependency chains, plus the
// key-schedule wave NCW.  Crypt wave w runs on SIMD w % 4; SIMD 0 also runs the key-schedule wave
// (the longer chain), so its crypt waves take fewer 4 KiB groups.  Group counts per wave, 4 bits
// each (wave 0 first), and first groups, 8 bits:
//   {1, 3, 3, 3, 0, 2, 2, 2}  -> SIMD loads 1, 5, 5, 5 (wave 4 idles until phase 2)
// Waves 4..7 take the HSalsa20 subkey from wave w - 4 (same SIMD) through LDS instead of computing
// it again: a SIMD's second wave only gets the issue slots its first leaves.  (One crypt wave per
// SIMD, and an even two groups per wave, measured slower: DESIGN.md section 3e.)
template <int NCW>
__device__ __forceinline__ uint32_t f2_count(uint32_t w) {
  static_assert(NCW == 8, "the group split below is for eight crypt waves");
  return (0x22203331u >> (4u * w)) & 15u;
}
template <int NCW>
__device__ __forceinline__ uint32_t f2_first(uint32_t w) {
  return (uint32_t)(0x0E0C0A0A07040100ull >> (8u * w)) & 255u;
}
template <int NCW>
constexpr int f2_max_groups() { return 3; }
// LDS words: stage (16 groups of 4 KiB, indexed by group), relay (4 KiB per crypt wave), the
// accumulators of crypt waves 1..NCW-1 (8 KiB each), the Toeplitz digit rows (3 KiB)
template <int NCW>
constexpr int f2_lds_words() { return 16 * 1024 + NCW * 1024 + (NCW - 1) * 2048 + 64 * 12; }

// Sum of a P5 over the 64 lanes of a wave, left in every lane, without LDS round trips: quad DPP
// (lanes l ^ 1, l ^ 2), row half-mirror and mirror (the other quad of 8 lanes, the other 8 of a
// 16-lane row: the partial sums are uniform within those groups by then), v_permlane16_swap (the
// other row of a 32-lane half) and v_permlane32_swap (the other half).  Limbs come in pnorm-bounded
// (< 2^26 + 2^6); one pnorm after 32 lanes keeps every limb below 2^32.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ void wave_sum5(P5& h) {
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint32_t v = h.v[i];
    v += dpp_u32<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_u32<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_u32<0x141>(v);  // row_half_mirror
    v += dpp_u32<0x140>(v);  // row_mirror
    const auto s16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    h.v[i] = s16[0] + s16[1];
  }
  pnorm(h);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const auto s32 = __builtin_amdgcn_permlane32_swap(h.v[i], h.v[i], false, false);
    h.v[i] = s32[0] + s32[1];
  }
}

// The key wave of a ranged read's open (a group window: the VALU tag below).  Keystream words
// 0..7 of blocks 0 (lanes < 32: r, s) and 1024 (lanes >= 32: the last two chunks) -- from the
// host's key setup, or made here from wave 0's subkey -- go into *kl and raise r_flag.  Then the
// weight table the crypt waves' Horner sums need, one entry per lane: lane i < 32 holds
// r^(126 - 4i), lane 32 + j holds r^(128 j), from one square-and-multiply pass over r^(2^s),
// s = 0..11 (lanes < 32 take bits 1..6, lanes >= 32 bits 7..11), into tab, then tab_flag.
__device__ __forceinline__ void fused_key_wave_vtag(const uint32_t n[6], BlockKey* kl, const uint32_t* sk_lds,
                                                    const uint32_t* sk_flag, uint32_t* r_flag, uint32_t (*tab)[5],
                                                    uint32_t* tab_flag, bool use_kp, const XsKeyPre& kp) {
  const uint32_t l = threadIdx.x & 63u;
  uint32_t ks[16];
  if (use_kp) {  // wave-uniform (scalar) loads, selected per lane afterwards (see keygen_wave_body)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t a = __builtin_amdgcn_readfirstlane(kp.k0[i]), b = __builtin_amdgcn_readfirstlane(kp.k1024[i]);
      ks[i] = as_varying(l < 32 ? a : b);
    }
  } else {
    uint32_t sk[8];
    lds_wait_subkey(sk_flag, sk_lds, sk);
    salsa20_block_lazy(sk, n[4], n[5], l < 32 ? 0u : 1024u, ks);
  }
  if (l == 32) {
#pragma unroll
    for (int i = 0; i < 8; i++) kl->ks1024[i] = ks[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) ks[i] = __shfl(ks[i], 0);  // block 0 words 0..7 (r, s) everywhere
  P5 r;
  r.v[0] = ks[0] & 0x3ffffffu;
  r.v[1] = alignbit(ks[1], ks[0], 26) & 0x3ffff03u;
  r.v[2] = alignbit(ks[2], ks[1], 20) & 0x3ffc0ffu;
  r.v[3] = alignbit(ks[3], ks[2], 14) & 0x3f03fffu;
  r.v[4] = (ks[3] >> 8) & 0x00fffffu;
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 4; i++) kl->s[i] = ks[4 + i];
#pragma unroll
    for (int i = 0; i < 5; i++) kl->r[i] = r.v[i];
  }
  lds_raise_flag(r_flag);
  // exponent of this lane's entry: 126 - 4i = 2 + 4 (31 - i) (bit 1 set, bit 0 clear), or 128 j
  const uint32_t e = l < 32u ? 126u - 4u * l : (l - 32u) << 7;
  P5 sq = r, acc;
  acc.v[0] = 1; acc.v[1] = acc.v[2] = acc.v[3] = acc.v[4] = 0;
#pragma unroll
  for (int s = 0; s < 12; s++) {
    const bool take = (e >> s) & 1u;
    if (s == 1 || s == 7) {  // a lane's first factor (its entry is still 1 there): no multiply
      if (take) acc = sq;
    } else if (s > 1) {
      const P5 q = pmul(acc, sq);
      if (take) acc = q;
    }
    if (s < 11) sq = pmul(sq, sq);
  }
  put5(tab[l], acc);
  lds_raise_flag(tab_flag);
}

template <bool SEAL, int NCW>
__global__ void __launch_bounds__(64 * (NCW + 1)) xs_crypt_fused2(KeyArg key, NonceArg bounds, const xs_block_desc* __restrict__ desc,
                                                                    const XsInlineDescs inl,
                                                       uint64_t nblocks, const uint8_t* __restrict__ src,
                                                       uint8_t* __restrict__ dst, uint8_t* __restrict__ ok,
                                                       uint32_t* __restrict__ ctr, uint32_t* __restrict__ flag,
                                                       uint32_t seq) {
  constexpr int MODE = SEAL ? 2 : 3;
  static_assert(f2_lds_words<NCW>() >= LDS_WORDS, "the fallback path runs crypt_wave in this LDS");
  __shared__ __attribute__((aligned(16))) uint32_t lds[f2_lds_words<NCW>()];
  __shared__ BlockKey kl;
  // hs_flag[0..3]: subkeys of waves 0..3 published (for waves 4..7 / the key wave); [4]: Z table ready
  // (a windowed open: r, s and ks1024 in kl); [5]: C and D power tables in kl, wave 0's finalisation
  // factor (a windowed open: the weight table in vtab).  vpart: each crypt wave's VALU tag sum.
  __shared__ uint32_t hs_key[4][8], hs_flag[6];
  __shared__ uint32_t vtab[64][5], vpart[NCW][5];
  if (blockIdx.x >= nblocks) return;  // uniform per workgroup (grid == nblocks)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63u;
  const uint64_t blk = blockIdx.x;
  if (threadIdx.x < 6u) hs_flag[threadIdx.x] = 0u;
  uint32_t nn[6];
  uint64_t soff, doff;
  uint32_t len;
  // descriptors of small batches come in the kernel arguments (no PCIe read of the pinned array)
  const bool valid = blk < inl.n ? desc_params<MODE>(inl.d[blk], bounds, nn, soff, doff, len)
                                : block_params<MODE>(bounds, 0, 0, desc, blk, nn, soff, doff, len);
  // The descriptor is uniform: move it into SGPRs now.  vmcnt drains in order, so a later use of
  // a descriptor word still in a VGPR would make the compiler wait for every data load of the
  // block issued after it.
#pragma unroll
  for (int i = 0; i < 6; i++) nn[i] = __builtin_amdgcn_readfirstlane(nn[i]);
  // (readfirstlane returns int: both halves go through uint32_t, or an offset with bit 31 set
  // in its low word would sign-extend over the high word)
  soff = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(soff >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)soff);
  doff = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(doff >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)doff);
  len = __builtin_amdgcn_readfirstlane(len);
  // OPEN of a ranged read: decrypt only the 4 KiB groups the caller reads (XS_DESC_WINDOW)
  uint32_t gwin = 0xFFFFu;
  if (!SEAL) {
    const uint32_t rsv = blk < inl.n ? inl.d[blk].reserved : desc[blk].reserved;
    if (rsv & XS_DESC_WINDOW) gwin = rsv & 0xFFFFu;
  }
  gwin = __builtin_amdgcn_readfirstlane(gwin);
  // the smallest batches bring each block's key setup from the host (XsKeyPre): no HSalsa20 in the
  // crypt waves, no Salsa20 core in front of the key wave's power tables
  const bool host_key = blk < inl.npre;
  // A ranged read's open (a group window) computes its tag on the VALU: with only a group or two to
  // decrypt, the crypt waves are idle once r exists, and a short key chain (11 squarings) replaces
  // the power tables, the Toeplitz table and the correction term of the matrix-core tag, which stays
  // the path of whole blocks (there the keystream keeps the VALU busy).  DESIGN.md section 3e.
  const bool vtag = !SEAL && gwin != 0xFFFFu;
  __syncthreads();  // hs_flag cleared before any wave can poll or raise it
  if (!valid || len != XS_BLOCK_DATA) {
    // rejected descriptor or partial block: the fused-v1 order (the other waves idle)
    if (wave == 0) {
      if (valid) {
        keygen_wave_body<MODE>(key, nn, soff, doff, len, &kl, nullptr, nullptr);
      } else if (l == 0u) {
        kl.flags = 1;
        kl.len = 0;
      }
    }
    __syncthreads();
    if (wave < 4) crypt_wave<SEAL, 4, true>(&kl, nblocks, src, dst, ok, lds);
  } else {
    uint32_t* const stage = lds;                      // [16][1024]: group u at 1024 u
    uint32_t* const relay = lds + 16 * 1024;          // [NCW][1024]: OPEN output relayout; wave 0's transpose
    uint32_t* const xacc = relay + NCW * 1024;        // [NCW - 1][2048]: accumulators of waves 1..NCW-1
    uint32_t* const zt = xacc + (NCW - 1) * 2048;     // [64][12]: Toeplitz digit rows
    const uint8_t* in = src + soff;
    uint8_t* out = dst + doff;
    const uint8_t* pin = SEAL ? in : in + XS_BLOCK_HDR;
    uint8_t* pout = SEAL ? out + XS_BLOCK_HDR : out;
    const uint8_t* pin_m32 = pin - 32;
    uint8_t* pout_m32 = pout - 32;
    const uint32_t lane_off = 16u * (4u * (l & 15u) + (l >> 4));
    const bool not_key = (l & 47u) != 0u;
    const uint32_t n = l & 15u, kg = l >> 4;
    uint4 tail[2];  // wave 0 lane 63: chunks 4094, 4095 (fetched early, used in the finalisation)
    if (wave < NCW) {
      // ---- phase 1: stage all this wave's groups, keystream + XOR + output, ciphertext kept in LDS
      if (wave == 0 && l == 0u) {  // key slots (chunks -2, -1): never loaded or stored
        *reinterpret_cast<uint4*>(stage) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(stage + 64) = make_uint4(0u, 0u, 0u, 0u);
      }
      const uint32_t g0 = f2_first<NCW>(wave), gn = f2_count<NCW>(wave);
#pragma unroll
      for (uint32_t g = 0; g < (uint32_t)f2_max_groups<NCW>(); g++) {
        if (g >= gn) break;
        const uint32_t u = g0 + g;
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (j > 0 || u > 0 || not_key)
            __builtin_amdgcn_global_load_lds(pin_m32 + 4096u * u + lane_off + 1024 * j,
                                             (lds_void*)(stage + 1024 * u + 256 * j), 16, 0, 0);
      }
      if (wave == 0) {  // every lane loads the same two chunks (lane 63 uses them); a lane-varying
                        // zero keeps them VGPR loads that nothing waits for before the finalisation
        const uint8_t* tp = pin + 16u * 4094u + as_varying(0u);
        tail[0] = *reinterpret_cast<const uint4*>(tp);
        tail[1] = *reinterpret_cast<const uint4*>(tp + 16);
      }
      uint32_t sk[8];
      if (host_key) {
#pragma unroll
        for (int i = 0; i < 8; i++) sk[i] = inl.pre[blk].sk[i];
      } else if (NCW == 8 && wave >= 4u) {  // the subkey of wave - 4, which shares this SIMD
        if (gn != 0u) lds_wait_subkey(&hs_flag[wave - 4u], hs_key[wave - 4u], sk);
      } else {
        uint32_t x[16] = {SIG0, key.k[0], key.k[1], key.k[2], key.k[3], SIG1, nn[0], nn[1],
                          nn[2], nn[3],     SIG2,     key.k[4], key.k[5], key.k[6], key.k[7], SIG3};
#pragma unroll
        for (int i = 0; i < 16; i++) x[i] = as_varying(x[i]);  // on the VALU: see as_varying
        salsa_rounds_lazy(x);  // HSalsa20 (the crypt waves derive the subkey themselves: no wait on the key wave)
        sk[0] = x[0]; sk[1] = x[5]; sk[2] = x[10]; sk[3] = x[15];
        sk[4] = x[6]; sk[5] = x[7]; sk[6] = x[8]; sk[7] = x[9];
        if (l == 0u) {
#pragma unroll
          for (int i = 0; i < 8; i++) hs_key[wave][i] = sk[i];
        }
        lds_raise_flag(&hs_flag[wave]);
      }
      const SalsaPre pre = salsa_pre(sk, nn[4], nn[5]);
      uint32_t* const rl = relay + 1024 * wave;
#pragma unroll 1
      for (uint32_t g = 0; g < gn; g++) {
        const uint32_t u = g0 + g;
        if (!((gwin >> u) & 1u)) continue;  // outside the window: staged for the tag only
        uint32_t ks[16];
        salsa20_block_pre(pre, 64u * u + l, ks);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t* sb = stage + 1024 * u;
        uint4* mine = reinterpret_cast<uint4*>(sb + 256 * (l >> 4) + 4 * (l & 15u));
        uint32_t o[16];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint4 v = mine[16 * j];
          o[4 * j] = v.x ^ ks[4 * j];
          o[4 * j + 1] = v.y ^ ks[4 * j + 1];
          o[4 * j + 2] = v.z ^ ks[4 * j + 2];
          o[4 * j + 3] = v.w ^ ks[4 * j + 3];
        }
        // SEAL: the ciphertext replaces the plaintext in the stage; OPEN: the stage keeps the
        // ciphertext and the plaintext is laid out through the relay slot
        uint32_t* lay = SEAL ? sb : rl;
        uint4* lmine = reinterpret_cast<uint4*>(lay + 256 * (l >> 4) + 4 * (l & 15u));
#pragma unroll
        for (int j = 0; j < 4; j++) lmine[16 * j] = make_uint4(o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]);
        asm volatile("" ::: "memory");  // LDS ops of one wave execute in order
        uint4 w[4];
#pragma unroll
        for (int j = 0; j < 4; j++) w[j] = *reinterpret_cast<const uint4*>(lay + 256 * j + 4 * l);
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (j > 0 || u > 0 || not_key)
            *reinterpret_cast<uint4*>(pout_m32 + 4096u * u + lane_off + 1024 * j) = w[j];
      }
      if (!SEAL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // plaintext out before any zero-fill
    } else {
      // ---- the key wave: key schedule into LDS; as soon as the A and B power tables exist, the
      // shared Toeplitz digit table and the Z-ready flag (the crypt waves' MFMA phase needs no
      // more), then C, D and the correction term, which only the finalisation reads (after B2).
      // It shares a SIMD with wave 0 and is the longer chain: it issues first.
      __builtin_amdgcn_s_setprio(3);
      if (vtag) {
        fused_key_wave_vtag(nn, &kl, hs_key[0], &hs_flag[0], &hs_flag[4], vtab, &hs_flag[5], host_key,
                            inl.pre[host_key ? blk : 0]);
      } else {
      auto z_table = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        P5 qa, qb;
        const uint32_t k = 63u - l;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          qa.v[i] = kl.full.A[k & 7u][i];
          qb.v[i] = kl.full.B[k >> 3][i];
        }
        const P32 wq = to32(pmul(qa, qb));
        uint32_t w0 = wq.w0, w1 = wq.w1, w2 = wq.w2, w3 = wq.w3, w4 = wq.w4;
        unsigned cy;
        w0 = __builtin_addc(w0, 0x80808080u, 0u, &cy);
        w1 = __builtin_addc(w1, 0x80808080u, cy, &cy);
        w2 = __builtin_addc(w2, 0x80808080u, cy, &cy);
        w3 = __builtin_addc(w3, 0x80808080u, cy, &cy);
        w4 = (w4 + 0x80u + cy) ^ 0x80u;
        w0 ^= 0x80808080u;
        w1 ^= 0x80808080u;
        w2 ^= 0x80808080u;
        w3 ^= 0x80808080u;
        uint4* row = reinterpret_cast<uint4*>(zt + 12u * l);
        row[0] = make_uint4(0u, 0u, 0u, w4 << 24);
        row[1] = make_uint4(__builtin_bswap32(w3), __builtin_bswap32(w2), __builtin_bswap32(w1), __builtin_bswap32(w0));
        row[2] = make_uint4(0u, 0u, 0u, 0u);
        lds_raise_flag(&hs_flag[4]);
      };
      // the descriptor fields this kernel already holds (no second read over PCIe); wave 0's subkey,
      // or the whole key setup from the host
      keygen_wave_body<MODE>(key, nn, soff, doff, len, &kl, hs_key[0], &hs_flag[0], z_table, &hs_flag[5], host_key,
                             inl.pre[host_key ? blk : 0]);
      }
    }
    xs_v4i acc[4][2];
    P5 tl;  // wave 0, lane 63: the Poly1305 terms of chunks 4094, 4095
#pragma unroll
    for (int i = 0; i < 5; i++) tl.v[i] = 0;
    if (wave < NCW) {
      lds_wait_flag(&hs_flag[4]);  // the Z table (each wave reads only its own staged groups); vtag: r
      if (wave == 0 && l == 63u) {
        // chunks 4094, 4095 (keystream block 1024 words 0..7): exponents 2 and 1.  r and ks1024
        // are in kl before the Z flag rises, so this leaves the finalisation's critical path.
        P5 rr;
#pragma unroll
        for (int i = 0; i < 5; i++) rr.v[i] = kl.r[i];
#pragma unroll
        for (int j = 0; j < 2; j++) {
          const uint32_t w[4] = {tail[j].x, tail[j].y, tail[j].z, tail[j].w};
          uint32_t o4[4];
#pragma unroll
          for (int i = 0; i < 4; i++) o4[i] = w[i] ^ kl.ks1024[4 * j + i];
          *reinterpret_cast<uint4*>(pout + 16u * (4094u + j)) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
          const uint32_t* cw = SEAL ? o4 : w;
          padd_full(tl, cw[0], cw[1], cw[2], cw[3]);
          tl = pmul(tl, rr);
        }
      }
      if (vtag) {
        // ---- phase 2, windowed open: Poly1305 of the LDS-resident ciphertext on the VALU.  Lane l
        // takes, in each of the wave's 4 KiB groups u, the four consecutive chunks at stage slots
        // 256u + 4l + j (slot = chunk index + 2: slots 0 and 1 are the key slots and hash nothing),
        // Horner with r: h_u = sum_j c r^(4 - j).  The wave's groups are consecutive (u0..u1), so
        // H = sum_u h_u r^(256 (u1 - u)) (Horner with r^256), and H r^(254 - 4l) r^(256 (15 - u1))
        // gives slot 256u + 4l + j the power r^(4098 - slot), i.e. chunk k its r^(4096 - k).  That
        // weight is two entries of the key wave's table: r^(126 - 4 (l & 31)) and r^(128 jx),
        // jx = 2 (15 - u1) + [l < 32].  The wave sums its lanes; wave 0 adds the waves after B2.
        P5 part;
#pragma unroll
        for (int i = 0; i < 5; i++) part.v[i] = 0;
        const uint32_t g0 = f2_first<NCW>(wave), gn = f2_count<NCW>(wave);
        if (gn != 0u) {
          P5 rr;
#pragma unroll
          for (int i = 0; i < 5; i++) rr.v[i] = kl.r[i];
          const PMul R = pmul_prep(rr);
          P5 h[f2_max_groups<NCW>()];
#pragma unroll
          for (uint32_t g = 0; g < (uint32_t)f2_max_groups<NCW>(); g++) {
#pragma unroll
            for (int i = 0; i < 5; i++) h[g].v[i] = 0;
            if (g >= gn) continue;
            const uint32_t u = g0 + g;
            const uint4* mine = reinterpret_cast<const uint4*>(stage + 1024 * u + 256 * (l >> 4) + 4 * (l & 15u));
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const uint4 v = mine[16 * j];
              if (j >= 2 || u > 0u || l > 0u) padd_full(h[g], v.x, v.y, v.z, v.w);
              h[g] = pmul_u(h[g], R);
            }
          }
          lds_wait_flag(&hs_flag[5]);  // the weight table
          const uint32_t u1 = g0 + gn - 1u;
          const uint32_t jx = 2u * (15u - u1) + (l < 32u ? 1u : 0u);
          P5 t1, t2, r256;
#pragma unroll
          for (int i = 0; i < 5; i++) {
            t1.v[i] = vtab[l & 31u][i];
            t2.v[i] = vtab[32u + jx][i];
            r256.v[i] = vtab[34][i];  // r^(128 * 2)
          }
          const P5 tw = pmul(t1, t2);
          P5 H = h[0];
#pragma unroll
          for (uint32_t g = 1; g < (uint32_t)f2_max_groups<NCW>(); g++) {
            if (g >= gn) break;
            H = pmul(H, r256);
            add5(H, h[g]);
            pnorm(H);
          }
          part = pmul(H, tw);
        }
        add5(part, tl);  // zero except in wave 0, lane 63
        pnorm(part);
        wave_sum5(part);
        if (l == 0u) put5(vpart[wave], part);
      } else {
      // ---- phase 2: matrix-core Poly1305 over the LDS-resident ciphertext
      const uint32_t zlo = (15u - n) >> 2, zsh = (31u - n) & 3u;
      uint32_t zaddr = (uint32_t)(uintptr_t)((const lds_u32*)zt + 12u * kg + zlo);
      asm volatile("" : "+v"(zaddr));
      const lds_u32* zl = (const lds_u32*)(uintptr_t)zaddr;
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
          for (int i = 0; i < 4; i++) acc[j][mt][i] = wave == 0 ? 1 << 24 : 0;  // the bias once per block
      const uint32_t g0 = f2_first<NCW>(wave), gn = f2_count<NCW>(wave);
#pragma unroll 1
      for (uint32_t g = 0; g < gn; g++) {
        const uint32_t u = g0 + g;
        const uint4* mine = reinterpret_cast<const uint4*>(stage + 1024 * u + 256 * (l >> 4) + 4 * (l & 15u));
        uint32_t cw[16];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint4 v = mine[16 * j];
          cw[4 * j] = v.x; cw[4 * j + 1] = v.y; cw[4 * j + 2] = v.z; cw[4 * j + 3] = v.w;
        }
        const lds_u32* zr = zl + 48u * u;
        uint32_t z[9];
#pragma unroll
        for (int i = 0; i < 9; i++) z[i] = zr[i];
        xs_v4i A[2];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          A[1][i] = (int)__builtin_amdgcn_alignbyte(z[i + 1], z[i], zsh);
          A[0][i] = (int)__builtin_amdgcn_alignbyte(z[i + 5], z[i + 4], zsh);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
          xs_v4i B;
#pragma unroll
          for (int i = 0; i < 4; i++) B[i] = (int)(cw[4 * j + i] ^ 0x80808080u);
#pragma unroll
          for (int mt = 0; mt < 2; mt++) acc[j][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[mt], B, acc[j][mt], 0, 0, 0);
        }
      }
      if (wave > 0) {
        // lane-contiguous 16-byte groups: conflict-free ds_write_b128 / ds_read_b128
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
          for (int mt = 0; mt < 2; mt++)
            *reinterpret_cast<xs_v4i*>(xacc + (wave - 1u) * 2048u + (uint32_t)(2 * j + mt) * 256u + 4u * l) = acc[j][mt];
      }
      }
    }
    P5 rexp;  // wave 0: its lane's column exponent r^e, e = 66 - (4n + kg), formed before B2
    if (wave == 0 && !vtag) {
      lds_wait_flag(&hs_flag[5]);  // C and D are in kl
      const uint32_t e = 66u - (4u * n + kg);
      P5 t1, t2;
#pragma unroll
      for (int i = 0; i < 5; i++) {
        t1.v[i] = kl.full.C[e & 7u][i];
        t2.v[i] = kl.full.D[e >> 3][i];
      }
      rexp = pmul(t2, t1);
    }
    __syncthreads();  // B2: the other waves' accumulators are in LDS
    if (wave == 0) {
      const BlockKey* bk = &kl;
      P5 hs;
      if (vtag) {  // the waves' sums (each < 2^27 + 2^7)
#pragma unroll
        for (int i = 0; i < 5; i++) hs.v[i] = 0;
        if (l == 0u) {
#pragma unroll
          for (int w = 0; w < NCW; w++) {
#pragma unroll
            for (int i = 0; i < 5; i++) hs.v[i] += vpart[w][i];
          }
        }
      } else {
#pragma unroll
      for (int w = 0; w < NCW - 1; w++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
          for (int mt = 0; mt < 2; mt++)
            acc[j][mt] += *reinterpret_cast<const xs_v4i*>(xacc + (uint32_t)w * 2048u + (uint32_t)(2 * j + mt) * 256u + 4u * l);
      // transpose the partial words through wave 0's relay slot (as crypt_block_mfma)
      uint64_t* t64 = reinterpret_cast<uint64_t*>(relay);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint64_t sx[2];
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
          sx[mt] = (uint64_t)(uint32_t)acc[j][mt][0] + ((uint64_t)(uint32_t)acc[j][mt][1] << 8) +
                   ((uint64_t)(uint32_t)acc[j][mt][2] << 16) + ((uint64_t)(uint32_t)acc[j][mt][3] << 24);
        *reinterpret_cast<ulonglong2*>(t64 + (((n * 4u + j) * 4u + kg) * 2u)) = make_ulonglong2(sx[0], sx[1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint64_t xw[8];
      {
        const uint64_t* rd = t64 + (n * 4u + kg) * 8u;
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
          const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(rd + 2 * kk);
          xw[kk] = v.x;
          xw[4 + kk] = v.y;
        }
      }
      hs = pmul(column_value(xw), rexp);
      if (l == 0u) {
#pragma unroll
        for (int i = 0; i < 5; i++) hs.v[i] += bk->corr[i];
      }
      if (l == 63u) {  // chunks 4094, 4095, computed before B2
#pragma unroll
        for (int i = 0; i < 5; i++) hs.v[i] += tl.v[i];
      }
      pnorm(hs);
      wave_sum5(hs);
      }
      uint32_t verdict = 1;
      if (l == 0) {
        const P5 hc = pcanon(hs);
        const uint32_t s4[4] = {bk->s[0], bk->s[1], bk->s[2], bk->s[3]};
        uint32_t tag[4];
        ptag(hc, s4, tag);
        if (SEAL) {
          *reinterpret_cast<uint4*>(out) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
        } else {
          const uint4 want = *reinterpret_cast<const uint4*>(in);
          const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) | (want.w ^ tag[3]);
          verdict = diff == 0 ? 1u : 0u;
          ok[blk] = diff == 0 ? 1 : 0;
        }
      }
      if (!SEAL) {
        verdict = (uint32_t)__shfl((int)verdict, 0, 64);
        if (verdict == 0) {  // authentication failed: zero the block (every wave's stores are done, B2)
          __builtin_amdgcn_s_waitcnt(0);
          for (uint32_t off = 16u * l; off < XS_BLOCK_DATA; off += 16u * LANES)
            *reinterpret_cast<uint4*>(pout + off) = make_uint4(0, 0, 0, 0);
        }
      }
    }
  }
  if (ctr) xs_fused_complete(ctr, flag, seq, nblocks);
}

__global__ void __launch_bounds__(256) xs_seal_split(const BlockKey* __restrict__ keys, uint64_t nblocks,
                                                     const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_WORDS];
  crypt_wave<true, 4>(keys, nblocks, src, dst, nullptr, lds);
}

__global__ void __launch_bounds__(256) xs_open_split(const BlockKey* __restrict__ keys, uint64_t nblocks,
                                                     const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     uint8_t* __restrict__ ok) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_WORDS];
  crypt_wave<false, 4>(keys, nblocks, src, dst, ok, lds);
}

// SplitMix64 fill (synthetic benchmark objects generated in HBM).  Global word g of the stream
// is mix(seed + (g+1)*golden); local 64 KiB block b of the buffer holds global block
// first_block + b*stride (8192 words per block), so a rank's round-robin share of an object
// set gets the same bytes whatever the world size.  stride 1, first_block 0 = plain stream.
__global__ void xs_fill_splitmix(uint64_t* __restrict__ dst, uint64_t nwords, uint64_t seed, uint64_t first_block,
                                 uint64_t stride) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = (first_block + (k >> 13) * stride) * 8192u + (k & 8191u);
    uint64_t z = seed + (g + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[k] = z ^ (z >> 31);
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_keygen(int mode, const KeyArg& key, const NonceArg& nonce0, uint64_t first_block,
                         uint64_t total_len, uint64_t nblocks, const xs_block_desc* desc, BlockKey* out,
                         hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  static const uint64_t wide_max = [] {  // env XS_KEYGEN_WIDE_MAX overrides (A/B, 0 = never)
    const char* v = getenv("XS_KEYGEN_WIDE_MAX");
    return v ? strtoull(v, nullptr, 10) : (uint64_t)XS_KEYGEN_WIDE_MAX;
  }();
  if (nblocks <= wide_max) {  // few blocks: one wave per block (latency)
    const dim3 g((unsigned)nblocks);
    switch (mode) {
      case 0: hipLaunchKernelGGL(xs_keygen_wide<0>, g, dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
      case 1: hipLaunchKernelGGL(xs_keygen_wide<1>, g, dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
      case 2: hipLaunchKernelGGL(xs_keygen_wide<2>, g, dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
      default: hipLaunchKernelGGL(xs_keygen_wide<3>, g, dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
    }
    return hipGetLastError();
  }
  const uint64_t grid = (nblocks + 63) / 64;
  switch (mode) {
    case 0: hipLaunchKernelGGL(xs_keygen<0>, dim3((unsigned)grid), dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
    case 1: hipLaunchKernelGGL(xs_keygen<1>, dim3((unsigned)grid), dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
    case 2: hipLaunchKernelGGL(xs_keygen<2>, dim3((unsigned)grid), dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
    default: hipLaunchKernelGGL(xs_keygen<3>, dim3((unsigned)grid), dim3(64), 0, stream, key, nonce0, first_block, total_len, nblocks, desc, out); break;
  }
  return hipGetLastError();
}

hipError_t launch_crypt(bool seal, const BlockKey* keys, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                        uint8_t* ok, hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  static const uint64_t split_max = [] {  // env XS_SPLIT_MAX overrides (A/B, 0 = never)
    const char* v = getenv("XS_SPLIT_MAX");
    return v ? strtoull(v, nullptr, 10) : (uint64_t)XS_SPLIT_MAX;
  }();
  if (nblocks <= split_max) {  // few blocks: four waves per block (shorter launch)
    if (seal) hipLaunchKernelGGL(xs_seal_split, dim3((unsigned)nblocks), dim3(256), 0, stream, keys, nblocks, src, dst);
    else hipLaunchKernelGGL(xs_open_split, dim3((unsigned)nblocks), dim3(256), 0, stream, keys, nblocks, src, dst, ok);
    return hipGetLastError();
  }
  const unsigned grid = (unsigned)((nblocks + 3) / 4);  // four blocks (waves) per workgroup
  if (seal) hipLaunchKernelGGL(xs_seal, dim3(grid), dim3(256), 0, stream, keys, nblocks, src, dst);
  else hipLaunchKernelGGL(xs_open, dim3(grid), dim3(256), 0, stream, keys, nblocks, src, dst, ok);
  return hipGetLastError();
}

// ---- host key setup for the smallest fused batches (XsKeyPre): the same Salsa20 core as the
// kernels' (salsa20_block / HSalsa20 of keygen), on one host core
static inline uint32_t hrotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static void host_salsa_rounds(uint32_t (&x)[16]) {
  for (int i = 0; i < 10; i++) {
#define XS_HQR(a, b, c, d)        \
  x[b] ^= hrotl(x[a] + x[d], 7);  \
  x[c] ^= hrotl(x[b] + x[a], 9);  \
  x[d] ^= hrotl(x[c] + x[b], 13); \
  x[a] ^= hrotl(x[d] + x[c], 18);
    XS_HQR(0, 4, 8, 12) XS_HQR(5, 9, 13, 1) XS_HQR(10, 14, 2, 6) XS_HQR(15, 3, 7, 11)
    XS_HQR(0, 1, 2, 3) XS_HQR(5, 6, 7, 4) XS_HQR(10, 11, 8, 9) XS_HQR(15, 12, 13, 14)
#undef XS_HQR
  }
}
static void host_key_pre(const KeyArg& key, const uint8_t nonce[24], XsKeyPre& p) {
  uint32_t n[6];
  memcpy(n, nonce, 24);  // little-endian words, as the kernels' nonce words
  uint32_t x[16] = {SIG0, key.k[0], key.k[1], key.k[2], key.k[3], SIG1, n[0], n[1],
                    n[2], n[3],     SIG2,     key.k[4], key.k[5], key.k[6], key.k[7], SIG3};
  host_salsa_rounds(x);  // HSalsa20: no feed-forward; words 0, 5, 10, 15, 6..9
  const uint32_t sk[8] = {x[0], x[5], x[10], x[15], x[6], x[7], x[8], x[9]};
  memcpy(p.sk, sk, sizeof sk);
  for (int b = 0; b < 2; b++) {
    const uint32_t ctr = b ? 1024u : 0u;
    const uint32_t in[16] = {SIG0, sk[0], sk[1], sk[2], sk[3], SIG1, n[4], n[5], ctr, 0u, SIG2, sk[4], sk[5], sk[6], sk[7], SIG3};
    uint32_t y[16];
    memcpy(y, in, sizeof y);
    host_salsa_rounds(y);
    for (int i = 0; i < 8; i++) (b ? p.k1024 : p.k0)[i] = y[i] + in[i];
  }
}

hipError_t launch_crypt_fused(bool seal, const KeyArg& key, const NonceArg& bounds, const xs_block_desc* desc,
                              const xs_block_desc* host_desc, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                              uint8_t* ok, uint32_t* ctr, uint32_t* flag, uint32_t seq, hipStream_t stream) {
  if (nblocks == 0) return hipSuccess;
  static const uint64_t pre_max = [] {  // env XS_KEY_PRE_MAX overrides (A/B, 0 = never)
    const char* v = getenv("XS_KEY_PRE_MAX");
    return std::min<uint64_t>(v ? strtoull(v, nullptr, 10) : (uint64_t)XS_KEY_PRE, (uint64_t)XS_KEY_PRE);
  }();
  XsInlineDescs inl{};
  if (host_desc && nblocks <= (uint64_t)XS_INLINE_DESCS) {
    for (uint64_t i = 0; i < nblocks; i++) inl.d[i] = host_desc[i];
    inl.n = (uint32_t)nblocks;
    // every block or none: the launch lasts as long as its slowest workgroup
    if (nblocks <= pre_max) {
      for (uint64_t i = 0; i < nblocks; i++) host_key_pre(key, host_desc[i].nonce, inl.pre[i]);
      inl.npre = (uint32_t)nblocks;
    }
  }
  // eight crypt waves (two per SIMD) + the key-schedule wave
  if (seal) hipLaunchKernelGGL((xs_crypt_fused2<true, 8>), dim3((unsigned)nblocks), dim3(576), 0, stream, key, bounds, desc, inl, nblocks, src, dst, ok, ctr, flag, seq);
  else hipLaunchKernelGGL((xs_crypt_fused2<false, 8>), dim3((unsigned)nblocks), dim3(576), 0, stream, key, bounds, desc, inl, nblocks, src, dst, ok, ctr, flag, seq);
  return hipGetLastError();
}

uint64_t fused_max_blocks() {
  static const uint64_t m = [] {  // env XS_FUSED_MAX overrides (A/B, 0 = never)
    const char* v = getenv("XS_FUSED_MAX");
    return v ? strtoull(v, nullptr, 10) : (uint64_t)XS_FUSED_MAX;
  }();
  return m;
}

hipError_t launch_fill(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t first_block, uint64_t stride,
                       hipStream_t stream) {
  if (nwords == 0) return hipSuccess;
  uint64_t grid = (nwords + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(xs_fill_splitmix, dim3((unsigned)grid), dim3(256), 0, stream, dst, nwords, seed, first_block,
                     stride);
  return hipGetLastError();
}

}  // namespace xs
