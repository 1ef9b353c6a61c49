// xs_eme.hip -- batched EME-AES-256 name cipher for gfx950: the file-name half of rclone's
// crypt overlay, encryptSegment / decryptSegment (backend/crypt/cipher.go:264-312), which
// calls eme.Transform(aes(nameKey), nameTweak, pkcs7(name), direction) of
// github.com/rfjakob/eme v1.2.0 (go.mod:78).
//
// One name per 16-lane group, 16 names per 256-lane workgroup, grid-stride over the batch.
// Lane g of a group owns the name's 16-byte blocks j = g + 16k (k < ceil(m/16), m <= 128):
//   phase 1  PPP_j = AES(P_j ^ L_j)                    L_j = 2^(j+1) E(0)
//   mix      MP = T ^ xor_j PPP_j  (group butterfly), MC = AES(MP), M = MP ^ MC
//   phase 2  CCC_j = PPP_j ^ 2^j M  (j >= 1),  CCC_0 = MC ^ T ^ xor_{j>=1} CCC_j
//   phase 3  C_j = AES(CCC_j) ^ L_j
// (AES = decryption in the decrypt direction; L always uses AES encryption of 0.)  The PPP /
// CCC blocks live in the output buffer between phases, like the reference's C slice.
// Powers 2^j in GF(2^128) (little-endian bytes, reduction 0x87) are one shift-and-fold step
// per lane: x * 2^k = (x << k) ^ clmul(x >> (128-k), 0x87) for k <= 24.
// AES is T-table based with the four tables (and the inverse S-box) in LDS, built per
// workgroup from the compile-time S-box (xs_aes.h); round keys are kernel arguments (SGPRs).
#include "xs_aes.h"
#include "xs_internal.h"

namespace xs {

namespace {

__constant__ aes::Sbox kSbox = aes::make_sbox();

struct Tables {
  uint32_t te[4][256];
  uint32_t td[4][256];
  uint8_t isb[256];
};

__device__ __forceinline__ void aes_enc(const Tables& T, const uint32_t* rk, uint32_t s[4]) {
  uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
#pragma unroll
  for (int r = 1; r < 14; r++) {
    uint32_t t0 = T.te[0][s0 & 255] ^ T.te[1][(s1 >> 8) & 255] ^ T.te[2][(s2 >> 16) & 255] ^ T.te[3][s3 >> 24] ^ rk[4 * r];
    uint32_t t1 = T.te[0][s1 & 255] ^ T.te[1][(s2 >> 8) & 255] ^ T.te[2][(s3 >> 16) & 255] ^ T.te[3][s0 >> 24] ^ rk[4 * r + 1];
    uint32_t t2 = T.te[0][s2 & 255] ^ T.te[1][(s3 >> 8) & 255] ^ T.te[2][(s0 >> 16) & 255] ^ T.te[3][s1 >> 24] ^ rk[4 * r + 2];
    uint32_t t3 = T.te[0][s3 & 255] ^ T.te[1][(s0 >> 8) & 255] ^ T.te[2][(s1 >> 16) & 255] ^ T.te[3][s2 >> 24] ^ rk[4 * r + 3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  // te[2][x] = (s, 3s, 2s, s) and te[0][x] = (2s, s, s, 3s): pick S[x] out of the right byte.
#define SB_ROW(a, b, c, d) \
  ((T.te[2][(a) & 255] & 0xffu) | (T.te[0][((b) >> 8) & 255] & 0xff00u) | (T.te[0][((c) >> 16) & 255] & 0xff0000u) | \
   (T.te[2][(d) >> 24] & 0xff000000u))
  s[0] = SB_ROW(s0, s1, s2, s3) ^ rk[56];
  s[1] = SB_ROW(s1, s2, s3, s0) ^ rk[57];
  s[2] = SB_ROW(s2, s3, s0, s1) ^ rk[58];
  s[3] = SB_ROW(s3, s0, s1, s2) ^ rk[59];
#undef SB_ROW
}

__device__ __forceinline__ void aes_dec(const Tables& T, const uint32_t* dk, uint32_t s[4]) {
  uint32_t s0 = s[0] ^ dk[0], s1 = s[1] ^ dk[1], s2 = s[2] ^ dk[2], s3 = s[3] ^ dk[3];
#pragma unroll
  for (int r = 1; r < 14; r++) {
    uint32_t t0 = T.td[0][s0 & 255] ^ T.td[1][(s3 >> 8) & 255] ^ T.td[2][(s2 >> 16) & 255] ^ T.td[3][s1 >> 24] ^ dk[4 * r];
    uint32_t t1 = T.td[0][s1 & 255] ^ T.td[1][(s0 >> 8) & 255] ^ T.td[2][(s3 >> 16) & 255] ^ T.td[3][s2 >> 24] ^ dk[4 * r + 1];
    uint32_t t2 = T.td[0][s2 & 255] ^ T.td[1][(s1 >> 8) & 255] ^ T.td[2][(s0 >> 16) & 255] ^ T.td[3][s3 >> 24] ^ dk[4 * r + 2];
    uint32_t t3 = T.td[0][s3 & 255] ^ T.td[1][(s2 >> 8) & 255] ^ T.td[2][(s1 >> 16) & 255] ^ T.td[3][s0 >> 24] ^ dk[4 * r + 3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
#define ISB_ROW(a, b, c, d)                                                                       \
  ((uint32_t)T.isb[(a) & 255] | (uint32_t)T.isb[((b) >> 8) & 255] << 8 | (uint32_t)T.isb[((c) >> 16) & 255] << 16 | \
   (uint32_t)T.isb[(d) >> 24] << 24)
  s[0] = ISB_ROW(s0, s3, s2, s1) ^ dk[56];
  s[1] = ISB_ROW(s1, s0, s3, s2) ^ dk[57];
  s[2] = ISB_ROW(s2, s1, s0, s3) ^ dk[58];
  s[3] = ISB_ROW(s3, s2, s1, s0) ^ dk[59];
#undef ISB_ROW
}

// x *= 2^k in GF(2^128), little-endian bytes (eme multByTwo applied k times), 0 <= k <= 24.
__device__ __forceinline__ void gf_mul_pow2(uint32_t x[4], uint32_t k) {
  uint32_t t = (uint32_t)(((uint64_t)x[3] << k) >> 32);
  x[3] = (uint32_t)(((((uint64_t)x[3] << 32) | x[2]) << k) >> 32);
  x[2] = (uint32_t)(((((uint64_t)x[2] << 32) | x[1]) << k) >> 32);
  x[1] = (uint32_t)(((((uint64_t)x[1] << 32) | x[0]) << k) >> 32);
  x[0] = (x[0] << k) ^ t ^ (t << 1) ^ (t << 2) ^ (t << 7);
}

__device__ __forceinline__ void group_xor(uint32_t v[4]) {
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1)
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] ^= (uint32_t)__shfl_xor((int)v[i], d, 16);
}

template <bool ENC>
__device__ __forceinline__ void aes_dir(const Tables& T, const aes::EmeKey& key, uint32_t s[4]) {
  if (ENC)
    aes_enc(T, key.erk, s);
  else
    aes_dec(T, key.drk, s);
}

template <bool ENC>
__global__ __launch_bounds__(256) void xs_eme(aes::EmeKey key, const xs_name_desc* __restrict__ desc, uint64_t n,
                                              const uint8_t* src, uint8_t* dst, uint64_t buf_len) {
  __shared__ Tables T;
  for (int x = threadIdx.x; x < 256; x += blockDim.x) {
    uint32_t e = aes::te0(kSbox.fwd[x]);
#pragma unroll
    for (int w = 0; w < 4; w++) T.te[w][x] = w ? aes::rotl32(e, 8 * w) : e;
    if (!ENC) {
      uint32_t d = aes::td0(kSbox.inv[x]);
#pragma unroll
      for (int w = 0; w < 4; w++) T.td[w][x] = w ? aes::rotl32(d, 8 * w) : d;
      T.isb[x] = kSbox.inv[x];
    }
  }
  __syncthreads();

  const uint32_t g = threadIdx.x & 15;
  // L_g = 2^(g+1) * E(0): every lane encrypts the zero block once per workgroup.
  uint32_t Lb[4] = {0, 0, 0, 0};
  aes_enc(T, key.erk, Lb);
  gf_mul_pow2(Lb, g + 1);

  for (uint64_t base = (uint64_t)blockIdx.x * 16; base < n; base += (uint64_t)gridDim.x * 16) {
    const uint64_t idx = base + (threadIdx.x >> 4);
    uint32_t m = 0;
    uint64_t off = 0;
    if (idx < n) {
      xs_name_desc d = desc[idx];
      m = d.nblk;
      off = d.off;
      // a malformed descriptor is skipped (the host validates; this keeps the device safe)
      if (m == 0 || m > 128 || (off & 15) || off + 16ull * m > buf_len) m = 0;
    }
    const uint32_t kmax = (m + 15) >> 4;
    const uint4* in = (const uint4*)(src + off);
    uint4* out = (uint4*)(dst + off);

    // phase 1: PPP_j = AES(P_j ^ L_j), MP = T ^ xor PPP_j
    uint32_t acc[4] = {0, 0, 0, 0};
    uint32_t L[4] = {Lb[0], Lb[1], Lb[2], Lb[3]};
    for (uint32_t k = 0; k < kmax; k++) {
      uint32_t j = g + 16 * k;
      if (j < m) {
        uint4 p = in[j];
        uint32_t s[4] = {p.x ^ L[0], p.y ^ L[1], p.z ^ L[2], p.w ^ L[3]};
        aes_dir<ENC>(T, key, s);
        out[j] = make_uint4(s[0], s[1], s[2], s[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] ^= s[i];
      }
      gf_mul_pow2(L, 16);
    }
    group_xor(acc);
    uint32_t MP[4], MC[4], M[4];
#pragma unroll
    for (int i = 0; i < 4; i++) MP[i] = MC[i] = acc[i] ^ key.tweak[i];
    aes_dir<ENC>(T, key, MC);
#pragma unroll
    for (int i = 0; i < 4; i++) M[i] = MP[i] ^ MC[i];

    // phase 2: CCC_j = PPP_j ^ 2^j M (j >= 1); CCC_0 = MC ^ T ^ xor_{j>=1} CCC_j
    gf_mul_pow2(M, g);
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = 0;
    for (uint32_t k = 0; k < kmax; k++) {
      uint32_t j = g + 16 * k;
      if (j < m && j >= 1) {
        uint4 p = out[j];
        uint4 c = make_uint4(p.x ^ M[0], p.y ^ M[1], p.z ^ M[2], p.w ^ M[3]);
        out[j] = c;
        acc[0] ^= c.x;
        acc[1] ^= c.y;
        acc[2] ^= c.z;
        acc[3] ^= c.w;
      }
      gf_mul_pow2(M, 16);
    }
    group_xor(acc);

    // phase 3: C_j = AES(CCC_j) ^ L_j
#pragma unroll
    for (int i = 0; i < 4; i++) L[i] = Lb[i];
    for (uint32_t k = 0; k < kmax; k++) {
      uint32_t j = g + 16 * k;
      if (j < m) {
        uint32_t s[4];
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < 4; i++) s[i] = MC[i] ^ key.tweak[i] ^ acc[i];
        } else {
          uint4 p = out[j];
          s[0] = p.x;
          s[1] = p.y;
          s[2] = p.z;
          s[3] = p.w;
        }
        aes_dir<ENC>(T, key, s);
        out[j] = make_uint4(s[0] ^ L[0], s[1] ^ L[1], s[2] ^ L[2], s[3] ^ L[3]);
      }
      gf_mul_pow2(L, 16);
    }
  }
}

}  // namespace

hipError_t launch_eme(bool encrypt, const aes::EmeKey& key, const xs_name_desc* desc, uint64_t n, const uint8_t* src,
                      uint8_t* dst, uint64_t buf_len, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t groups = (n + 15) / 16;
  unsigned grid = (unsigned)(groups < 4096 ? groups : 4096);
  if (encrypt)
    hipLaunchKernelGGL(xs_eme<true>, dim3(grid), dim3(256), 0, stream, key, desc, n, src, dst, buf_len);
  else
    hipLaunchKernelGGL(xs_eme<false>, dim3(grid), dim3(256), 0, stream, key, desc, n, src, dst, buf_len);
  return hipGetLastError();
}

}  // namespace xs
