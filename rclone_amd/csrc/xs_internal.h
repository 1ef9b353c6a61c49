// Internal declarations shared by the HIP kernels and the C-ABI implementation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/rclone_crypt_gpu.h"

namespace xs {

struct KeyArg {
  uint32_t k[8];
};
struct NonceArg {
  uint32_t n[6];
};

// Per-block key schedule written by xs_keygen, read by xs_seal / xs_open (976 bytes).  Power
// tables (radix-2^26 limbs, uncanonicalised pmul outputs) depend on the block's length:
// full 64 KiB blocks take the matrix-core path, shorter ones the VALU Horner path.
struct __attribute__((aligned(16))) BlockKey {
  uint32_t subkey[8];  // HSalsa20(key, nonce[0:16])
  uint32_t n2[2];      // nonce[16:24] (Salsa20 words 6, 7)
  uint32_t len;        // plaintext bytes of this block
  uint32_t flags;
  uint64_t src;        // byte offset of the block's input (seal: plaintext; open: tag)
  uint64_t dst;        // byte offset of the block's output (seal: tag; open: plaintext)
  uint32_t s[4];       // Poly1305 s
  uint32_t ks1024[8];  // keystream block 1024 words 0..7 (message chunks 4094, 4095)
  uint32_t r[5];       // clamped r, radix 2^26
  uint32_t R[5];       // partial blocks: r^253 (gap between a lane's chunk groups)
  uint32_t corr[5];    // full blocks: key-only correction term added once per block
  uint32_t pad[1];
  union {
    struct {             // partial blocks (crypt_block)
      uint32_t T1[32][5];  // r^0 .. r^31
      uint32_t T2[8][5];   // r^(32a), a = 0..7 (a lane's final exponent is < 256)
    } part;
    struct {             // full blocks (crypt_block_mfma): r^(64k) = A[k&7] B[k>>3], r^e = C[e&7] D[e>>3]
      uint32_t A[8][5];    // r^(64i)
      uint32_t B[8][5];    // r^(512j)
      uint32_t C[8][5];    // r^b
      uint32_t D[9][5];    // r^(8a), a = 0..8
    } full;
  };
};
static_assert(sizeof(BlockKey) == 976, "BlockKey layout");

hipError_t launch_keygen(int mode, const KeyArg& key, const NonceArg& nonce0, uint64_t first_block,
                         uint64_t total_len, uint64_t nblocks, const xs_block_desc* desc, BlockKey* out,
                         hipStream_t stream);
hipError_t launch_crypt(bool seal, const BlockKey* keys, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                        uint8_t* ok, hipStream_t stream);
// keygen + split crypt in one launch for a tiny descriptor batch under one key (ranged reads);
// use only when nblocks <= fused_max_blocks().  With ctr != nullptr the last workgroup to finish
// resets *ctr (device memory, zero before the launch) and stores seq to *flag (pinned host
// memory, system scope) after every output of the batch is visible to the host.  host_desc
// (optional): the same descriptors in host memory; batches of <= XS_INLINE_DESCS blocks then travel
// in the kernel arguments and the kernel does not read desc over PCIe (v2 / v3).
constexpr int XS_INLINE_DESCS = 16;
// OPEN descriptors built by the engine for a ranged read (xs_engine_open_range) carry a group
// window in xs_block_desc.reserved: 0 = decrypt the whole block; XS_DESC_WINDOW | mask = decrypt
// only the 4 KiB groups g with bit g of mask set (the tag is verified over the whole block either
// way).  Group g is keystream blocks 64g..64g+63 = plaintext bytes [4096g - 32, 4096g + 4064); the
// block's last 32 bytes (keystream block 1024) are always written.  Only the fused v2 / v3
// kernels act on it (full blocks); every other path writes all bytes.
constexpr uint32_t XS_DESC_WINDOW = 0x80000000u;
constexpr uint64_t XS_WINDOW_GROUP = 4096;
// A fused batch of at most XS_KEY_PRE blocks (a ranged read: one or two) also carries each block's
// key setup, derived on the host while the launch is prepared: the HSalsa20 subkey and words 0..7
// of keystream blocks 0 (Poly1305 r, s) and 1024 (the last two chunks).  Three Salsa20 cores per
// block (~0.3 us on one host core) that would otherwise sit in front of the kernel's power tables
// and keystream, one after the other.
constexpr int XS_KEY_PRE = 2;
struct XsKeyPre {
  uint32_t sk[8], k0[8], k1024[8];
};
struct XsInlineDescs {
  xs_block_desc d[XS_INLINE_DESCS];
  XsKeyPre pre[XS_KEY_PRE];
  uint32_t n;     // d[0..n) valid; blocks >= n read desc
  uint32_t npre;  // pre[0..npre) valid (blocks >= npre derive their key setup in the kernel)
};
hipError_t launch_crypt_fused(bool seal, const KeyArg& key, const NonceArg& bounds, const xs_block_desc* desc,
                              const xs_block_desc* host_desc, uint64_t nblocks, const uint8_t* src, uint8_t* dst,
                              uint8_t* ok, uint32_t* ctr, uint32_t* flag, uint32_t seq, hipStream_t stream);
uint64_t fused_max_blocks();
hipError_t launch_md5(const xs_md5_desc* d, uint64_t n, const uint8_t* src, uint64_t src_len, uint8_t* digest,
                      uint8_t* ok, hipStream_t stream);
hipError_t launch_fill(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t first_block, uint64_t stride,
                       hipStream_t stream);

void set_error(const char* fmt, ...);
std::vector<int> default_devices();  // see rc_internal.h

}  // namespace xs
