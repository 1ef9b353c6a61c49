// xs_probe.hip -- benchmark utilities: the in-window shader clock probe (bench.py) and the
// round-trip check of synthetic SplitMix64 objects (the object-set mode, BASELINE configs[3]).
//
// One wave runs beside the crypt kernels on its own stream and records the shader clock counter
// (s_memtime) against the 100 MHz constant clock (s_memrealtime) at its start and then every
// ~20 us until the host raises a stop word (or max_ticks of the constant clock pass): the ratio
// over the timed window is the clock the crypt kernels ran at (MI355X_MICROARCH.md: the clock
// settles under sustained load; the VALU issue bound is priced at it).  Every store is a vector
// store from lane-indexed addresses.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xs_internal.h"

namespace {

__global__ void __launch_bounds__(64) xs_clock_probe(const volatile uint32_t* stop, uint64_t* out, uint64_t max_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t1 = t0, r1 = r0, n = 0;
  for (;;) {
    const uint64_t r = __builtin_amdgcn_s_memrealtime();
    if (r - r1 >= 2000) {  // ~20 us at 100 MHz
      t1 = __builtin_amdgcn_s_memtime();
      r1 = __builtin_amdgcn_s_memrealtime();
      n++;
      if (stop[0] != 0u || r1 - r0 >= max_ticks) break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x < 5) {  // lane-indexed vector stores
    const uint64_t v[5] = {t0, r0, t1, r1, n};
    out[threadIdx.x] = v[threadIdx.x];
  }
}

// Round-trip check of a synthetic object set: counts the 64-bit words of src that differ from
// the SplitMix64 stream xs_fill_splitmix (xs_kernels.hip) wrote -- the same formula and block
// layout (local 64 KiB block b = global block first_block + b*stride) -- into *mismatch.  Reading
// the opened plaintext alone halves the check's HBM bytes against comparing it with a kept copy.
// A lane adds its count with a vector atomic only when it found a mismatch.
__global__ void __launch_bounds__(256) xs_verify_splitmix(const uint64_t* __restrict__ src, uint64_t nwords,
                                                          uint64_t seed, uint64_t first_block, uint64_t stride,
                                                          unsigned long long* __restrict__ mismatch) {
  uint32_t bad = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = (first_block + (k >> 13) * stride) * 8192u + (k & 8191u);
    uint64_t z = seed + (g + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    bad += src[k] != (z ^ (z >> 31)) ? 1u : 0u;
  }
  if (bad) atomicAdd(mismatch, (unsigned long long)bad);
}

}  // namespace

extern "C" int xs_verify_blocks_dev(const void* d, uint64_t nblocks, uint64_t first_block, uint64_t block_stride,
                                    uint64_t seed, uint64_t* d_mismatch, void* stream) {
  if (!d || ((uintptr_t)d & 7u) || !d_mismatch || ((uintptr_t)d_mismatch & 7u) || block_stride == 0) {
    xs::set_error("xs_verify_blocks_dev: need 8-byte aligned buffers and block_stride >= 1");
    return XS_ERR_INVALID;
  }
  const uint64_t nwords = nblocks * 8192u;
  if (nwords == 0) return XS_OK;
  uint64_t grid = (nwords + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(xs_verify_splitmix, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t*)d, nwords, seed, first_block, block_stride, (unsigned long long*)d_mismatch);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    xs::set_error("verify launch: %s", hipGetErrorString(e));
    return XS_ERR_HIP;
  }
  return XS_OK;
}

extern "C" int xs_clock_probe_dev(const uint32_t* d_stop, uint64_t* d_out, double max_seconds, void* stream) {
  if (!d_stop || !d_out || max_seconds <= 0) {
    xs::set_error("xs_clock_probe_dev: bad argument");
    return XS_ERR_INVALID;
  }
  const uint64_t ticks = (uint64_t)(max_seconds * 1e8);
  hipLaunchKernelGGL(xs_clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, d_stop, d_out, ticks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    xs::set_error("clock probe launch: %s", hipGetErrorString(e));
    return XS_ERR_HIP;
  }
  return XS_OK;
}
