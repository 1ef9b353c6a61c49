// xs_probe.hip -- in-window shader clock probe for the benchmark (bench.py).
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

}  // namespace

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
