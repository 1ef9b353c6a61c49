// The kernel of tools/microbench/aql_launch.cpp: one wave stores seq into pinned host memory
// (system scope), once, with a vector store.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void aql_word(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
