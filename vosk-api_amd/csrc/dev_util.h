// Device helpers shared by the HIP translation units (kernels.hip, decoder.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace vamd {

// agent-scope relaxed accesses: global memory shared between the phases of
// a workgroup (and across launches) bypass the non-coherent per-CU cache
#define AG_LD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define AG_ST(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

// order-preserving float <-> uint32 map (costs packed into 64-bit min keys)
__device__ __forceinline__ uint32_t ford(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funord(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

}  // namespace vamd
