// Device helpers shared by the HIP translation units (kernels.hip, decoder.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace vamd {

// agent-scope relaxed accesses: global memory shared between the phases of
// a workgroup (and across launches) bypass the non-coherent per-CU cache
#define AG_LD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define AG_ST(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

// the same for 16-byte records (two 8-byte agent-scope accesses)
__device__ __forceinline__ int4 ag_ld4(const int4* p) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(const_cast<int4*>(p));
  const unsigned long long lo = AG_LD(q), hi = AG_LD(q + 1);
  return make_int4((int)(unsigned)lo, (int)(unsigned)(lo >> 32), (int)(unsigned)hi, (int)(unsigned)(hi >> 32));
}
__device__ __forceinline__ void ag_st4(int4* p, int4 v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  AG_ST(q, (unsigned long long)(unsigned)v.x | ((unsigned long long)(unsigned)v.y << 32));
  AG_ST(q + 1, (unsigned long long)(unsigned)v.z | ((unsigned long long)(unsigned)v.w << 32));
}

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
