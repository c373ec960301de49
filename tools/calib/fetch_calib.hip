// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the decoder's access
// patterns on gfx950 (MI355X_MICROARCH.md "HBM": only 16-B/lane coalesced
// streaming reads and stores are calibrated; other widths must be calibrated
// on a known byte count).  Four kernels over a 2 GiB buffer (well past the
// 256 MiB Infinity Cache), each touching a known number of bytes:
//   stream_read   : every int4 once, coalesced                 (2 GiB)
//   gather16      : one 16-B load in each of N distinct 128-B lines
//   scatter4      : one 4-B store in each of N distinct 128-B lines
//   scatter16     : one 16-B store in each of N distinct 128-B lines
// Run under rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE); the
// printed byte counts are the denominators.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// line permutation: an odd multiplier modulo a power of two is a bijection
__device__ __forceinline__ unsigned long long perm(unsigned long long i, unsigned long long mask) {
  return (i * 0x9E3779B97F4A7C15ull + 12345ull) & mask;
}

__global__ void stream_read(const int4* __restrict__ a, long long n, int* out) {
  int acc = 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

__global__ void gather16(const int4* __restrict__ a, long long nlines_mask, long long n, int* out) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int4 v = a[perm(i, nlines_mask) * 8];  // one int4 at the start of a 128-B line
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7fffffff) out[0] = 1;
}

__global__ void scatter4(int* a, long long nlines_mask, long long n) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[perm(i, nlines_mask) * 32] = (int)i;  // one dword per 128-B line
}

__global__ void scatter16(int4* a, long long nlines_mask, long long n) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[perm(i, nlines_mask) * 8] = make_int4((int)i, 0, 0, 0);
}

int main() {
  const long long bytes = 2LL << 30;
  const long long n4 = bytes / 16, nlines = bytes / 128;
  int4* a;
  int* out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, bytes));
  const long long N = 1LL << 22;  // distinct lines touched by the scattered kernels
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(stream_read, dim3(8192), dim3(256), 0, 0, a, n4, out);
    hipLaunchKernelGGL(gather16, dim3((N + 255) / 256), dim3(256), 0, 0, a, nlines - 1, N, out);
    hipLaunchKernelGGL(scatter4, dim3((N + 255) / 256), dim3(256), 0, 0, (int*)a, nlines - 1, N);
    hipLaunchKernelGGL(scatter16, dim3((N + 255) / 256), dim3(256), 0, 0, a, nlines - 1, N);
  }
  CK(hipDeviceSynchronize());
  printf("{\"stream_read_bytes\": %lld, \"gather16_lines\": %lld, \"gather16_bytes\": %lld, "
         "\"scatter4_lines\": %lld, \"scatter4_bytes\": %lld, \"scatter16_lines\": %lld, \"scatter16_bytes\": %lld}\n",
         bytes, N, N * 16, N, N * 4, N, N * 16);
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
