// DPP wave-scan check (decoder.hip wave_incl_min / wave_shr1): inclusive and exclusive min over 64 lanes vs a host loop
#include <hip/hip_runtime.h>
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_i(int old, int x) { return __builtin_amdgcn_update_dpp(old, x, CTRL, ROWM, 0xf, false); }
__device__ __forceinline__ float wave_incl_min_f(float v) {
  constexpr int inf = 0x7f800000;
  v = fminf(v, __int_as_float(dpp_i<0x111, 0xf>(inf, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_i<0x112, 0xf>(inf, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_i<0x114, 0xf>(inf, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_i<0x118, 0xf>(inf, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_i<0x142, 0xa>(inf, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_i<0x143, 0xc>(inf, __float_as_int(v))));
  return v;
}
__global__ void k(const float* in, float* out, float* ex) {
  float v = in[threadIdx.x];
  float s = wave_incl_min_f(v);
  out[threadIdx.x] = s;
  ex[threadIdx.x] = __int_as_float(dpp_i<0x138, 0xf>(0x7f800000, __float_as_int(s)));
}
int main() {
  float h[64], o[64], e[64]; for (int i = 0; i < 64; i++) h[i] = (float)((i * 37) % 61) - (i == 40 ? 100 : 0);
  float *di, *dout, *de; hipMalloc(&di, 256); hipMalloc(&dout, 256); hipMalloc(&de, 256);
  hipMemcpy(di, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(di, dout, de);
  hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost); hipMemcpy(e, de, 256, hipMemcpyDeviceToHost);
  int bad = 0; float run = INFINITY, prev = INFINITY;
  for (int i = 0; i < 64; i++) { run = fminf(run, h[i]); if (o[i] != run || e[i] != prev) { bad++; printf("lane %d: incl %g want %g, excl %g want %g\n", i, o[i], run, e[i], prev); } prev = run; }
  printf("dpp scan %s\n", bad ? "BAD" : "OK");
  return bad != 0;
}
