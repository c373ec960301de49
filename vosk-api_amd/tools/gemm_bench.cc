// Standalone timing of the nnet GEMM kernel on the recipe's op shapes with
// synthetic rings/weights (no model, no decoder): `make gemm_bench` then
// ./build/gemm_bench [reps].  Development tool; results are not checked.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/kernels.h"
#include "../csrc/nnet_plan.h"

using namespace vamd;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

template <class T>
static T* Up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, sizeof(T) * v.size()));
  CK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

typedef float fx16 __attribute__((ext_vector_type(16)));
// MFMA-only throughput: NACC independent 32x32x2 f32 accumulators per wave
template <int NACC>
__global__ __launch_bounds__(256) void mfma_peak(float* out, int iters, long long* clk) {
  fx16 acc[NACC];
  for (int i = 0; i < NACC; i++)
    for (int j = 0; j < 16; j++) acc[i][j] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0f - a;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < NACC; i++)
    for (int j = 0; j < 16; j++) s += acc[i][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

static void PeakTest() {
  float* out;
  long long* clk;
  CK(hipMalloc(&out, sizeof(float) * 1024 * 256 * 8));
  CK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int wgs : {256, 512, 1024, 2048}) {
    const int iters = 2000;
    hipLaunchKernelGGL(mfma_peak<4>, dim3(wgs), dim3(256), 0, 0, out, iters, clk);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(mfma_peak<4>, dim3(wgs), dim3(256), 0, 0, out, iters, clk);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long c[2];
    CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
    const double fl = (double)wgs * 4 * iters * 4 * 32 * 32 * 2 * 2;
    printf("mfma_peak wgs=%d: %.1f us, %.1f TF/s, shader clk/realtime(100MHz) = %lld/%lld -> %.2f GHz\n",
           wgs, ms * 1e3, fl / (ms * 1e-3) * 1e-12, c[0], c[1], c[1] ? 0.1 * (double)c[0] / (double)c[1] : 0.0);
  }
}

int main(int argc, char** argv) {
  PeakTest();
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int S = 256, R = 512;
  // nodes: 0 = "prev" (512), 1 = "bottleneck" (96), 2 = out512, 3 = out96
  const int dims[4] = {512, 96, 512, 96};
  std::vector<float*> base(4);
  for (int i = 0; i < 4; i++) {
    size_t n = (size_t)R * S * dims[i];
    std::vector<float> h(n);
    for (size_t j = 0; j < n; j++) h[j] = (float)((j * 2654435761u) % 1000) * 1e-3f - 0.5f;
    base[i] = Up(h);
  }
  RingSet rs;
  rs.base = Up(base);
  rs.dim = Up(std::vector<int>(dims, dims + 4));
  rs.mask = R - 1;
  rs.ring = R;
  rs.slots = S;
  rs.input_node = -1;
  std::vector<float> w(512 * 1024);
  for (size_t j = 0; j < w.size(); j++) w[j] = (float)((j * 40503u) % 997) * 1e-3f - 0.5f;
  float* W = Up(w);
  std::vector<float> vv(512, 0.1f);
  float* V = Up(vv);
  std::vector<DevJob> jobs(S);
  for (int s = 0; s < S; s++) jobs[s] = DevJob{s, 100, 1 << 20, 0};
  DevJob* dj = Up(jobs);
  float* llh;
  CK(hipMalloc(&llh, sizeof(float) * 16 * 1024 * 1024));
  struct Shape { const char* name; int P, N, K, noop; };
  const Shape shapes[] = {{"linear P17", 17, 96, 1024, 0}, {"linear P51", 51, 96, 1024, 0},
                          {"noop P17", 17, 512, 192, 1},   {"noop P51", 51, 512, 192, 1},
                          {"output P17", 17, 2000, 192, 0}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool compact = getenv("GB_COMPACT") != nullptr;
  if (compact) {  // every A row inside a 512 KB (L2-resident) footprint
    rs.mask = 0;
    printf("compact A footprint\n");
  }
  const int only = getenv("GB_VAR") ? atoi(getenv("GB_VAR")) : -1;
  for (const Shape& sh : shapes) {
    std::vector<int> pat(sh.P);
    for (int k = 0; k < sh.P; k++) pat[k] = sh.P == 17 ? 3 * k : k;
    NnetOpArgs a;
    memset(&a, 0, sizeof(a));
    a.N = sh.N;
    a.K = sh.K;
    a.P = sh.P;
    a.M = S * sh.P;
    a.pattern = Up(pat);
    a.W = W;
    a.jobs = dj;
    a.rings = rs;
    a.llh = llh;
    const int src = sh.noop ? 1 : 0, sd = dims[src];
    a.nsegs = 2;
    a.segs[0] = DevSeg{base[src], sd, 0, -3, 0, sh.K / 2, 0};
    a.segs[1] = DevSeg{base[src], sd, 0, 0, sh.K / 2, sh.K / 2, 0};
    if (sh.N == 2000) {
      a.out_node = -1;
    } else {
      a.out_node = sh.noop ? 2 : 3;
      a.out_base = base[a.out_node];
      a.out_ldim = dims[a.out_node];
    }
    if (sh.noop) {
      a.nstages = 4;
      a.stages[0] = DevStage{nullptr, V, nullptr, 0, 0, 0, 0, 0, 0, 0.f};
      a.stages[1] = DevStage{nullptr, nullptr, nullptr, 1, 0, 0, 0, 0, 0, 0.f};
      a.stages[2] = DevStage{nullptr, V, V, 2, 0, 0, 0, 0, 0, 0.f};
      a.stages[3] = DevStage{base[0], nullptr, nullptr, 3, 512, 0, -3, 0, 1, 0.66f};
    }
    const double flops = 2.0 * a.M * a.N * a.K;
    a.kslices = GemmKSlices(a.K);
    for (int var = 1; var <= 3; var++) {
      if (only >= 0 && var != only) continue;
      if (var != 3 && !GemmStreamable(a)) continue;
      if (var == 3 && a.kslices != 1) continue;
      g_gemm_variant = var;
      for (int i = 0; i < 3; i++) LaunchNnetGemm(a, 32, st);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; i++) LaunchNnetGemm(a, 32, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      static const char* vn[4] = {"", "stream", "stream nb1", "lds bk32"};
      printf("%-11s M=%5d N=%4d K=%4d kslices=%d %-10s %8.1f us  %6.1f TF/s\n", sh.name, a.M, a.N,
             a.K, a.kslices, vn[var], us, flops / us * 1e-6);
    }
  }
  return 0;
}
