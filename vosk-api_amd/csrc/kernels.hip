// HIP kernels of the MI355X-native Vosk hot path (gfx950 / CDNA4).
//
// Numerics contract: every kernel reproduces, operation for operation, the
// fp32 sequence of the CPU oracle (oracle/oracle.c) -- compiled with
// -ffp-contract=off, explicit fmaf where a fused multiply-add is meant, and
// fp32 MFMA (v_mfma_f32_32x32x2_f32, a k-ordered fma chain) for the GEMMs --
// so GPU-vs-oracle parity is bit-exact.
//
//   append_samples  PCM chunk -> per-stream sample ring
//   mfcc            one wave per 25 ms frame: DC removal, pre-emphasis,
//                   window, LDS radix-2 FFT, mel, log, DCT, lifter
//                   (Kaldi feat/feature-mfcc.cc [K]; src/model.cc:218-221)
//   nnet_gemm       fp32 MFMA GEMM whose A tiles are gathered from the
//                   per-stream activation time rings (spliced TDNN context
//                   staged in LDS) with fused bias/ReLU/BatchNorm/bypass
//                   epilogue (nnet3 components [K]; src/model.cc:233-246)
//   nnet_gather     descriptor evaluation (Append/Sum/Scale/Offset)
//   decode          one 1024-thread workgroup per stream, persistent over the
//                   chunk's frames: exact max-active cutoff by LDS radix
//                   select, load-balanced (token, arc) expansion, 64-bit
//                   atomicMin token recombination, epsilon closure by rounds
//                   (Kaldi LatticeFasterDecoder [K]; src/recognizer.cc:39-43)
//   traceback       best-path end selection + backpointer walk
#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine_dev.h"
#include "kernels.h"

namespace vamd {

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define AG_LD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define AG_ST(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

__device__ __forceinline__ uint32_t ford(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funord(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// natural log; identical operation sequence to orc_logf (oracle/oracle.c)
__device__ __forceinline__ float dev_logf(float x) {
  const float C0 = 1.000000000e+00f, C1 = -5.000000000e-01f, C2 = 3.333330154e-01f,
              C3 = -2.500002384e-01f, C4 = 2.000257671e-01f, C5 = -1.666804254e-01f,
              C6 = 1.421260685e-01f, C7 = -1.239922047e-01f, C8 = 1.192392558e-01f,
              C9 = -1.172722951e-01f, C10 = 6.740232557e-02f;
  uint32_t u = __float_as_uint(x);
  int e = (int)((u >> 23) & 0xff) - 127;
  float m = __uint_as_float((u & 0x7fffffu) | 0x3f800000u);
  if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
  float f = m - 1.0f;
  float p = C10;
  p = __builtin_fmaf(p, f, C9);
  p = __builtin_fmaf(p, f, C8);
  p = __builtin_fmaf(p, f, C7);
  p = __builtin_fmaf(p, f, C6);
  p = __builtin_fmaf(p, f, C5);
  p = __builtin_fmaf(p, f, C4);
  p = __builtin_fmaf(p, f, C3);
  p = __builtin_fmaf(p, f, C2);
  p = __builtin_fmaf(p, f, C1);
  p = __builtin_fmaf(p, f, C0);
  float fp = f * p;
  return __builtin_fmaf((float)e, 0.693147182f, fp);
}

// ===========================================================================
// samples
// ===========================================================================
__global__ void append_samples_kernel(const SampleJob* jobs, float* ring, int ring_len) {
  const SampleJob j = jobs[blockIdx.x];
  float* r = ring + (size_t)j.slot * ring_len;
  for (int i = threadIdx.x; i < j.count; i += blockDim.x)
    r[(j.pos + i) & (ring_len - 1)] = j.src[i];
}

void LaunchAppendSamples(const SampleJob* jobs, int njobs, float* ring, int ring_len,
                         hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(append_samples_kernel, dim3(njobs), dim3(256), 0, s, jobs, ring, ring_len);
}

// ===========================================================================
// MFCC: 4 frames per 256-thread block, one wave per frame
// ===========================================================================
constexpr int kMfccMaxN = 512;

__global__ __launch_bounds__(256) void mfcc_kernel(MfccDev m, const MfccJob* jobs, int njobs,
                                                   int total, const float* ring, int ring_len,
                                                   RingSet rings) {
  __shared__ float X[4][kMfccMaxN];
  __shared__ float RE[4][kMfccMaxN];
  __shared__ float IM[4][kMfccMaxN];
  __shared__ float MEL[4][64];
  __shared__ float SC[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  const bool valid = row < total;
  // locate the job (rows are grouped per job, ascending row0)
  int slot = 0, frame = 0;
  if (valid) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].row0 <= row) lo = mid; else hi = mid - 1;
    }
    slot = jobs[lo].slot;
    frame = jobs[lo].first + (row - jobs[lo].row0);
  }
  const int L = m.frame_length, N = m.padded;
  float* x = X[w];
  float* re = RE[w];
  float* im = IM[w];
  const float* src = ring + (size_t)slot * ring_len;
  const long long s0 = (long long)frame * m.frame_shift;
  for (int i = lane; i < L; i += 64)
    x[i] = valid ? src[(s0 + i) & (ring_len - 1)] : 0.0f;
  __syncthreads();
  if (lane == 0) {
    float c = 0.0f;
    if (m.remove_dc) {
      float sum = 0.0f;
      for (int i = 0; i < L; i++) sum = sum + x[i];
      c = -sum / (float)L;
    }
    SC[w][0] = c;
  }
  __syncthreads();
  if (m.remove_dc) {
    const float c = SC[w][0];
    for (int i = lane; i < L; i += 64) x[i] = x[i] + c;
  }
  __syncthreads();
  if (m.use_energy && lane == 0) {
    float e = 0.0f;
    for (int i = 0; i < L; i++) e = __builtin_fmaf(x[i], x[i], e);
    SC[w][1] = dev_logf(e > 1.1920929e-07f ? e : 1.1920929e-07f);
  }
  // pre-emphasis (from the un-emphasised values), window, bit-reversed store
  const float p = m.preemph;
  for (int i = lane; i < N; i += 64) {
    float v = 0.0f;
    if (i < L) {
      float xi = x[i];
      if (p != 0.0f) {
        float xp = i > 0 ? x[i - 1] : x[0];
        xi = xi - p * xp;
      }
      v = xi * m.window[i];
    }
    int r = (int)(__brev((unsigned)i) >> (32 - m.log2n));
    re[r] = v;
    im[r] = 0.0f;
  }
  // radix-2 DIT FFT
  for (int len = 2; len <= N; len <<= 1) {
    __syncthreads();
    const int half = len >> 1, step = N / len;
    for (int b = lane; b < (N >> 1); b += 64) {
      const int grp = b / half, j = b - grp * half, i = grp * len + j;
      const float wr = m.twr[j * step], wi = m.twi[j * step];
      const float br = re[i + half], bi = im[i + half];
      const float tr = br * wr - bi * wi;
      const float ti = br * wi + bi * wr;
      const float ur = re[i], ui = im[i];
      re[i] = ur + tr;
      im[i] = ui + ti;
      re[i + half] = ur - tr;
      im[i + half] = ui - ti;
    }
  }
  __syncthreads();
  if (lane < m.num_bins) {
    float e = 0.0f;
    const int f0 = m.mel_first[lane], f1 = m.mel_last[lane];
    const float* wrow = m.melw + (size_t)lane * m.nfft;
    if (f0 >= 0)
      for (int i = f0; i <= f1; i++) {
        float pw = re[i] * re[i] + im[i] * im[i];
        e = __builtin_fmaf(wrow[i], pw, e);
      }
    if (e < 1.1920929e-07f) e = 1.1920929e-07f;
    MEL[w][lane] = dev_logf(e);
  }
  __syncthreads();
  if (valid && lane < m.num_ceps) {
    float c = 0.0f;
    const float* drow = m.dct + (size_t)lane * m.num_bins;
    for (int j = 0; j < m.num_bins; j++) c = __builtin_fmaf(drow[j], MEL[w][j], c);
    float out = c * m.lifter[lane];
    if (m.use_energy && lane == 0) out = SC[w][1];
    const int in = rings.input_node;
    float* dst = rings.base[in] +
                 ((size_t)slot * rings.ring + (frame & rings.mask)) * rings.dim[in];
    dst[lane] = out;
  }
}

void LaunchMfcc(const MfccDev& m, const MfccJob* jobs, int njobs, int total, const float* ring,
                int ring_len, const RingSet& rings, hipStream_t s) {
  if (total <= 0) return;
  hipLaunchKernelGGL(mfcc_kernel, dim3((total + 3) / 4), dim3(256), 0, s, m, jobs, njobs, total,
                     ring, ring_len, rings);
}

// ===========================================================================
// nnet3 ops
// ===========================================================================
__device__ __forceinline__ const float* ring_row(const RingSet& r, int node, int slot, int tau,
                                                int clamp_max) {
  if (node == r.input_node) {
    if (tau < 0) tau = 0;
    if (tau > clamp_max) tau = clamp_max;
  }
  return r.base[node] + ((size_t)slot * r.ring + (tau & r.mask)) * r.dim[node];
}

__device__ __forceinline__ float apply_stages(const NnetOpArgs& a, float x, int col, int slot,
                                              int tau, int clamp_max) {
  for (int s = 0; s < a.nstages; s++) {
    const DevStage& st = a.stages[s];
    switch (st.kind) {
      case 0: x = x + a.vecs[st.vec0][col]; break;                   // bias
      case 1: x = x < 0.0f ? 0.0f : x; break;                        // ReLU
      case 2: x = x * a.vecs[st.vec0][col] + a.vecs[st.vec1][col]; break;  // BN / scale+offset
      case 3: {                                                      // bypass Sum()
        float z = ring_row(a.rings, st.node, slot, tau + st.offset, clamp_max)[st.src_col + col];
        x = st.scaled ? (st.c * z) + x : z + x;
        break;
      }
      default: x = x * st.c; break;                                  // scale
    }
  }
  return x;
}

__device__ __forceinline__ void row_info(const NnetOpArgs& a, int r, int* slot, int* tau,
                                         int* clamp) {
  const int job = r / a.P, k = r - job * a.P;
  const DevJob j = a.jobs[job];
  *slot = j.slot;
  *tau = j.base_t + a.pattern[k];
  *clamp = j.clamp_max;
}

__device__ __forceinline__ void store_out(const NnetOpArgs& a, int r, int col, int slot, int tau,
                                          float v) {
  if (a.out_node < 0) {
    a.llh[(size_t)r * a.N + col] = v;
  } else {
    float* dst = a.rings.base[a.out_node] +
                 ((size_t)slot * a.rings.ring + (tau & a.rings.mask)) * a.rings.dim[a.out_node];
    dst[col] = v;
  }
}

// 64x64 output tile per 256-thread workgroup; each wave owns a 32x32 block
// computed with v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate, exact
// k-ordered fma chain).  A rows are gathered from the stored-node rings at
// (tau + segment offset): the TDNN splice happens in the LDS staging.
template <int BK>
__global__ __launch_bounds__(256) void nnet_gemm_kernel(NnetOpArgs a) {
  __shared__ float As[64][BK + 1];
  __shared__ float Bs[BK][65];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  constexpr int Q = BK / 4;           // float4 per row per K-step
  constexpr int NV = 64 * Q;          // float4 per tile
  // per-thread A rows (fixed across K-steps)
  int r_slot[(NV + 255) / 256], r_tau[(NV + 255) / 256], r_clamp[(NV + 255) / 256];
  bool r_ok[(NV + 255) / 256];
#pragma unroll
  for (int v = 0; v < (NV + 255) / 256; v++) {
    const int idx = tid + v * 256;
    const int row = idx / Q;
    const int gr = m0 + row;
    r_ok[v] = idx < NV && gr < a.M;
    r_slot[v] = 0; r_tau[v] = 0; r_clamp[v] = 0;
    if (r_ok[v]) row_info(a, gr, &r_slot[v], &r_tau[v], &r_clamp[v]);
  }
  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;
  int seg = 0;
  for (int k0 = 0; k0 < a.K; k0 += BK) {
    while (!(k0 >= a.segs[seg].col0 && k0 < a.segs[seg].col0 + a.segs[seg].dim)) seg++;
    const DevSeg S = a.segs[seg];
#pragma unroll
    for (int v = 0; v < (NV + 255) / 256; v++) {
      const int idx = tid + v * 256;
      if (idx < NV) {
        const int row = idx / Q, q = idx - row * Q;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r_ok[v]) {
          const float* p = ring_row(a.rings, S.node, r_slot[v], r_tau[v] + S.offset, r_clamp[v]);
          val = *reinterpret_cast<const float4*>(p + S.src_col + (k0 - S.col0) + 4 * q);
        }
        As[row][4 * q + 0] = val.x;
        As[row][4 * q + 1] = val.y;
        As[row][4 * q + 2] = val.z;
        As[row][4 * q + 3] = val.w;
      }
    }
#pragma unroll
    for (int v = 0; v < (NV + 255) / 256; v++) {
      const int idx = tid + v * 256;
      if (idx < NV) {
        const int n = idx / Q, q = idx - n * Q;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n0 + n < a.N)
          val = *reinterpret_cast<const float4*>(a.W + (size_t)(n0 + n) * a.K + k0 + 4 * q);
        Bs[4 * q + 0][n] = val.x;
        Bs[4 * q + 1][n] = val.y;
        Bs[4 * q + 2][n] = val.z;
        Bs[4 * q + 3][n] = val.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float av = As[wr * 32 + (lane & 31)][kk + (lane >> 5)];
      const float bv = Bs[kk + (lane >> 5)][wc * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = n0 + wc * 32 + (lane & 31);
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int row = m0 + wr * 32 + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
    if (row < a.M && col < a.N) {
      int slot, tau, clamp;
      row_info(a, row, &slot, &tau, &clamp);
      const float v = apply_stages(a, acc[j], col, slot, tau, clamp);
      store_out(a, row, col, slot, tau, v);
    }
  }
}

void LaunchNnetGemm(const NnetOpArgs& a, int bk, hipStream_t s) {
  if (a.M <= 0) return;
  dim3 grid((a.M + 63) / 64, (a.N + 63) / 64);
  if (bk == 32) hipLaunchKernelGGL(nnet_gemm_kernel<32>, grid, dim3(256), 0, s, a);
  else if (bk == 16) hipLaunchKernelGGL(nnet_gemm_kernel<16>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(nnet_gemm_kernel<8>, grid, dim3(256), 0, s, a);
}

__global__ __launch_bounds__(256) void nnet_gather_kernel(NnetOpArgs a) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)a.M * a.N) return;
  const int row = (int)(e / a.N), col = (int)(e - (long long)row * a.N);
  int slot, tau, clamp;
  row_info(a, row, &slot, &tau, &clamp);
  int p = 0;
  while (col >= a.parts[p].col0 + a.parts[p].dim) p++;
  const DevPart P = a.parts[p];
  const int d = col - P.col0;
  float stack[8];
  int sp = 0;
  for (int i = 0; i < P.ninstr; i++) {
    const DevInstr in = a.instr[P.instr0 + i];
    if (in.op == 0) stack[sp++] = ring_row(a.rings, in.node, slot, tau + in.offset, clamp)[in.src_col + d];
    else if (in.op == 1) stack[sp - 1] = in.c * stack[sp - 1];
    else if (in.op == 2) { stack[sp - 2] = stack[sp - 2] + stack[sp - 1]; sp--; }
    else stack[sp++] = in.c;
  }
  const float v = apply_stages(a, stack[0], col, slot, tau, clamp);
  store_out(a, row, col, slot, tau, v);
}

void LaunchNnetGather(const NnetOpArgs& a, hipStream_t s) {
  long long n = (long long)a.M * a.N;
  if (n <= 0) return;
  hipLaunchKernelGGL(nnet_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

// ===========================================================================
// token passing
// ===========================================================================
constexpr int DT = 1024;         // threads per decoder workgroup
constexpr int DW = DT / 64;      // waves
constexpr int kLlhLds = 8192;    // log-likelihood row staged in LDS up to this size
constexpr unsigned long long kEmpty = 0xffffffffffffffffull;

struct DecShared {
  int scan[DT + 1];   // exclusive prefix sums of the chunk's degrees
  int abeg[DT];       // first arc per chunk token
  float tcost[DT];    // cost per chunk token
  unsigned hist[256];
  unsigned long long red_u[DW];
  float red_f[DW];
  int red_i[DW];
  int n_new, n_next, total, sel_k;
  unsigned sel_prefix, sel_mask;
  float seed;
  int bad;
};

__device__ __forceinline__ float wave_min_f(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

__device__ float block_min_f(DecShared& sh, float v) {
  v = wave_min_f(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh.red_f[w] = v;
  __syncthreads();
  float r = sh.red_f[0];
  for (int i = 1; i < DW; i++) r = fminf(r, sh.red_f[i]);
  return r;
}

__device__ unsigned long long block_min_u64(DecShared& sh, unsigned long long v) {
  v = wave_min_u64(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh.red_u[w] = v;
  __syncthreads();
  unsigned long long r = sh.red_u[0];
  for (int i = 1; i < DW; i++) r = sh.red_u[i] < r ? sh.red_u[i] : r;
  return r;
}

// exclusive scan of deg over the block; writes sh.scan[0..DT], sh.total
__device__ void block_scan(DecShared& sh, int deg) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int v = deg;
  for (int o = 1; o < 64; o <<= 1) {
    int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  __syncthreads();
  if (lane == 63) sh.red_i[w] = v;
  __syncthreads();
  int off = 0;
  for (int i = 0; i < w; i++) off += sh.red_i[i];
  sh.scan[threadIdx.x] = off + v - deg;
  if (threadIdx.x == DT - 1) {
    sh.scan[DT] = off + v;
    sh.total = off + v;
  }
  __syncthreads();
}

// token index j within the chunk that owns item `it` (largest j: scan[j] <= it)
__device__ __forceinline__ int owner(const DecShared& sh, int it) {
  int lo = 0, hi = DT - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (sh.scan[mid] <= it) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// exact k-th smallest (0-based) of cost[0..n) by 4-pass 8-bit radix select
__device__ float kth_smallest(DecShared& sh, const float* cost, int n, int k) {
  if (threadIdx.x == 0) {
    sh.sel_prefix = 0;
    sh.sel_mask = 0;
    sh.sel_k = k;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += DT) sh.hist[i] = 0;
    __syncthreads();
    const unsigned prefix = sh.sel_prefix, mask = sh.sel_mask;
    for (int i = threadIdx.x; i < n; i += DT) {
      const unsigned u = ford(AG_LD(&cost[i]));
      if ((u & mask) == prefix) atomicAdd(&sh.hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int kk = sh.sel_k;
      unsigned b = 0;
      for (; b < 256; b++) {
        if (kk < (int)sh.hist[b]) break;
        kk -= (int)sh.hist[b];
      }
      sh.sel_k = kk;
      sh.sel_prefix = prefix | (b << shift);
      sh.sel_mask = mask | (255u << shift);
    }
  }
  __syncthreads();
  return funord(sh.sel_prefix);
}

struct DecPtrs {
  unsigned long long* key;
  int* pos_cur;
  int* pos_new;
  int* stamp;
  int* cs;
  float* cc;
  int* nl;
  int* fa;
  int* fb;
  int2* arena;
};

// relax dest with (tot, arc); appends newly created tokens; returns improvement
__device__ __forceinline__ bool relax(const DecArgs& a, DecShared& sh, const DecPtrs& p, int dest,
                                      float tot, int arc) {
  const unsigned long long k = ((unsigned long long)ford(tot) << 32) | (unsigned)arc;
  const unsigned long long old = atomicMin(&p.key[dest], k);
  if (old == kEmpty) {
    const int pos = atomicAdd(&sh.n_new, 1);
    if (pos < a.max_tok) {
      AG_ST(&p.nl[pos], dest);
      AG_ST(&p.pos_new[dest], pos);
    } else {
      sh.bad |= 1;
    }
  }
  return k < old;
}

// epsilon closure of the frame under construction (ProcessNonemitting)
__device__ void eps_closure(const DecArgs& a, DecShared& sh, DecPtrs& p, DecSlot& st, float cutoff,
                            int* arcs_eps) {
  int nfront = sh.n_new < a.max_tok ? sh.n_new : a.max_tok;
  const int* front = p.nl;
  int* next = p.fa;
  int examined = 0;
  while (nfront > 0) {
    st.stamp++;
    const int stamp = st.stamp;
    __syncthreads();
    if (threadIdx.x == 0) sh.n_next = 0;
    for (int c0 = 0; c0 < nfront; c0 += DT) {
      const int i = c0 + threadIdx.x;
      int deg = 0, ab = 0;
      float c = 0.0f;
      if (i < nfront) {
        const int s = AG_LD(&front[i]);
        c = funord((uint32_t)(AG_LD(&p.key[s]) >> 32));
        if (c <= cutoff) {
          const int4 si = a.sinfo[s];
          ab = si.y;
          deg = si.z - si.y;
        }
      }
      block_scan(sh, deg);
      sh.abeg[threadIdx.x] = ab;
      sh.tcost[threadIdx.x] = c;
      __syncthreads();
      const int total = sh.total;
      examined += total;
      for (int it = threadIdx.x; it < total; it += DT) {
        const int j = owner(sh, it);
        const int arc = sh.abeg[j] + (it - sh.scan[j]);
        const int4 A = a.arcs[arc];
        const float tot = sh.tcost[j] + __int_as_float(A.y);
        if (tot < cutoff) {
          if (relax(a, sh, p, A.x, tot, arc) && atomicExch(&p.stamp[A.x], stamp) != stamp) {
            const int q = atomicAdd(&sh.n_next, 1);
            if (q < a.max_tok) AG_ST(&next[q], A.x);
            else sh.bad |= 1;
          }
        }
      }
      __syncthreads();
    }
    nfront = sh.n_next < a.max_tok ? sh.n_next : a.max_tok;
    front = next;
    next = (next == p.fa) ? p.fb : p.fa;
  }
  *arcs_eps += examined;
}

// move the frame under construction into the arena + current token arrays
__device__ void commit(const DecArgs& a, DecShared& sh, DecPtrs& p, DecSlot& st, float* best_out) {
  __syncthreads();
  const int n = sh.n_new < a.max_tok ? sh.n_new : a.max_tok;
  const int base = st.arena_used;
  bool ok = (long long)base + n <= a.arena_cap;
  float best = __int_as_float(0x7f800000);
  if (ok) {
    for (int j = threadIdx.x; j < n; j += DT) {
      const int s = AG_LD(&p.nl[j]);
      const unsigned long long k = AG_LD(&p.key[s]);
      const int arc = (int)(unsigned)(k & 0xffffffffu);
      const float cost = funord((uint32_t)(k >> 32));
      int prev = -1;
      if (arc >= 0) {
        const int src = a.arc_src[arc];
        prev = a.arcs[arc].z >= 0 ? st.cur_base + AG_LD(&p.pos_cur[src])
                                  : base + AG_LD(&p.pos_new[src]);
      }
      p.arena[base + j] = make_int2(prev, arc);
      AG_ST(&p.cs[j], s);
      AG_ST(&p.cc[j], cost);
      best = fminf(best, cost);
    }
  }
  // keys must be reset even if the arena overflowed
  for (int j = threadIdx.x; j < n; j += DT) {
    const int s = AG_LD(&p.nl[j]);
    AG_ST(&p.key[s], kEmpty);
  }
  best = block_min_f(sh, best);
  if (!ok) sh.bad |= 2;
  __syncthreads();
  if (ok) {
    st.cur_base = base;
    st.arena_used = base + n;
    st.ntok = n;
  } else {
    st.ntok = 0;
  }
  int* t = p.pos_cur;
  p.pos_cur = p.pos_new;
  p.pos_new = t;
  st.parity ^= 1;
  *best_out = best;
}

__global__ __launch_bounds__(DT) void decode_kernel(DecArgs a) {
  __shared__ DecShared sh;
  __shared__ float L[kLlhLds];
  const DecJob job = a.jobs[blockIdx.x];
  const int slot = job.slot;
  const long long S = a.num_states;
  DecSlot st = a.slots[slot];
  DecPtrs p;
  p.key = a.key + slot * S;
  p.pos_cur = a.posmap + slot * 2 * S + st.parity * S;
  p.pos_new = a.posmap + slot * 2 * S + (st.parity ^ 1) * S;
  p.stamp = a.stamp + slot * S;
  p.cs = a.cur_state + (long long)slot * a.max_tok;
  p.cc = a.cur_cost + (long long)slot * a.max_tok;
  p.nl = a.new_list + (long long)slot * a.max_tok;
  p.fa = a.front_a + (long long)slot * a.max_tok;
  p.fb = a.front_b + (long long)slot * a.max_tok;
  p.arena = a.arena + (long long)slot * a.arena_cap;
  if (threadIdx.x == 0) sh.bad = 0;
  int arcs_eps = 0;

  if (job.reset) {  // InitDecoding: start token, closure with cutoff = beam
    st.ntok = 0;
    st.cur_base = 0;
    st.arena_used = 0;
    st.frames = 0;
    st.offset_sum = 0.0;
    st.err = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      sh.n_new = 1;
      AG_ST(&p.key[a.start_state], ((unsigned long long)ford(0.0f) << 32) | 0xffffffffu);
      AG_ST(&p.nl[0], a.start_state);
      AG_ST(&p.pos_new[a.start_state], 0);
    }
    __syncthreads();
    eps_closure(a, sh, p, st, a.beam, &arcs_eps);
    float b;
    commit(a, sh, p, st, &b);
  }

  for (int f = 0; f < job.nframes; f++) {
    if (st.ntok == 0 || st.err) break;
    const float* llh = a.llh + (size_t)(job.llh_row0 + f) * a.P;
    const float* Lp = llh;
    if (a.P <= kLlhLds) {
      for (int i = threadIdx.x; i < a.P; i += DT) L[i] = llh[i];
      Lp = L;
    }
    const int ntok = st.ntok;
    // ---- GetCutoff
    unsigned long long bk = kEmpty;
    for (int i = threadIdx.x; i < ntok; i += DT) {
      const unsigned long long k =
          ((unsigned long long)ford(AG_LD(&p.cc[i])) << 32) | (unsigned)AG_LD(&p.cs[i]);
      bk = k < bk ? k : bk;
    }
    bk = block_min_u64(sh, bk);
    const float best = funord((uint32_t)(bk >> 32));
    const int best_state = (int)(unsigned)(bk & 0xffffffffu);
    const float beam_cutoff = best + a.beam;
    float max_cut = __int_as_float(0x7f800000), min_cut = __int_as_float(0x7f800000);
    float adaptive, cutoff;
    if (ntok > a.max_active) max_cut = kth_smallest(sh, p.cc, ntok, a.max_active);
    if (max_cut < beam_cutoff) {
      adaptive = max_cut - best + a.beam_delta;
      cutoff = max_cut;
    } else {
      if (ntok > a.min_active)
        min_cut = a.min_active == 0 ? best : kth_smallest(sh, p.cc, ntok, a.min_active);
      if (min_cut > beam_cutoff) {
        adaptive = min_cut - best + a.beam_delta;
        cutoff = min_cut;
      } else {
        adaptive = a.beam;
        cutoff = beam_cutoff;
      }
    }
    const float cost_offset = -best;
    // ---- ProcessEmitting: seed from the best token's arcs
    if (threadIdx.x == 0) {
      float seed = __int_as_float(0x7f800000);
      const int4 si = a.sinfo[best_state];
      for (int arc = si.x; arc < si.y; arc++) {
        const int4 A = a.arcs[arc];
        const float nw = ((__int_as_float(A.y) + cost_offset) - Lp[A.z]) + best;
        if (nw + adaptive < seed) seed = nw + adaptive;
      }
      sh.seed = seed;
      sh.n_new = 0;
    }
    // pass A: minimum tot over all emitting expansions; pass B: relax
    float m = __int_as_float(0x7f800000);
    float next_cutoff = 0.0f;
    int examined = 0;
    for (int pass = 0; pass < 2; pass++) {
      for (int c0 = 0; c0 < ntok; c0 += DT) {
        const int i = c0 + threadIdx.x;
        int deg = 0, ab = 0;
        float c = 0.0f;
        if (i < ntok) {
          c = AG_LD(&p.cc[i]);
          if (c <= cutoff) {
            const int4 si = a.sinfo[AG_LD(&p.cs[i])];
            ab = si.x;
            deg = si.y - si.x;
          }
        }
        block_scan(sh, deg);
        sh.abeg[threadIdx.x] = ab;
        sh.tcost[threadIdx.x] = c;
        __syncthreads();
        const int total = sh.total;
        if (pass == 0) examined += total;
        for (int it = threadIdx.x; it < total; it += DT) {
          const int j = owner(sh, it);
          const int arc = sh.abeg[j] + (it - sh.scan[j]);
          const int4 A = a.arcs[arc];
          const float ac = cost_offset - Lp[A.z];
          const float tot = (sh.tcost[j] + ac) + __int_as_float(A.y);
          if (pass == 0) m = fminf(m, tot);
          else if (tot < next_cutoff) relax(a, sh, p, A.x, tot, arc);
        }
        __syncthreads();
      }
      if (pass == 0) {
        m = block_min_f(sh, m);
        next_cutoff = sh.seed;
        if (m + adaptive < next_cutoff) next_cutoff = m + adaptive;
      }
    }
    // ---- ProcessNonemitting
    eps_closure(a, sh, p, st, next_cutoff, &arcs_eps);
    float new_best;
    commit(a, sh, p, st, &new_best);
    st.offset_sum += (double)cost_offset;
    st.frames++;
    if (threadIdx.x == 0 && a.stats) {
      FrameStat fs;
      fs.ntok_in = ntok;
      fs.ntok_out = st.ntok;
      fs.arcs_emit = examined;
      fs.arcs_eps = arcs_eps;
      fs.best = new_best;
      fs.cutoff = cutoff;
      fs.next_cutoff = next_cutoff;
      fs.adaptive_beam = adaptive;
      a.stats[job.stats_row0 + f] = fs;
    }
    arcs_eps = 0;
    __syncthreads();
    if (sh.bad) st.err |= sh.bad;
  }
  __syncthreads();
  if (sh.bad) st.err |= sh.bad;
  if (st.ntok == 0 && !st.err) st.err |= 4;
  if (threadIdx.x == 0) a.slots[slot] = st;
}

void LaunchDecode(const DecArgs& a, int njobs, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(decode_kernel, dim3(njobs), dim3(DT), 0, s, a);
}

// ---------------------------------------------------------------------------
// traceback: best end token (with final costs if any is final), then walk
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void traceback_kernel(TraceArgs a) {
  __shared__ unsigned long long red[4];
  __shared__ float redf[4][2];
  __shared__ int endpos;
  const int slot = a.req_slot[blockIdx.x];
  const DecSlot st = a.slots[slot];
  const int* cs = a.cur_state + (long long)slot * a.max_tok;
  const float* cc = a.cur_cost + (long long)slot * a.max_tok;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float bn = __int_as_float(0x7f800000), bf = __int_as_float(0x7f800000);
  for (int i = threadIdx.x; i < st.ntok; i += 256) {
    const float c = cc[i];
    bn = fminf(bn, c);
    const float fc = __int_as_float(a.sinfo[cs[i]].w);
    if (fc != __int_as_float(0x7f800000)) bf = fminf(bf, c + fc);
  }
  for (int o = 32; o > 0; o >>= 1) {
    bn = fminf(bn, __shfl_xor(bn, o, 64));
    bf = fminf(bf, __shfl_xor(bf, o, 64));
  }
  if (lane == 0) { redf[w][0] = bn; redf[w][1] = bf; }
  __syncthreads();
  bn = fminf(fminf(redf[0][0], redf[1][0]), fminf(redf[2][0], redf[3][0]));
  bf = fminf(fminf(redf[0][1], redf[1][1]), fminf(redf[2][1], redf[3][1]));
  const bool any_final = bf != __int_as_float(0x7f800000);
  const bool use_f = a.use_final && any_final;
  unsigned long long bk = kEmpty;
  for (int i = threadIdx.x; i < st.ntok; i += 256) {
    float c = cc[i];
    if (use_f) c = c + __int_as_float(a.sinfo[cs[i]].w);
    const unsigned long long k = ((unsigned long long)ford(c) << 32) | (unsigned)cs[i];
    bk = k < bk ? k : bk;
  }
  bk = wave_min_u64(bk);
  if (lane == 0) red[w] = bk;
  if (threadIdx.x == 0) endpos = -1;
  __syncthreads();
  bk = red[0];
  for (int i = 1; i < 4; i++) bk = red[i] < bk ? red[i] : bk;
  for (int i = threadIdx.x; i < st.ntok; i += 256)
    if (cs[i] == (int)(unsigned)(bk & 0xffffffffu)) endpos = i;
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = 0;
    int* out = a.path + (long long)blockIdx.x * a.path_cap;
    if (endpos >= 0) {
      const int2* arena = a.arena + (long long)slot * a.arena_cap;
      int k = st.cur_base + endpos;
      while (k >= 0) {
        const int2 e = arena[k];
        if (e.y < 0) break;
        if (n < a.path_cap) out[n] = e.y;
        n++;
        k = e.x;
      }
    }
    a.path_len[blockIdx.x] = n;
    a.end_cost[blockIdx.x] = endpos >= 0 ? funord((uint32_t)(bk >> 32)) : __int_as_float(0x7f800000);
    a.final_rel[blockIdx.x] = any_final ? bf - bn : __int_as_float(0x7f800000);
    a.end_state[blockIdx.x] = endpos >= 0 ? (int)(unsigned)(bk & 0xffffffffu) : -1;
  }
}

void LaunchTraceback(const TraceArgs& a, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(traceback_kernel, dim3(n), dim3(256), 0, s, a);
}

__global__ void init_keys_kernel(unsigned long long* key, int* stamp, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    key[i] = kEmpty;
    stamp[i] = -1;
  }
}

void LaunchInitKeys(unsigned long long* key, int* stamp, long long n, hipStream_t s) {
  if (n <= 0) return;
  long long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(init_keys_kernel, dim3((unsigned)blocks), dim3(256), 0, s, key, stamp, n);
}

}  // namespace vamd
