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
//   decode          one 512-thread workgroup per stream, persistent over the
//                   chunk's frames: exact max-active cutoff by LDS radix
//                   select, load-balanced (token, arc) expansion, 64-bit
//                   atomicMin token recombination, epsilon closure by rounds
//                   (Kaldi LatticeFasterDecoder [K]; src/recognizer.cc:39-43)
//   traceback       best-path end selection + backpointer walk
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdint>

#include "dev_util.h"
#include "engine_dev.h"
#include "kernels.h"

namespace vamd {

typedef float floatx16 __attribute__((ext_vector_type(16)));


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

// one block per job, one thread per output sample (taps ~ 12-40)
__global__ __launch_bounds__(256) void resample_kernel(const ResampleJob* jobs,
                                                       const ResampleDev* tables,
                                                       const float* raw, int raw_len, float* ring,
                                                       int ring_len) {
  const ResampleJob j = jobs[blockIdx.x];
  const ResampleDev t = tables[j.table];
  const float* src = raw + (size_t)j.slot * raw_len;
  float* dst = ring + (size_t)j.slot * ring_len;
  for (int i = threadIdx.x; i < j.count; i += blockDim.x) {
    const long long k = j.out_first + i;
    const long long unit = k / t.out_unit;
    const int ph = (int)(k - unit * t.out_unit);
    const long long first = t.first[ph] + unit * t.in_unit;
    const int nt = t.ntaps[ph];
    const float* w = t.w + (size_t)ph * t.taps;
    float acc = 0.0f;
    for (int q = 0; q < nt; q++) {
      const long long idx = first + q;
      if (idx < 0 || idx >= j.raw_total) continue;
      acc = __builtin_fmaf(w[q], src[idx & (raw_len - 1)], acc);
    }
    dst[(j.pos + i) & (ring_len - 1)] = acc;
  }
}

__global__ __launch_bounds__(256) void gather_copy_kernel(const CopyItem* items, unsigned* dst) {
  const CopyItem it = items[blockIdx.x];
  unsigned* d = dst + it.dst_off;
  for (long long i = threadIdx.x; i < it.nwords; i += blockDim.x) d[i] = it.src[i];
}

void LaunchGatherCopy(const CopyItem* items, int nitems, unsigned* dst, hipStream_t s) {
  if (nitems <= 0) return;
  hipLaunchKernelGGL(gather_copy_kernel, dim3(nitems), dim3(256), 0, s, items, dst);
}

void LaunchResample(const ResampleJob* jobs, int njobs, const ResampleDev* tables, const float* raw,
                    int raw_len, float* ring, int ring_len, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(resample_kernel, dim3(njobs), dim3(256), 0, s, jobs, tables, raw, raw_len,
                     ring, ring_len);
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
  const long long s0 = (long long)frame * m.frame_shift + m.first_offset;
  for (int i = lane; i < L; i += 64) {
    long long k = s0 + i;
    if (k < 0) k = -k - 1;  // Kaldi ExtractWindow reflection (snip-edges=false)
    x[i] = valid ? src[k & (ring_len - 1)] : 0.0f;
  }
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
        if (m.fbank && !m.use_power) pw = sqrtf(pw);
        e = __builtin_fmaf(wrow[i], pw, e);
      }
    if (!(m.fbank && !m.use_log_fbank)) {
      if (e < 1.1920929e-07f) e = 1.1920929e-07f;
      e = dev_logf(e);
    }
    MEL[w][lane] = e;
  }
  __syncthreads();
  float* dst = m.out + ((size_t)(frame & rings.mask) * rings.slots + slot) * m.feat_dim;
  if (m.fbank) {  // [log energy,] log mel energies
    const int off = m.use_energy ? 1 : 0;
    if (valid && lane < m.num_bins) dst[off + lane] = MEL[w][lane];
    if (valid && m.use_energy && lane == 0) dst[0] = SC[w][1];
  } else if (valid && lane < m.num_ceps) {
    float c = 0.0f;
    const float* drow = m.dct + (size_t)lane * m.num_bins;
    for (int j = 0; j < m.num_bins; j++) c = __builtin_fmaf(drow[j], MEL[w][j], c);
    float out = c * m.lifter[lane];
    if (m.use_energy && lane == 0) out = SC[w][1];
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
__device__ __forceinline__ const float* ring_at(const float* base, int ldim, int is_input,
                                               const RingSet& r, int slot, int tau, int clamp_max) {
  if (is_input) {
    if (tau < 0) tau = 0;
    if (tau > clamp_max) tau = clamp_max;
  }
  return base + ((size_t)(tau & r.mask) * r.slots + slot) * ldim;
}

__device__ __forceinline__ float apply_stages(const NnetOpArgs& a, float x, int col, int slot,
                                              int tau, int clamp_max) {
  for (int s = 0; s < a.nstages; s++) {
    const DevStage& st = a.stages[s];
    switch (st.kind) {
      case 0: x = x + st.v0[col]; break;                       // bias
      case 1: x = x < 0.0f ? 0.0f : x; break;                  // ReLU
      case 2: x = x * st.v0[col] + st.v1[col]; break;          // BN / scale+offset
      case 3: {                                                // bypass Sum()
        float z = ring_at(st.base, st.ldim, st.is_input, a.rings, slot, tau + st.offset,
                          clamp_max)[st.src_col + col];
        x = st.scaled ? (st.c * z) + x : z + x;
        break;
      }
      case 5: x = col >= st.src_col ? x * x : x; break;       // square (i-vector UBM input)
      default: x = x * st.c; break;                            // scale
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
    float* dst = a.out_base + ((size_t)(tau & a.rings.mask) * a.rings.slots + slot) * a.out_ldim;
    dst[col] = v;
  }
}

// Epilogue for the 16 accumulator values a lane holds for one column of a
// 32x32 MFMA block: tile rows lr0 + (j&3) + 8*(j>>2).  Stages run outermost
// (uniform branches), per-column stage vectors are loaded once per lane, the
// bypass rows are fetched as one batch of independent loads, and all stores
// come after all loads.  Per element the arithmetic is exactly apply_stages'.
template <int TMR>
__device__ __forceinline__ void epilogue_16(const NnetOpArgs& a, float (&v)[16], int col, int m0,
                                            int lr0, const int (*Rinfo)[TMR]) {
  const bool cok = col < a.N;
  const int cc = cok ? col : 0;
  for (int s = 0; s < a.nstages; s++) {
    const DevStage& st = a.stages[s];
    const int kind = st.kind;
    if (kind == 0) {
      const float b = st.v0[cc];
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = v[j] + b;
    } else if (kind == 1) {
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = v[j] < 0.0f ? 0.0f : v[j];
    } else if (kind == 2) {
      const float m = st.v0[cc], c = st.v1[cc];
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = v[j] * m + c;
    } else if (kind == 3) {
      float z[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int lr = lr0 + (j & 3) + 8 * (j >> 2);
        z[j] = 0.0f;
        if (cok && m0 + lr < a.M)
          z[j] = ring_at(st.base, st.ldim, st.is_input, a.rings, Rinfo[0][lr],
                         Rinfo[1][lr] + st.offset, Rinfo[2][lr])[st.src_col + col];
      }
      if (st.scaled) {
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = (st.c * z[j]) + v[j];
      } else {
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = z[j] + v[j];
      }
    } else if (kind == 5) {
      if (col >= st.src_col) {
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = v[j] * v[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; j++) v[j] = v[j] * st.c;
    }
  }
  if (!cok) return;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int lr = lr0 + (j & 3) + 8 * (j >> 2);
    if (m0 + lr < a.M) store_out(a, m0 + lr, col, Rinfo[0][lr], Rinfo[1][lr], v[j]);
  }
}

// ---- nnet GEMMs.  Canonical dot-product order (shared with oracle.c): K is
// cut into GemmKSlices(K) slices whose sums are added left to right; inside a
// slice the fma chain starts from 0 and visits each aligned group of eight k
// as (0,4),(1,5),(2,6),(3,7): lane half h of a 32x32x2 MFMA holds k+4h..k+4h+3
// of a group as one float4, and MFMA j consumes component j (lanes 0-31 give
// the first k of the pair).

// Streaming kernel: one wave per K-slice of a 32 x (32*NB) output block, so a
// workgroup is GemmKSlices(K) waves.  No LDS staging and no barriers in the
// main loop: each lane streams its own A row and B rows as float4 groups
// straight into registers through a D-deep prefetch ring (L2 serves the
// reuse of W across blocks).  Slice partials are summed in LDS in slice
// order by wave 0, which runs the fused epilogue.
// Requirements (checked on the host): K/slices % (8*D) == 0, segment
// boundaries multiples of 8.
template <int NB, int KS>
__global__ __launch_bounds__(64 * KS) void nnet_gemm_stream_kernel(NnetOpArgs a) {
  // prefetch depth in groups of 8 k; kept shallow for NB = 3 so that a wave
  // fits beside the decoder's waves on a SIMD (pipeline mode)
  constexpr int D = NB >= 3 ? 2 : 4;
  __shared__ int Rinfo[3][32];
  __shared__ float Red[KS > 1 ? (KS - 1) * NB * 1024 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * (32 * NB);
  int slot = 0, tau = 0, clamp = 0;
  if (m0 + r < a.M) row_info(a, m0 + r, &slot, &tau, &clamp);
  if (tid < 32) {
    Rinfo[0][tid] = slot;
    Rinfo[1][tid] = tau;
    Rinfo[2][tid] = clamp;
  }
  const int kw = a.K / KS, kbeg = wave * kw, ngr = kw / 8;
  const float* bp[NB];
#pragma unroll
  for (int b = 0; b < NB; b++) {
    int n = n0 + b * 32 + r;
    n = n < a.N ? n : a.N - 1;  // columns past N are computed but never stored
    bp[b] = a.W + (size_t)n * a.K + kbeg + 4 * h;
  }
  int seg = 0;
  while (kbeg >= a.segs[seg].col0 + a.segs[seg].dim) seg++;
  int kl = kbeg, seg_end;
  const float* ap;
  auto seg_ptr = [&]() {
    const DevSeg& S = a.segs[seg];
    seg_end = S.col0 + S.dim;
    ap = ring_at(S.base, S.ldim, S.is_input, a.rings, slot, tau + S.offset, clamp) + S.src_col +
         (kl - S.col0) + 4 * h;
  };
  seg_ptr();
  float4 ra[D], rb[D][NB];
  auto load = [&](int d) {
    if (kl >= seg_end) {  // wave-uniform
      seg++;
      seg_ptr();
    }
    ra[d] = *reinterpret_cast<const float4*>(ap);
    ap += 8;
    kl += 8;
#pragma unroll
    for (int b = 0; b < NB; b++) {
      rb[d][b] = *reinterpret_cast<const float4*>(bp[b]);
      bp[b] += 8;
    }
  };
  floatx16 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc[b][i] = 0.0f;
#pragma unroll
  for (int d = 0; d < D; d++) load(d);
  for (int g = 0; g < ngr; g += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d].x, rb[d][b].x, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d].y, rb[d][b].y, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d].z, rb[d][b].z, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d].w, rb[d][b].w, acc[b], 0, 0, 0);
      if (g + d + D < ngr) load(d);
    }
  }
  float v[NB][16];
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int j = 0; j < 16; j++) v[b][j] = acc[b][j];
  if (KS > 1) {
    if (wave > 0) {
#pragma unroll
      for (int b = 0; b < NB; b++)
#pragma unroll
        for (int j = 0; j < 16; j++) Red[((wave - 1) * NB + b) * 1024 + j * 64 + lane] = v[b][j];
    }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll 1
    for (int z = 1; z < KS; z++)
#pragma unroll
      for (int b = 0; b < NB; b++)
#pragma unroll
        for (int j = 0; j < 16; j++)
          v[b][j] = v[b][j] + Red[((z - 1) * NB + b) * 1024 + j * 64 + lane];
  } else {
    __syncthreads();
  }
#pragma unroll
  for (int b = 0; b < NB; b++) epilogue_16(a, v[b], n0 + b * 32 + r, m0, 4 * h, Rinfo);
}

// LDS-staged kernel: output tile (32*WM) x (32*NB) per workgroup of WM waves,
// each wave owning 32 rows x 32*NB columns (NB accumulators sharing one A
// fragment).  A and B are staged row-major in k with row stride BK+4: one
// ds_read_b128 per operand feeds four MFMAs, conflict-free in the b128 lane
// groups.  Register prefetch one K-step ahead; loads are unconditional (rows
// past M / columns past N read valid memory and are never stored) so no
// divergent branch pins a wait next to a load.  kslices must be 1.
template <int BK, int WM, int NB>
__global__ __launch_bounds__(64 * WM) void nnet_gemm_lds_kernel(NnetOpArgs a) {
  constexpr int TM = 32 * WM, TN = 32 * NB, NT = 64 * WM;
  constexpr int Q = BK / 4, LDA = BK + 4;
  constexpr int NLA = (TM * Q + NT - 1) / NT, NLB = (TN * Q + NT - 1) / NT;
  __shared__ float4 As4[2][TM * LDA / 4];
  __shared__ float4 Bs4[2][TN * LDA / 4];
  __shared__ int Rinfo[3][TM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  if (tid < TM) {
    int sl = 0, ta = 0, cl = 0;
    if (m0 + tid < a.M) row_info(a, m0 + tid, &sl, &ta, &cl);
    Rinfo[0][tid] = sl;
    Rinfo[1][tid] = ta;
    Rinfo[2][tid] = cl;
  }
  __syncthreads();
  int r_slot[NLA], r_tau[NLA], r_clamp[NLA];
#pragma unroll
  for (int v = 0; v < NLA; v++) {
    const int idx = tid + v * NT, row = (idx / Q) % TM;
    r_slot[v] = Rinfo[0][row];
    r_tau[v] = Rinfo[1][row];
    r_clamp[v] = Rinfo[2][row];
  }
  float4 ra[NLA], rb[NLB];
  int seg = 0;
  auto load = [&](int k0) {
    while (!(k0 >= a.segs[seg].col0 && k0 < a.segs[seg].col0 + a.segs[seg].dim)) seg++;
    const DevSeg S = a.segs[seg];
#pragma unroll
    for (int v = 0; v < NLA; v++) {
      const int idx = tid + v * NT, q = idx % Q;
      const float* p = ring_at(S.base, S.ldim, S.is_input, a.rings, r_slot[v],
                               r_tau[v] + S.offset, r_clamp[v]);
      ra[v] = *reinterpret_cast<const float4*>(p + S.src_col + (k0 - S.col0) + 4 * q);
    }
#pragma unroll
    for (int v = 0; v < NLB; v++) {
      const int idx = tid + v * NT, q = idx % Q;
      int n = n0 + (idx / Q) % TN;
      n = n < a.N ? n : a.N - 1;
      rb[v] = *reinterpret_cast<const float4*>(a.W + (size_t)n * a.K + k0 + 4 * q);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NLA; v++) {
      const int idx = tid + v * NT, row = idx / Q, q = idx - row * Q;
      if (NLA * NT == TM * Q || idx < TM * Q) As4[buf][(row * LDA) / 4 + q] = ra[v];
    }
#pragma unroll
    for (int v = 0; v < NLB; v++) {
      const int idx = tid + v * NT, n = idx / Q, q = idx - n * Q;
      if (NLB * NT == TN * Q || idx < TN * Q) Bs4[buf][(n * LDA) / 4 + q] = rb[v];
    }
  };
  floatx16 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc[b][i] = 0.0f;
  const int nk = a.K / BK;
  const int r32 = lane & 31, h = lane >> 5;
  const int aoff = ((wave * 32 + r32) * LDA) / 4 + h, boff = (r32 * LDA) / 4 + h;
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ks++) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load((ks + 1) * BK);
#pragma unroll
    for (int g = 0; g < BK / 4; g += 2) {
      const float4 av = As4[buf][aoff + g];
      float4 bv[NB];
#pragma unroll
      for (int b = 0; b < NB; b++) bv[b] = Bs4[buf][boff + b * 8 * LDA + g];
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[b].x, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[b].y, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[b].z, acc[b], 0, 0, 0);
#pragma unroll
      for (int b = 0; b < NB; b++)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[b].w, acc[b], 0, 0, 0);
    }
    if (ks + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  float v[NB][16];
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int j = 0; j < 16; j++) v[b][j] = acc[b][j];
#pragma unroll
  for (int b = 0; b < NB; b++)
    epilogue_16(a, v[b], n0 + b * 32 + r32, m0, wave * 32 + 4 * h, Rinfo);
}

int g_gemm_variant = 0;  // development override (tools/gemm_bench): 0 = default

template <int BK, int WM, int NB>
static void LaunchLds(const NnetOpArgs& a, hipStream_t s) {
  dim3 grid((a.M + 32 * WM - 1) / (32 * WM), (a.N + 32 * NB - 1) / (32 * NB));
  hipLaunchKernelGGL((nnet_gemm_lds_kernel<BK, WM, NB>), grid, dim3(64 * WM), 0, s, a);
}

template <int NB>
static void LaunchStream(const NnetOpArgs& a, hipStream_t s) {
  dim3 grid((a.M + 31) / 32, (a.N + 32 * NB - 1) / (32 * NB));
  switch (a.kslices) {
    case 1: hipLaunchKernelGGL((nnet_gemm_stream_kernel<NB, 1>), grid, dim3(64), 0, s, a); break;
    case 2: hipLaunchKernelGGL((nnet_gemm_stream_kernel<NB, 2>), grid, dim3(128), 0, s, a); break;
    case 4: hipLaunchKernelGGL((nnet_gemm_stream_kernel<NB, 4>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((nnet_gemm_stream_kernel<NB, 8>), grid, dim3(512), 0, s, a); break;
  }
}

bool GemmStreamable(const NnetOpArgs& a) {
  if (a.kslices != 1 && a.kslices != 2 && a.kslices != 4 && a.kslices != 8) return false;
  if ((a.K / a.kslices) % 32) return false;
  for (int i = 0; i < a.nsegs; i++)
    if (a.segs[i].col0 % 8 || a.segs[i].dim % 8) return false;
  return true;
}

void LaunchNnetGemm(const NnetOpArgs& a, int bk, hipStream_t s) {
  if (a.M <= 0) return;
  const int nb = GemmTileN(a.N) / 32;
  int var = g_gemm_variant;
  // streaming kernel wherever it applies: faster on every recipe shape and
  // small in LDS (co-resides with the decoder in pipeline mode)
  if (var == 0) var = GemmStreamable(a) ? 1 : 3;
  if ((var == 1 || var == 2) && !GemmStreamable(a)) var = 3;
  if (var == 1) {
    // small grids: one 32-column block per wave (3x / 2x the waves, more of
    // the chip busy) beats the wider tile's operand reuse
    const long long waves = (long long)((a.M + 31) / 32) * ((a.N + 32 * nb - 1) / (32 * nb)) * a.kslices;
    static const int nb1_waves = getenv("VOSK_AMD_NB1_WAVES") ? atoi(getenv("VOSK_AMD_NB1_WAVES")) : 4000;
    if (waves < nb1_waves && g_gemm_variant == 0) LaunchStream<1>(a, s);
    else if (nb == 3) LaunchStream<3>(a, s);
    else LaunchStream<2>(a, s);
  } else if (var == 2) {
    LaunchStream<1>(a, s);
  } else {
    if (a.kslices != 1) return;  // host guarantees streamable ops for split K
    if (bk >= 32) {
      if (nb == 3) LaunchLds<32, 2, 3>(a, s);
      else LaunchLds<32, 4, 2>(a, s);
    } else if (bk == 16) {
      if (nb == 3) LaunchLds<16, 2, 3>(a, s);
      else LaunchLds<16, 4, 2>(a, s);
    } else {
      if (nb == 3) LaunchLds<8, 2, 3>(a, s);
      else LaunchLds<8, 4, 2>(a, s);
    }
  }
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
    if (in.op == 0)
      stack[sp++] = ring_at(in.base, in.ldim, in.is_input, a.rings, slot, tau + in.offset,
                            clamp)[in.src_col + d];
    else if (in.op == 1) stack[sp - 1] = in.c * stack[sp - 1];
    else if (in.op == 2) { stack[sp - 2] = stack[sp - 2] + stack[sp - 1]; sp--; }
    else if (in.op == 3) stack[sp++] = in.c;
    else stack[sp++] = in.base[(size_t)(row / a.P) * in.ldim + in.src_col + d];  // job's i-vector
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
// Online i-vector extraction: Kaldi OnlineIvectorFeature semantics, operation
// for operation as the restatement in oracle/oracle.c orc_ivector_extract
// (double statistics, fixed summation orders), so the result is
// bit-identical.  Per step:
//   cmvn_kernel           per stream: online CMVN of the new frames
//                         (running double sums, sequential in time) into a
//                         ring laid out like the MFCC ring
//   3 GEMM launches       (engine.cc, the nnet GEMM kernels) over blocks of
//                         frames: LDA of the spliced normalized frames -> [x |
//                         x*x], LDA of the raw frames, UBM log-likelihoods
//   ivector_top_kernel    one wave per frame: 5-best Gaussians, posteriors
//   ivector_acc_kernel    Kaldi's per-frame OnlineIvectorEstimationStats
//                         updates, XCD-partitioned, frames in order
//   ivector_cg_kernel     one workgroup per stream: warm-started CG per request

__device__ float dev_expf(float x) {  // oracle.c orc_expf
  if (x < -87.0f) return 0.0f;
  const float k = rintf(x * 1.44269504f);
  float r = fmaf(-k, 0.693145752f, x);
  r = fmaf(-k, 1.42860677e-6f, r);
  float p = 1.98412698e-4f;
  p = fmaf(p, r, 1.38888889e-3f);
  p = fmaf(p, r, 8.33333333e-3f);
  p = fmaf(p, r, 4.16666667e-2f);
  p = fmaf(p, r, 1.66666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, (int)k);
}

__device__ __forceinline__ const float* iv_raw(const IvArgs& a, int slot, int u) {
  return a.in_base + ((size_t)(u & a.in_mask) * a.slots + slot) * a.m.feat_dim;
}

// Online CMVN with global stats (Kaldi OnlineCmvn::GetFrame: the window sums
// of ComputeStatsForFrame, SmoothOnlineCmvnStats, ApplyCmvn without variance
// normalization), as oracle.c orc_online_cmvn: one lane per dimension walks
// the stream's new frames in order.  Used on the nnet input (global_cmvn.stats)
// and inside the i-vector extractor.
__global__ __launch_bounds__(128) void cmvn_kernel(CmvnDev c, const CmvnJob* jobs) {
  const CmvnJob J = jobs[blockIdx.x];
  const int d = threadIdx.x, D = c.D, W = c.window, slot = J.slot;
  if (d >= D) return;
  float* hist = c.hist + (size_t)slot * kCmvnHist * D;
  double csum = J.reset ? 0.0 : c.sums[(size_t)slot * D + d];
  const double gcount = c.gstats[D], gmean = c.gstats[d];
  auto in_row = [&](int u) { return c.in_base + ((size_t)(u & c.mask) * c.slots + slot) * D; };
  // blocks of 16 frames, all loads first (window >= 16: no frame leaving the
  // window is stored in the same block)
  for (int u0 = J.from; u0 < J.to; u0 += 16) {
    float xn[16], xo[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int u = u0 + k;
      xn[k] = u < J.to ? in_row(u)[d] : 0.0f;
      xo[k] = (u < J.to && u - W >= 0) ? hist[(size_t)((u - W) % kCmvnHist) * D + d] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int u = u0 + k;
      if (u >= J.to) break;
      const float x = xn[k];
      csum = csum + (double)x;
      hist[(size_t)(u % kCmvnHist) * D + d] = x;
      if (u - W >= 0) csum = csum - (double)xo[k];
      double cnt = (double)min(u + 1, W), stv = csum;
      if (cnt < W) {
        double cgf = W - cnt;
        if (cgf > c.global_frames) cgf = c.global_frames;
        const double scl = cgf / gcount;
        stv = stv + scl * gmean;
        cnt = cnt + scl * gcount;
      }
      const float alpha = (float)(-1.0 / cnt);
      const float off = (float)((double)alpha * stv);
      c.out_base[((size_t)(u & c.mask) * c.slots + slot) * D + d] = x + off;
    }
  }
  c.sums[(size_t)slot * D + d] = csum;
}

// Max of a 64-bit key over the wave: DPP butterflies inside each 16-lane row
// (quad_perm 1,0,3,2 / 2,3,0,1, half-row and row mirrors), then the four
// row results combined through readlane.
__device__ __forceinline__ unsigned long long iv_dpp_step(unsigned long long v, int ctrl_id) {
  int lo = (int)(unsigned)v, hi = (int)(unsigned)(v >> 32), lo2, hi2;
  switch (ctrl_id) {
    case 0:
      lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0xB1, 0xF, 0xF, false);
      hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0xB1, 0xF, 0xF, false);
      break;
    case 1:
      lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x4E, 0xF, 0xF, false);
      hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x4E, 0xF, 0xF, false);
      break;
    case 2:
      lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x141, 0xF, 0xF, false);
      hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x141, 0xF, 0xF, false);
      break;
    default:
      lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x140, 0xF, 0xF, false);
      hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x140, 0xF, 0xF, false);
      break;
  }
  const unsigned long long w = ((unsigned long long)(unsigned)hi2 << 32) | (unsigned)lo2;
  return w > v ? w : v;
}
__device__ __forceinline__ unsigned long long iv_wave_max_u64(unsigned long long v) {
  v = iv_dpp_step(v, 0);
  v = iv_dpp_step(v, 1);
  v = iv_dpp_step(v, 2);
  v = iv_dpp_step(v, 3);
  unsigned long long r = 0;
#pragma unroll
  for (int row = 0; row < 4; row++) {
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, row * 16);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), row * 16);
    const unsigned long long x = ((unsigned long long)hi << 32) | lo;
    r = x > r ? x : r;
  }
  return r;
}

// 5-best Gaussians (descending, ties to the lower index) and posteriors of
// each frame: one wave per frame over the UBM GEMM's log-likelihood row.
__global__ __launch_bounds__(256) void ivector_top_kernel(IvArgs a, const float* ll, int M) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= M) return;
  const IvFrameBlock B = a.blocks[r / kIvFrameBlock];
  const int k0 = r % kIvFrameBlock;
  if (k0 >= B.nf) {  // padding row of the block: an empty record
    if (lane == 0) a.frames[r].nsel = 0;
    return;
  }
  const IvectorDev& m = a.m;
  const int G = m.num_gauss;
  const float* row = ll + (size_t)r * G;
  unsigned long long key[kIvMaxG / 64];
#pragma unroll
  for (int i = 0; i < kIvMaxG / 64; i++) {
    const int g = lane + 64 * i;
    float v = g < G ? row[g] : 0.0f;
    v = v == 0.0f ? 0.0f : v;  // -0 ties with +0 as in a float comparison
    key[i] = g < G ? ((unsigned long long)ford(v) << 32) | (0xFFFFFFFFu - (unsigned)g) : 0ull;
  }
  int chosen[5];
  float val[5];
  unsigned used = 0;
  const int ng = min(m.num_gselect, G);
  for (int kk = 0; kk < ng; kk++) {
    unsigned long long b = 0;
#pragma unroll
    for (int i = 0; i < kIvMaxG / 64; i++)
      if (!((used >> i) & 1) && key[i] > b) b = key[i];
    b = iv_wave_max_u64(b);
    const int g = (int)(0xFFFFFFFFu - (unsigned)b);
    chosen[kk] = g;
    val[kk] = row[g];
    if ((g & 63) == lane) used |= 1u << (g >> 6);
  }
  if (lane == 0) {
    int ns = ng;
    while (ns > 1 && val[ns - 1] < val[0] + m.log_min_post) ns--;
    float e[5], tot = 0.0f;
    for (int k = 0; k < ns; k++) {
      e[k] = dev_expf(val[k] - val[0]);
      tot = tot + e[k];
    }
    IvFrame& F = a.frames[r];
    F.nsel = ns;
    F.xrow = r;
    for (int k = 0; k < ns; k++) {
      F.sel[k] = chosen[k];
      F.post[k] = (e[k] / tot) * (m.posterior_scale * 1.0f);
    }
    if (B.ring >= 0) {  // history record: posteriors before the frame weight
      IvFrame& H = a.ring[B.ring + (B.t0 + k0) % kIvRing];
      H.nsel = ns;
      H.xrow = B.t0 + k0;
      for (int k = 0; k < ns; k++) {
        H.sel[k] = chosen[k];
        H.post[k] = e[k] / tot;
      }
    }
  }
  if (B.ring >= 0 && lane < m.lda_dim)
    a.ring_x[(size_t)(B.ring + (B.t0 + k0) % kIvRing) * m.lda_dim + lane] = a.xraw[(size_t)r * m.lda_dim + lane];
}

// Silence-weighted entries (OnlineIvectorFeature::UpdateStatsForFrames with
// delta weights): the record of each entry's frame from the history ring,
// posteriors scaled by posterior_scale * weight as Kaldi does
// (`posterior[j].second *= info_.posterior_scale * weight`), into the rows
// the statistics kernels read.  One wave per entry.
__global__ __launch_bounds__(256) void ivector_entry_kernel(IvArgs a) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= a.nents) return;
  const IvEntry E = a.ents[e];
  const int row = a.ent_row0 + e, DL = a.m.lda_dim;
  if (lane == 0) {
    const IvFrame H = a.ring[E.rec];
    IvFrame F;
    F.nsel = H.nsel;
    F.xrow = row;
    for (int k = 0; k < 5; k++) {
      F.sel[k] = k < H.nsel ? H.sel[k] : 0;
      F.post[k] = k < H.nsel ? H.post[k] * (a.m.posterior_scale * E.w) : 0.0f;
    }
    a.frames[row] = F;
  }
  if (lane < DL) a.xraw[(size_t)row * DL + lane] = a.ring_x[(size_t)E.rec * DL + lane];
}

__device__ __forceinline__ int iv_tri_row(int e) {  // packed lower-triangle row of entry e
  int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= e) i++;
  while (i * (i + 1) / 2 > e) i--;
  return i;
}

constexpr int kIvCgLds = 48;  // S up to this: the CG matrix lives in LDS

// i-vector statistics, batched as Kaldi's OnlineIvectorFeature::
// UpdateStatsForFrames -> OnlineIvectorEstimationStats::AccStats over a
// matrix of frames: per batch, zeroth / first order statistics per Gaussian
// (gamma_g, X_g = sum post * x in frame order), then per Gaussian in
// ascending index linear += SigmaInvM_g^T X_g and quadratic += gamma_g U_g,
// then the frame count and the max-count prior rescaling once per batch
// (oracle.c iv_accumulate_batch restates it).  NP workgroups per stream: part
// p owns a contiguous 1/NP of the packed quadratic term and of the linear
// columns (blocks b and b + 8 share an XCD, so each XCD's L2 holds only its
// slice of U and SigmaInvM); the per-Gaussian aggregation is recomputed by
// every part (identical).  A snapshot of the terms is taken at every request
// for the CG kernel.
constexpr int kIvGroup = 16;  // Gaussians whose X_g are held in LDS at a time
struct IvAccShared {
  unsigned short sel[kIvBatchRows][5];
  float post[kIvBatchRows][5];
  unsigned char ns[kIvBatchRows];
  int cnt[kIvMaxG], off[kIvMaxG], run[kIvMaxG];
  unsigned short dlist[kIvMaxG];
  unsigned short occ[kIvBatchRows * 5];  // row * 5 + k, grouped by Gaussian, rows ascending
  int ndist;
  int wsum[4];
  double X[kIvGroup][kIvMaxD];
  double gam[kIvGroup];
  double proj[kIvGroup][(kIvMaxS + 3) / 4];
  double tw;
};

template <int NQP, int NP>  // NP parts; packed quad entries per thread: ceil(ceil(QS / NP) / 256)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void ivector_acc_kernel(IvArgs a) {
  __shared__ IvAccShared sh;
  const int part = blockIdx.x % NP, jb = blockIdx.x / NP, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const IvStreamJob J = a.jobs[jb];
  const IvectorDev& m = a.m;
  const int S = m.ivec_dim, DL = m.lda_dim, QS = S * (S + 1) / 2, NE = QS + S, G = m.num_gauss;
  const int qchunk = (QS + NP - 1) / NP, q0 = part * qchunk, q1 = min(QS, q0 + qchunk);
  const int cw = (S + NP - 1) / NP, c0 = min(S, part * cw), ncol = min(S, c0 + cw) - c0;  // columns [c0, c0+ncol)
  IvState* st = a.state + J.slot;
  double* quad = a.quad + (size_t)J.slot * QS;
  const double po = m.prior_offset, mc = m.max_count;
  double qe[NQP];
  bool qd[NQP];
#pragma unroll
  for (int j = 0; j < NQP; j++) {
    const int e = q0 + tid + 256 * j, i = iv_tri_row(e);
    qd[j] = e == i * (i + 1) / 2 + i;
    qe[j] = e < q1 ? (J.reset ? (qd[j] ? 1.0 : 0.0) : quad[e]) : 0.0;
  }
  const int col = c0 + tid;  // lin column owned by threads tid < ncol
  double lin = 0.0;
  if (tid < ncol) lin = J.reset ? (col == 0 ? po : 0.0) : st->lin[col];
  double nfr = J.reset ? 0.0 : st->nfr;
  for (int q = 0; q < J.nreq; q++) {
    const IvReq R = a.reqs[J.req0 + q];
    for (int bi = 0; bi < R.nbatch; bi++) {
      const IvBatch B = a.batches[R.batch0 + bi];
      const int n = B.row_to - B.row_from;
      __syncthreads();  // previous batch done with the shared arrays
      for (int i = tid; i < n; i += 256) {
        const IvFrame F = a.frames[B.row_from + i];
        sh.ns[i] = (unsigned char)F.nsel;
#pragma unroll
        for (int k = 0; k < 5; k++) {
          sh.sel[i][k] = (unsigned short)(k < F.nsel ? F.sel[k] : 0);
          sh.post[i][k] = k < F.nsel ? F.post[k] : 0.0f;
        }
      }
      for (int g = tid; g < G; g += 256) {
        sh.cnt[g] = 0;
        sh.run[g] = 0;
      }
      __syncthreads();
      // per-Gaussian occurrence counts (zero posteriors contribute nothing)
      for (int i = tid; i < n * 5; i += 256) {
        const int r = i / 5, k = i - r * 5;
        if (k < sh.ns[r] && sh.post[r][k] != 0.0f) atomicAdd(&sh.cnt[sh.sel[r][k]], 1);
      }
      __syncthreads();
      // exclusive scan of the counts (two per thread, G <= 512) and the
      // ascending list of Gaussians present
      {
        const int g0 = 2 * tid;
        const int c_a = g0 < G ? sh.cnt[g0] : 0, c_b = g0 + 1 < G ? sh.cnt[g0 + 1] : 0;
        int v = c_a + c_b, d_v = (c_a > 0) + (c_b > 0);
        int incl = v, dincl = d_v;
        for (int o = 1; o < 64; o <<= 1) {
          const int u = __shfl_up(incl, o, 64), du = __shfl_up(dincl, o, 64);
          if (lane >= o) {
            incl += u;
            dincl += du;
          }
        }
        if (lane == 63) sh.wsum[wv] = (incl & 0xffff) | (dincl << 16);
        __syncthreads();
        int base = 0, dbase = 0;
        for (int w = 0; w < wv; w++) {
          base += sh.wsum[w] & 0xffff;
          dbase += sh.wsum[w] >> 16;
        }
        const int ex = base + incl - v, dex = dbase + dincl - d_v;
        if (g0 < G) {
          sh.off[g0] = ex;
          if (c_a > 0) sh.dlist[dex] = (unsigned short)g0;
        }
        if (g0 + 1 < G) {
          sh.off[g0 + 1] = ex + c_a;
          if (c_b > 0) sh.dlist[dex + (c_a > 0)] = (unsigned short)(g0 + 1);
        }
        if (tid == 255) sh.ndist = dbase + dincl;
      }
      __syncthreads();
      // occurrence lists in row order: one thread per Gaussian present scans
      // the batch's (row, k) pairs in order (uniform LDS reads broadcast)
      {
        const int nd0 = sh.ndist;
        for (int di = tid; di < nd0 + 255 - (nd0 + 255) % 256; di += 256) {
          const int g = di < nd0 ? sh.dlist[di] : -1;
          int c = 0;
          const int o0 = g >= 0 ? sh.off[g] : 0;
          for (int r = 0; r < n; r++) {
            const int nsr = sh.ns[r];
#pragma unroll
            for (int k = 0; k < 5; k++)
              if (k < nsr && sh.sel[r][k] == g && sh.post[r][k] != 0.0f) sh.occ[o0 + c++] = (unsigned short)(r * 5 + k);
          }
        }
      }
      if (tid == 0) sh.tw = 0.0;
      __syncthreads();
      const int nd = sh.ndist;
      for (int gb = 0; gb < nd; gb += kIvGroup) {
        const int ng = min(kIvGroup, nd - gb);
        // X_g and gamma_g of the group, each summed over its rows in order
        for (int i = tid; i < ng * (DL + 1); i += 256) {
          const int gi = i / (DL + 1), d = i - gi * (DL + 1);
          const int g = sh.dlist[gb + gi], o0 = sh.off[g], oc = sh.cnt[g];
          double acc = 0.0;
          for (int ob = 0; ob < oc; ob += 8) {  // batches of 8 row loads in flight
            float xv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
              xv[u] = 1.0f;
              if (ob + u < oc && d < DL) {
                const int r = sh.occ[o0 + ob + u] / 5;
                xv[u] = a.xraw[(size_t)(B.row_from + r) * DL + d];
              }
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
              if (ob + u >= oc) break;
              const int rk = sh.occ[o0 + ob + u], r = rk / 5, k = rk - r * 5;
              const double p = (double)sh.post[r][k];
              acc = d < DL ? acc + p * (double)xv[u] : acc + p;
            }
          }
          if (d < DL) sh.X[gi][d] = acc;
          else sh.gam[gi] = acc;
        }
        __syncthreads();
        for (int gi = 0; gi < ng; gi++) {
          const int g = sh.dlist[gb + gi];
          const double gm = sh.gam[gi];
          const double* U = m.U + (size_t)g * QS;
#pragma unroll
          for (int j = 0; j < NQP; j++)
            if (q0 + tid + 256 * j < q1) qe[j] = qe[j] + gm * U[q0 + tid + 256 * j];
        }
        // SigmaInvM_g^T X_g for every (Gaussian, column) of the group in
        // parallel, then each column adds them in Gaussian order
        for (int i = tid; i < ng * ncol; i += 256) {
          const int gi = i / ncol, c = i - gi * ncol;
          const double* sm = m.sigma_inv_m + (size_t)sh.dlist[gb + gi] * DL * S + c0 + c;
          double acc = 0.0;
          for (int d0 = 0; d0 < DL; d0 += 20) {  // batches of 20 loads in flight
            double sv[20];
#pragma unroll
            for (int u = 0; u < 20; u++) sv[u] = d0 + u < DL ? sm[(size_t)(d0 + u) * S] : 0.0;
#pragma unroll
            for (int u = 0; u < 20; u++) {
              if (d0 + u >= DL) break;
              acc = fma(sv[u], sh.X[gi][d0 + u], acc);
            }
          }
          sh.proj[gi][c] = acc;
        }
        __syncthreads();
        if (tid < ncol)
          for (int gi = 0; gi < ng; gi++) lin = lin + sh.proj[gi][tid];
        if (tid == 0)
          for (int gi = 0; gi < ng; gi++) sh.tw = sh.tw + sh.gam[gi];
        __syncthreads();  // the group's X / gamma / projections are consumed
      }
      // frame count and Kaldi's max-count prior rescaling, once per batch
      const double tw = sh.tw, newn = nfr + tw;
      if (mc > 0.0 && (nfr > mc || newn > mc)) {  // else both scales are exactly 1
        const double oldp = (nfr > mc ? nfr : mc) / mc;
        const double newp = (newn > mc ? newn : mc) / mc;
        const double ch = newp - oldp;
        if (ch != 0.0) {
#pragma unroll
          for (int j = 0; j < NQP; j++)
            if (qd[j] && q0 + tid + 256 * j < q1) qe[j] += ch;
          if (tid < ncol && col == 0) lin = lin + po * ch;
        }
      }
      nfr = newn;
    }
    if (R.upd) {
      double* sn = a.snap + (size_t)(J.req0 + q) * NE;
#pragma unroll
      for (int j = 0; j < NQP; j++)
        if (q0 + tid + 256 * j < q1) sn[q0 + tid + 256 * j] = qe[j];
      if (tid < ncol) sn[QS + col] = lin;
    }
    if (part == 0 && tid == 0) a.snap_nfr[J.req0 + q] = nfr;
  }
#pragma unroll
  for (int j = 0; j < NQP; j++)
    if (q0 + tid + 256 * j < q1) quad[q0 + tid + 256 * j] = qe[j];
  if (tid < ncol) st->lin[col] = lin;
  if (part == 0 && tid == 0) st->nfr = nfr;
}

__device__ double iv_dot(const double* x, const double* y, int n) {
  double s = 0.0;
#pragma unroll 8
  for (int i = 0; i < n; i++) s = s + x[i] * y[i];
  return s;
}

// y = Q v over the full symmetric matrix (row j read as column: lanes coalesced)
__device__ void iv_matvec(const double* Qf, int S, const double* v, double* y) {
  const int i = threadIdx.x;
  if (i < S) {
    double acc = 0.0;
#pragma unroll 8
    for (int j = 0; j < S; j++) acc = acc + Qf[(size_t)j * S + i] * v[j];
    y[i] = acc;
  }
}

struct IvCgShared {
  double cg[5][kIvMaxS];  // x (= current i-vector), p, r, Ap, b
  double sc[4];
  double q[kIvCgLds * kIvCgLds];
};

// Warm-started conjugate gradient (Kaldi LinearCgd) per request, in order.
__global__ __launch_bounds__(128) void ivector_cg_kernel(IvArgs a) {
  __shared__ IvCgShared sh;
  const IvStreamJob J = a.jobs[blockIdx.x];
  const IvectorDev& m = a.m;
  const int tid = threadIdx.x, S = m.ivec_dim, QS = S * (S + 1) / 2, NE = QS + S;
  IvState* st = a.state + J.slot;
  double* qfull = S <= kIvCgLds ? sh.q : a.qfull + (size_t)J.slot * S * S;
  const double po = m.prior_offset;
  double *X = sh.cg[0], *P = sh.cg[1], *Rr = sh.cg[2], *AP = sh.cg[3], *Bv = sh.cg[4];
  if (tid < S) X[tid] = J.reset ? (tid == 0 ? po : 0.0) : st->cur[tid];
  for (int q = 0; q < J.nreq; q++) {
    const IvReq R = a.reqs[J.req0 + q];
    if (R.upd && !(a.snap_nfr[J.req0 + q] > 0.0)) {
      // IvectorEstimationStats::GetIvector with no (net) frames: the default
      if (tid < S) X[tid] = tid == 0 ? po : 0.0;
    } else if (R.upd) {
      const double* sn = a.snap + (size_t)(J.req0 + q) * NE;
      __syncthreads();
      for (int e = tid; e < QS; e += 128) {
        const int r = iv_tri_row(e), c = e - r * (r + 1) / 2;
        const double v = sn[e];
        qfull[(size_t)r * S + c] = v;
        qfull[(size_t)c * S + r] = v;
      }
      if (tid < S) Bv[tid] = sn[QS + tid];
      __syncthreads();
      iv_matvec(qfull, S, X, AP);
      __syncthreads();
      if (tid < S) {
        P[tid] = Bv[tid] - AP[tid];
        Rr[tid] = -P[tid];
      }
      __syncthreads();
      if (tid == 0) sh.sc[0] = iv_dot(Rr, Rr, S);
      __syncthreads();
      double rcur = sh.sc[0], rrec = rcur;
      for (int k = 0; k < S + 5 && k != m.num_cg_iters; k++) {
        iv_matvec(qfull, S, P, AP);
        __syncthreads();
        if (tid == 0) sh.sc[1] = -iv_dot(P, Rr, S) / iv_dot(P, AP, S);
        __syncthreads();
        const double alpha = sh.sc[1];
        if (tid < S) {
          X[tid] = X[tid] + alpha * P[tid];
          Rr[tid] = Rr[tid] + alpha * AP[tid];
        }
        __syncthreads();
        if (tid == 0) sh.sc[2] = iv_dot(Rr, Rr, S);
        __syncthreads();
        double rnext = sh.sc[2];
        if (rnext < 1e-4 * rrec || rnext > 1e4 * rrec) {
          iv_matvec(qfull, S, X, AP);
          __syncthreads();
          if (tid < S) Rr[tid] = AP[tid] - Bv[tid];
          __syncthreads();
          if (tid == 0) sh.sc[3] = iv_dot(Rr, Rr, S);
          __syncthreads();
          rnext = sh.sc[3];
          rrec = rnext;
        }
        if (rnext <= 2.2250738585072014e-308) break;
        const double beta = rnext / rcur;
        if (tid < S) P[tid] = beta * P[tid] - Rr[tid];
        __syncthreads();
        rcur = rnext;
      }
    }
    __syncthreads();
    // i-vector rows of the request's chunk jobs (prior offset removed)
    for (int i = tid; i < (R.job_hi - R.job_lo) * S; i += 128) {
      const int r = R.job_lo + i / S, c = i % S;
      float v = (float)X[c];
      if (c == 0) v = v - (float)po;
      a.ivec[(size_t)r * S + c] = v;
    }
  }
  if (tid < S) st->cur[tid] = X[tid];
}

void LaunchCmvn(const CmvnDev& c, const CmvnJob* jobs, int njobs, hipStream_t s) {
  if (njobs > 0) hipLaunchKernelGGL(cmvn_kernel, dim3(njobs), dim3(128), 0, s, c, jobs);
}

void LaunchIvectorStats(const IvArgs& a, const float* ll, int rows, int njobs, hipStream_t s) {
  if (njobs <= 0) return;
  if (rows > 0) hipLaunchKernelGGL(ivector_top_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, a, ll, rows);
  if (a.nents > 0) hipLaunchKernelGGL(ivector_entry_kernel, dim3((a.nents + 3) / 4), dim3(256), 0, s, a);
  // parts: blocks b and b + 8 share an XCD, so part = b % NP keeps each XCD's
  // L2 on 1/NP of U and SigmaInvM
  // (VOSK_AMD_IV_PARTS: 2, 4 or 8; the per-part linear-term columns must fit
  // IvAccShared::proj, ceil(S / parts) <= 25)
  static const int np_env = getenv("VOSK_AMD_IV_PARTS") ? atoi(getenv("VOSK_AMD_IV_PARTS")) : 4;
  const int S = a.m.ivec_dim, QS = S * (S + 1) / 2;
  const int np = (np_env == 8 || (np_env == 2 && (S + 1) / 2 <= (kIvMaxS + 3) / 4)) ? np_env : 4;
  if (np == 8) {
    const int nqp = ((QS + 7) / 8 + 255) / 256;
    if (nqp <= 1) hipLaunchKernelGGL((ivector_acc_kernel<1, 8>), dim3(njobs * 8), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ivector_acc_kernel<3, 8>), dim3(njobs * 8), dim3(256), 0, s, a);
  } else if (np == 2) {
    const int nqp = ((QS + 1) / 2 + 255) / 256;
    if (nqp <= 3) hipLaunchKernelGGL((ivector_acc_kernel<3, 2>), dim3(njobs * 2), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ivector_acc_kernel<5, 2>), dim3(njobs * 2), dim3(256), 0, s, a);
  } else {
    const int nqp = ((QS + 3) / 4 + 255) / 256;
    if (nqp <= 1) hipLaunchKernelGGL((ivector_acc_kernel<1, 4>), dim3(njobs * 4), dim3(256), 0, s, a);
    else if (nqp <= 3) hipLaunchKernelGGL((ivector_acc_kernel<3, 4>), dim3(njobs * 4), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ivector_acc_kernel<5, 4>), dim3(njobs * 4), dim3(256), 0, s, a);
  }
  hipLaunchKernelGGL(ivector_cg_kernel, dim3(njobs), dim3(128), 0, s, a);
}

// ===========================================================================
// speaker x-vectors (xvector.h)
// ===========================================================================
// Kaldi SlidingWindowCmn (feat/feature-functions.cc SlidingWindowCmnInternal
// [K]) with the reference's options (centered 300-frame window, means only,
// src/recognizer.cc:393-397), in double, over each utterance's selected
// frames: one block per utterance of the batch, one lane per feature dim
// walking the frames with the running window sum; out = x + (-1 / frames) *
// sum into the utterance's slot of the nnet input ring.  Columns past D
// (input padding) are zero.
__global__ void xvec_cmn_kernel(const float* feats, int feat_mask, int feat_slots, int D,
                                const int* rows, const XvecUtt* utts, int window, float* out,
                                int out_mask, int out_slots, int out_dim) {
  const int d = threadIdx.x, b = blockIdx.x;
  if (d >= out_dim) return;
  const XvecUtt u = utts[b];
  const int n = u.nsel;
  const int* rw = rows + u.rows0;
  float* o = out + (size_t)b * out_dim + d;
  const size_t ostride = (size_t)out_slots * out_dim;
  if (d >= D) {
    for (int t = 0; t < n; t++) o[(size_t)(t & out_mask) * ostride] = 0.0f;
    return;
  }
  const float* f = feats + (size_t)b * D + d;
  const size_t fstride = (size_t)feat_slots * D;
  double sum = 0.0;
  int last_start = -1, last_end = -1;
  for (int t = 0; t < n; t++) {
    int ws = t - window / 2, we = ws + window;
    if (ws < 0) { we -= ws; ws = 0; }
    if (we > n) {
      ws -= we - n;
      we = n;
      if (ws < 0) ws = 0;
    }
    if (last_start < 0) {
      for (int v = ws; v < we; v++) sum = sum + (double)f[(size_t)(rw[v] & feat_mask) * fstride];
    } else {
      if (ws > last_start) sum = sum - (double)f[(size_t)(rw[last_start] & feat_mask) * fstride];
      if (we > last_end) sum = sum + (double)f[(size_t)(rw[last_end] & feat_mask) * fstride];
    }
    last_start = ws;
    last_end = we;
    const double alpha = -1.0 / (double)(we - ws);
    const double x = (double)f[(size_t)(rw[t] & feat_mask) * fstride];
    o[(size_t)(t & out_mask) * ostride] = (float)(x + alpha * sum);
  }
}

// statistics extraction + pooling (StatisticsExtractionComponent /
// StatisticsPoolingComponent, nnet3/nnet-general-component.cc [K]) of each
// utterance's frame-level rows [pool_row0, pool_row0 + npool) (grid y = the
// utterance): [log count x nlog], mean, stddev = sqrt(max(floor, E[x^2] -
// mean^2)); double sums in row order
__global__ void xvec_pool_kernel(const float* rows, int ld, const XvecUtt* utts, int D, int nlog,
                                 int stddevs, float var_floor, float* out, int out_stride) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  const XvecUtt u = utts[blockIdx.y];
  const int n = u.npool;
  float* o = out + (size_t)blockIdx.y * out_stride;
  if (d < nlog) o[d] = (float)log((double)n);
  if (d >= D) return;
  const float* r = rows + (size_t)u.pool_row0 * ld + d;
  double s = 0.0, s2 = 0.0;
  for (int t = 0; t < n; t++) {
    const double x = (double)r[(size_t)t * ld];
    s = s + x;
    s2 = s2 + x * x;
  }
  const double mean = s / (double)n;
  o[nlog + d] = (float)mean;
  if (stddevs) {
    double var = s2 / (double)n - mean * mean;
    if (var < (double)var_floor) var = (double)var_floor;
    o[nlog + D + d] = (float)sqrt(var);
  }
}

// one row of an affine map in the GEMM kernels' canonical order (nnet_plan.h
// GemmKSlices; groups of eight walked 0,4,1,5,2,6,3,7), oracle canon_dot,
// for G inputs at once (x + g * xstride): each weight is loaded once and
// every input keeps its own accumulator chain
template <int G>
__device__ void xvec_canon_dot(const float* w, const float* x, int xstride, int K, float* a) {
  int ns = 1;  // GemmKSlices
  if (K >= 512 && K % 256 == 0)
    while (ns < 8 && 2 * ns <= K / 256) ns *= 2;
  const int kw = K / ns;
  for (int z = 0; z < ns; z++) {
    float p[G];
#pragma unroll
    for (int g = 0; g < G; g++) p[g] = 0.0f;
    const int ke = (z + 1) * kw;
    for (int kg = z * kw; kg < ke; kg += 8)
      for (int i = 0; i < 8 && kg + i < ke; i++) {
        const int k = kg + 8 <= ke ? kg + ((i & 1) << 2) + (i >> 1) : kg + i;
        const float wk = w[k];
#pragma unroll
        for (int g = 0; g < G; g++) p[g] = __builtin_fmaf(x[(size_t)g * xstride + k], wk, p[g]);
      }
#pragma unroll
    for (int g = 0; g < G; g++) a[g] = z == 0 ? p[g] : a[g] + p[g];
  }
}

constexpr int kXvecGroup = 4;  // utterances per thread of the head affine

// head op of the pooled statistics, for the batch's utterances (grid y = a
// group of kXvecGroup of them): 1 affine (+ bias when b), 2 ReLU,
// 3 x * scale + offset
__global__ void xvec_affine_kernel(const float* W, const float* bias, const float* x, int K, int N,
                                   int kind, float* y, int stride, int nutt) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int u0 = blockIdx.y * kXvecGroup;
  if (n >= N) return;
  const int nu = nutt - u0 < kXvecGroup ? nutt - u0 : kXvecGroup;
  const float* xu = x + (size_t)u0 * stride;
  float* yu = y + (size_t)u0 * stride;
  if (kind == 1) {
    float a[kXvecGroup];
    if (nu == kXvecGroup) {
      xvec_canon_dot<kXvecGroup>(W + (size_t)n * K, xu, stride, K, a);
    } else {
      for (int g = 0; g < nu; g++) xvec_canon_dot<1>(W + (size_t)n * K, xu + (size_t)g * stride, stride, K, a + g);
    }
    for (int g = 0; g < nu; g++) yu[(size_t)g * stride + n] = bias ? a[g] + bias[n] : a[g];
  } else if (kind == 2) {
    for (int g = 0; g < nu; g++) {
      const float v = xu[(size_t)g * stride + n];
      yu[(size_t)g * stride + n] = v < 0.0f ? 0.0f : v;
    }
  } else {
    for (int g = 0; g < nu; g++) yu[(size_t)g * stride + n] = xu[(size_t)g * stride + n] * W[n] + bias[n];
  }
}

// whitening and length normalisation (src/recognizer.cc:406-416), one block
// per utterance: x - mean, transform rows (canonical order), norm = sqrt of
// the sequential float sum of squares, ratio = norm / sqrt(R) and scale
// 1/ratio rounded through double
__global__ __launch_bounds__(256) void xvec_finish_kernel(const float* x, int xstride,
                                                          const float* mean, int E, const float* T,
                                                          int R, float* out) {
  __shared__ float xc[1024];
  __shared__ float scale;
  const float* xb = x + (size_t)blockIdx.x * xstride;
  float* ob = out + (size_t)blockIdx.x * R;
  for (int e = threadIdx.x; e < E; e += blockDim.x) xc[e] = xb[e] - mean[e];
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    float a;
    xvec_canon_dot<1>(T + (size_t)r * E, xc, 0, E, &a);
    ob[r] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ss = 0.0f;
    for (int r = 0; r < R; r++) ss = ss + ob[r] * ob[r];
    const float norm = sqrtf(ss);
    const float ratio = (float)((double)norm / sqrt((double)R));
    scale = (float)(1.0 / (double)ratio);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) ob[r] = ob[r] * scale;
}

void LaunchXvecCmn(const float* feats, int feat_mask, int feat_slots, int D, const int* rows,
                   const XvecUtt* utts, int nutt, int window, float* out, int out_mask,
                   int out_slots, int out_dim, hipStream_t s) {
  if (nutt <= 0) return;
  hipLaunchKernelGGL(xvec_cmn_kernel, dim3(nutt), dim3((out_dim + 63) / 64 * 64), 0, s, feats,
                     feat_mask, feat_slots, D, rows, utts, window, out, out_mask, out_slots,
                     out_dim);
}

void LaunchXvecPool(const float* rows, int ld, const XvecUtt* utts, int nutt, int D, int nlog,
                    int stddevs, float var_floor, float* out, int out_stride, hipStream_t s) {
  if (nutt <= 0) return;
  const int threads = D > nlog ? D : nlog;
  hipLaunchKernelGGL(xvec_pool_kernel, dim3((threads + 255) / 256, nutt), dim3(256), 0, s, rows,
                     ld, utts, D, nlog, stddevs, var_floor, out, out_stride);
}

void LaunchXvecAffine(const float* W, const float* b, const float* x, int K, int N, int kind,
                      float* y, int stride, int nutt, hipStream_t s) {
  if (nutt <= 0) return;
  hipLaunchKernelGGL(xvec_affine_kernel, dim3((N + 255) / 256, (nutt + kXvecGroup - 1) / kXvecGroup),
                     dim3(256), 0, s, W, b, x, K, N, kind, y, stride, nutt);
}

void LaunchXvecFinish(const float* x, int xstride, const float* mean, int E, const float* T, int R,
                      float* out, int nutt, hipStream_t s) {
  if (nutt <= 0) return;
  hipLaunchKernelGGL(xvec_finish_kernel, dim3(nutt), dim3(256), 0, s, x, xstride, mean, E, T, R,
                     out);
}

}  // namespace vamd
