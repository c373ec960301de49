// Host-callable launchers for the HIP kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "engine_dev.h"

namespace vamd {

void LaunchAppendSamples(const SampleJob* jobs, int njobs, float* ring, int ring_len,
                         hipStream_t s);
// One workgroup per item: the segments' lattice records gathered into one
// contiguous block (one device-to-host copy instead of three per segment).
void LaunchGatherCopy(const CopyItem* items, int nitems, unsigned* dst, hipStream_t s);
void LaunchResample(const ResampleJob* jobs, int njobs, const ResampleDev* tables, const float* raw,
                    int raw_len, float* ring, int ring_len, hipStream_t s);
void LaunchMfcc(const MfccDev& m, const MfccJob* jobs, int njobs, int total_frames,
                const float* sample_ring, int sample_ring_len, const RingSet& rings,
                hipStream_t s);
// GEMM ops: bk = LDS-kernel K-step (8, 16 or 32; must divide every segment boundary)
// N tile width LaunchNnetGemm uses for an N-column op
inline int GemmTileN(int N) { return (N % 96 == 0 && N % 64 != 0) ? 96 : 64; }
void LaunchNnetGemm(const NnetOpArgs& a, int bk, hipStream_t s);
bool GemmStreamable(const NnetOpArgs& a);  // streaming kernel applies (else LDS kernel)
extern int g_gemm_variant;  // dev override: 1/2 streaming NB=natural/1, 3 LDS (tools/gemm_bench)
void LaunchNnetGather(const NnetOpArgs& a, hipStream_t s);
// i-vector extraction: online CMVN per stream (before the LDA / UBM GEMMs),
// then per-frame 5-best posteriors, statistics and CG per stream (after them)
void LaunchCmvn(const CmvnDev& c, const CmvnJob* jobs, int njobs, hipStream_t s);
void LaunchIvectorStats(const IvArgs& a, const float* ll, int rows, int njobs, hipStream_t s);
// token passing (decoder.hip)
int DecoderLdsProbe();  // default LDS probe limit of the frame table
void LaunchDecode(const DecArgs& a, int njobs, hipStream_t s);
// the last lattice prune of ending segments (slots: device list of n streams)
void LaunchPruneFinal(const DecArgs& a, const int* slots, int n, bool use_final, hipStream_t s);
void LaunchTraceback(const TraceArgs& a, int n, hipStream_t s);
// speaker x-vectors (xvector.h): selection + sliding CMN, statistics
// pooling, head ops, whitening
// x-vector chain over a batch of utterances (XvecUtt per utterance; slot b
// of the feature / input rings and row b of the pooled and head buffers)
void LaunchXvecCmn(const float* feats, int feat_mask, int feat_slots, int D, const int* rows,
                   const XvecUtt* utts, int nutt, int window, float* out, int out_mask,
                   int out_slots, int out_dim, hipStream_t s);
void LaunchXvecPool(const float* rows, int ld, const XvecUtt* utts, int nutt, int D, int nlog,
                    int stddevs, float var_floor, float* out, int out_stride, hipStream_t s);
void LaunchXvecAffine(const float* W, const float* b, const float* x, int K, int N, int kind,
                      float* y, int stride, int nutt, hipStream_t s);
void LaunchXvecFinish(const float* x, int xstride, const float* mean, int E, const float* T, int R,
                      float* out, int nutt, hipStream_t s);
void LaunchInitTables(int* state, unsigned long long* key, int* stamp, long long n, hipStream_t s);

}  // namespace vamd
