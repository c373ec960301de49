// Host-callable launchers for the HIP kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "engine_dev.h"

namespace vamd {

void LaunchAppendSamples(const SampleJob* jobs, int njobs, float* ring, int ring_len,
                         hipStream_t s);
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
void LdsHashSelfTest(int n, int blocks, int* out);  // dev (tools/gemm_bench)
int DecoderLdsFrameTokens();  // default LDS frame-construction threshold
void LaunchDecode(const DecArgs& a, int njobs, hipStream_t s);
void LaunchTraceback(const TraceArgs& a, int n, hipStream_t s);
void LaunchInitKeys(unsigned long long* key, int* stamp, long long n_states_total, hipStream_t s);

}  // namespace vamd
