// Looped nnet3 evaluation plan: fused ops + per-chunk time patterns.
//
// Replaces what the reference gets from Kaldi's DecodableNnetSimpleLoopedInfo
// (src/model.cc:245-246; compiled looped computation [K]) and
// CollapseModel (src/model.cc:241).  Every affine-like component
// (FixedAffine/Affine/NaturalGradientAffine/Linear/Tdnn) becomes one GEMM op
// whose A operand is gathered straight from per-slot activation time rings
// (time-spliced rows, "Offset()" descriptors); the element-wise components
// that follow it (ReLU, BatchNorm test mode, dropout/spec-augment identities,
// NoOp bypass sums "Sum(Scale(a, x), y)") become the op's fused epilogue.
// Descriptors that are not plain offsets (e.g. the delta layer) become a
// GATHER op evaluating a postfix program.
//
// Chunking: chunk c produces output frames t = c*fpc + fss*i, i < fpc/fss.
// Each op computes, per chunk, the times pattern[k] + c*fpc.  The first
// chunk of a stream is preceded by `priming_chunks` chunks at negative times
// (inputs clamped to frame 0, as Kaldi replicates the first frame), so every
// chunk job has the same shape and a batch of jobs is a plain GEMM.
#pragma once

#include <string>
#include <vector>

#include "model_io.h"

namespace vamd {

struct StoredNode {
  std::string name;
  int dim = 0;
  bool is_input = false;    // the feature input (time ring written by the MFCC kernel)
  bool is_ivector = false;  // a per-chunk input (no time ring: one row per chunk job)
};

struct ASegment {  // A columns [col0, col0+dim) <- node(tau + offset)[src_col ...]
  int node, offset, col0, dim, src_col;
};

struct EpiStage {
  enum Kind { BIAS = 0, RELU = 1, MUL_ADD = 2, ADD_NODE = 3, SCALE = 4 };
  int kind;
  int vec0 = -1, vec1 = -1;             // BIAS: vec0; MUL_ADD: x*vec0 + vec1
  int node = -1, offset = 0, src_col = 0;  // ADD_NODE: x = (c * node(tau+offset)) + x
  bool scaled = false;                  // ADD_NODE: whether the term carries Scale(c, .)
  float c = 1.f;                        // ADD_NODE / SCALE factor
};

struct GInstr {  // postfix program step for GATHER ops
  // PUSH_JOB: the chunk job's i-vector row (ReplaceIndex(ivector, t, 0))
  enum Op { PUSH = 0, SCALE = 1, ADD = 2, CONST = 3, PUSH_JOB = 4 };
  int op, node = -1, offset = 0, src_col = 0;
  float c = 0.f;
};

struct GPart {
  int col0, dim;
  std::vector<GInstr> prog;
};

struct Op {
  enum Kind { GEMM = 0, GATHER = 1 };
  int kind = GEMM;
  std::string name;   // last node fused into this op
  int out_node = -1;  // stored node index; -1 = log-likelihood output
  int N = 0, K = 0;
  int weight = -1;    // index into NnetPlan::mats (N x K row-major)
  std::vector<ASegment> segs;
  std::vector<GPart> parts;
  std::vector<EpiStage> epi;
  std::vector<int> pattern;  // times computed per chunk, relative to c*fpc
  std::vector<int> deps;     // op indices this op reads from
};

// Canonical summation order of every affine dot product (GPU and oracle):
// K is cut into GemmKSlices(K) equal slices, each an fma chain over its k in
// increasing order starting from 0, and the slice sums are added left to
// right; the bias is added last.  Kaldi leaves the order to BLAS; fixing one
// lets long reductions (K = 1024 bottlenecks) spread over more workgroups and
// keeps GPU and oracle bit-identical.  Mirrored by orc_kslices() in oracle.c.
// The count is K / 256 rounded down to a power of two, at most 8 (the split-K
// reduction of the streaming kernel): K = 1536 (a 768-dim TDNN-F layer
// spliced twice, the sre16 x-vector layers) runs as 4 slices of 384.
inline int GemmKSlices(int K) {
  if (K < 512 || K % 256) return 1;
  int n = 1;
  while (n < 8 && 2 * n <= K / 256) n *= 2;
  return n;
}

struct NnetPlan {
  int fpc = 0, fss = 1, opc = 0;  // frames per chunk, subsampling, outputs per chunk
  int out_dim = 0;
  int left_context = 0, right_context = 0;  // Kaldi ComputeSimpleNnetContext semantics
  int priming_chunks = 0;
  int max_age = 0;  // max (latest computed - oldest read) time distance inside a chunk
  int input_node = -1;
  int ivector_node = -1, ivector_dim = 0;  // per-chunk i-vector input, if the nnet has one
  std::vector<StoredNode> nodes;
  std::vector<Op> ops;
  std::vector<Matrix> mats;
  std::vector<std::vector<float>> vecs;
  int input_dim = 0;
  double flops_per_chunk = 0;  // algorithmic (2 * rows * N * K summed over GEMM ops)
  // ring length (power of two) sufficient for `jobs_per_slot` chunk jobs of
  // one stream inside one engine step
  int RingFrames(int jobs_per_slot) const;
  std::string Describe() const;
};

NnetPlan BuildNnetPlan(const Nnet& nnet, int frames_per_chunk, int frame_subsampling_factor,
                       float acoustic_scale);

// BatchNorm test-mode scale/offset (Kaldi BatchNormComponent::ComputeDerived):
// scale = target_rms / sqrt(max(var,0) + eps), offset = -mean * scale,
// computed in double and rounded to float once.
void BatchNormScaleOffset(const Component& c, std::vector<float>* scale,
                          std::vector<float>* offset);

}  // namespace vamd
