// Speaker x-vectors (reference src/spk_model.cc,
// src/recognizer.cc:326-419 GetSpkVector, :470-479 result fields).
//
// The reference keeps a second MFCC front end per recognizer (the speaker
// model's mfcc.conf, typically 30 cepstra with snip-edges=false), and at
// result time takes the segment's frames whose decoder frame (i / 3) is
// non-silence on the best path, applies sliding-window CMN (centered, 300
// frames), runs the x-vector nnet (TDNN layers, statistics extraction +
// pooling over the whole selection, the embedding affine), subtracts the
// global mean, applies transform.mat and scales the result to norm
// sqrt(dim).  Here all of it runs on the GPU at result time: the speaker MFCC
// over the segment's samples (mfcc_kernel with the speaker options), the
// selection + CMN (xvec_cmn_kernel), the frame-level layers as a chunked nnet
// plan on the GEMM kernels (the network up to the statistics input becomes a
// plan whose "output" is that node), the pooling (xvec_pool_kernel) and the
// head / whitening (xvec_affine_kernel, xvec_finish_kernel).
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "engine_dev.h"
#include "model_io.h"
#include "nnet_plan.h"
#include "resample.h"

namespace vamd {

struct SpkModelData {
  std::string dir;
  MfccOptions mfcc;          // mfcc.conf of the speaker model
  Nnet nnet;                 // final.ext.raw; input padded to input_dim
  int feat_dim = 0;          // MFCC dim
  int input_dim = 0;         // nnet input ring dim (feat_dim rounded up to 8; zero columns)
  std::vector<float> mean;   // mean.vec [embed]
  Matrix transform;          // transform.mat [out][embed]
  void Load(const std::string& dir);
};

// The x-vector network split at its statistics layer.
struct XvectorNet {
  NnetPlan frames;           // input -> input of the statistics extraction, fss 1
  int stats_in = 0;          // dim of that node
  int pool_left = 0, pool_right = 0;  // pooling window around output time 0
  int num_log_count = 0;     // StatisticsPoolingComponent configuration
  bool stddevs = true;
  float variance_floor = 1e-10f;
  struct HeadOp {
    enum Kind { AFFINE = 1, RELU = 2, MUL_ADD = 3 };
    int kind = AFFINE, in = 0, out = 0;
    std::vector<float> w, b;  // AFFINE: W [out][in], bias; MUL_ADD: scale, offset
  };
  std::vector<HeadOp> head;  // pooled statistics -> embedding ("output")
  int embed_dim = 0;
};
XvectorNet BuildXvectorNet(const SpkModelData& m, int frames_per_chunk);

// Kaldi FeatureWindow frame count of an online (not flushed) front end.
int SpkNumFrames(const MfccOptions& o, long long num_samples);

// GPU x-vector extraction for one speaker model on one device (serialised).
class SpkExtractor {
 public:
  SpkExtractor(std::shared_ptr<const SpkModelData> m, int device);
  ~SpkExtractor();
  // samples: the stream since its speaker front end started, at the speaker
  // MFCC rate; the segment's frames start at first_frame; frame i is used iff
  // keep[(i - first_frame) / 3].  Returns false (and *num_frames) when fewer
  // than 50 frames are selected (src/recognizer.cc:354,386-389).
  // Input at another rate is resampled first (Kaldi LinearResample, cutoff
  // min(rates)/2, 6 zeros, not flushed: the online feature's resampler).
  bool Extract(const float* samples, long long n, int rate, int first_frame,
               const std::vector<char>& keep, std::vector<float>* xvec, int* num_frames);
  int OutputDim() const { return md_->transform.rows; }
  const XvectorNet& net() const { return net_; }

 private:
  void Reserve(long long samples, int frames, int sel);
  template <class T> T* Upload(const std::vector<T>& v);
  void* DevAlloc(size_t bytes);
  void DevFree(void* p);

  std::shared_ptr<const SpkModelData> md_;
  XvectorNet net_;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  std::vector<void*> allocs_;
  MfccDev mfcc_{};
  std::vector<float*> vec_ptrs_;
  const float* const* d_vecs_ = nullptr;
  std::vector<const float*> weights_;
  std::vector<const int*> patterns_;
  std::vector<NnetOpArgs> op_args_;
  std::vector<int> op_bk_;
  int jobs_cap_ = 0;
  // per-extraction buffers (grown on demand)
  long long wave_cap_ = 0;
  int frame_cap_ = 0, sel_cap_ = 0, ring_ = 0;
  float* d_wave_ = nullptr;
  float* d_raw_ = nullptr;       // input before resampling
  long long raw_cap_ = 0;
  int table_rate_ = 0;           // rate of the cached resampling table
  ResampleDev* d_table_ = nullptr;
  ResampleJob* d_rjobs_ = nullptr;
  int rjobs_cap_ = 0;
  float* d_feats_ = nullptr;     // [frame ring][1][feat_dim]
  int feat_ring_ = 0;
  int* d_rows_ = nullptr;        // selected frame indices
  float* d_out_ = nullptr;       // frame-level output rows [jobs * fpc][stats_in]
  DevJob* d_jobs_ = nullptr;
  MfccJob* d_mjob_ = nullptr;
  std::vector<float*> ring_ptrs_;
  float** d_ring_ptrs_ = nullptr;
  int* d_ring_dims_ = nullptr;
  std::vector<float*> head_w_, head_b_;
  float* d_stats_ = nullptr;     // pooled statistics
  float* d_head_ = nullptr;      // head ping-pong [2][head_max_]
  float* d_mean_ = nullptr;
  float* d_transform_ = nullptr;
  float* d_xvec_ = nullptr;
  int head_max_ = 0;
  ResampleTable table_;
  std::mutex mu_;
};

}  // namespace vamd
