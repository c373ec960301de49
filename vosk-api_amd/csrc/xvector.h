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
#include <condition_variable>
#include <deque>
#include <exception>
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

// One x-vector request (the arguments of GetSpkVector's extraction).
struct XvecRequest {
  const float* samples = nullptr;
  long long n = 0;
  int rate = 0;
  int first_frame = 0;
  const std::vector<char>* keep = nullptr;
  std::vector<float>* xvec = nullptr;  // out
  int num_frames = 0;                  // out: selected frames
  bool ok = false;                     // out: a vector was produced
};

// GPU x-vector extraction for one speaker model on one device.  Requests are
// batched across utterances: every kernel of the chain takes the utterance
// as a grid dimension (one ring slot, one MFCC job list, one block of jobs
// per utterance), and concurrent Extract callers are group-committed -- the
// first caller to find the extractor idle runs everything queued (up to the
// slot and ring-memory caps) as one launch sequence while later callers wait
// for their result.  Each utterance's arithmetic is independent of the batch
// it runs in (row-independent GEMM order, per-utterance reductions), so a
// batched vector equals the one extracted alone bit for bit.
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
  // a batch of requests, extracted together (split only by the caps)
  void ExtractBatch(const std::vector<XvecRequest*>& reqs);
  int OutputDim() const { return md_->transform.rows; }
  const XvectorNet& net() const { return net_; }
  // launch sequences run and utterances extracted so far (group-commit probe)
  long long Batches() const { return batches_; }
  long long Utterances() const { return utterances_; }
  // frame-level layers: GEMM flops launched and their HIP-event time
  double LayerFlops() const { return gemm_flops_; }
  double LayerMs() const { return layers_ms_; }

 private:
  struct Pending {
    XvecRequest* r;
    bool done = false;
    std::exception_ptr err;
  };
  void RunBatch(const std::vector<XvecRequest*>& reqs);  // under mu_
  void Reserve(int slots, long long samples, long long raw, int frames, int sel, int jobs_per_slot,
               int jobs);
  int TableIndex(int rate);  // resampling table of an input rate in d_tables_
  long long RingBytesPerSlot(int jobs_per_slot) const;
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
  // per-batch buffers (grown on demand); slot b = the batch's utterance b
  int slot_cap_ = 0;             // utterance slots of the rings and buffers
  int jobs_cap_ = 0;             // nnet jobs over all slots
  int slot_jobs_cap_ = 0;        // nnet jobs of one slot the rings hold
  int ring_ = 0;
  long long wave_len_ = 0;       // per-slot sample buffer (power of two)
  long long raw_len_ = 0;        // per-slot raw input before resampling
  int feat_ring_ = 0;            // per-slot MFCC rows (power of two)
  int sel_cap_ = 0, rjobs_cap_ = 0;
  float* d_wave_ = nullptr;      // [slot][wave_len_]
  float* d_raw_ = nullptr;       // [slot][raw_len_]
  std::vector<ResampleTable> tables_;  // per input rate seen so far
  std::vector<int> table_rates_;
  ResampleDev* d_tables_ = nullptr;
  ResampleJob* d_rjobs_ = nullptr;
  float* d_feats_ = nullptr;     // [frame ring][slot][feat_dim]
  int* d_rows_ = nullptr;        // selected frame indices, per slot back to back
  XvecUtt* d_utts_ = nullptr;    // [slot]
  float* d_out_ = nullptr;       // frame-level output rows [jobs * fpc][stats_in]
  DevJob* d_jobs_ = nullptr;
  MfccJob* d_mjobs_ = nullptr;   // [slot]
  std::vector<float*> ring_ptrs_;
  float** d_ring_ptrs_ = nullptr;
  int* d_ring_dims_ = nullptr;
  std::vector<float*> head_w_, head_b_;
  float* d_stats_ = nullptr;     // pooled statistics [slot][head_max_]
  float* d_head_ = nullptr;      // head ping-pong [2][slot][head_max_]
  float* d_mean_ = nullptr;
  float* d_transform_ = nullptr;
  float* d_xvec_ = nullptr;      // [slot][R]
  float* h_xvec_ = nullptr;      // pinned copy of d_xvec_
  int head_max_ = 0;
  std::mutex mu_;                // the device buffers and stream
  std::mutex qmu_;               // the request queue
  std::condition_variable qcv_;
  std::deque<Pending*> queue_;
  bool leader_ = false;
  long long batches_ = 0, utterances_ = 0;
  double gemm_flops_ = 0.0, layers_ms_ = 0.0;
  hipEvent_t ev_[2] = {nullptr, nullptr};
};

}  // namespace vamd
