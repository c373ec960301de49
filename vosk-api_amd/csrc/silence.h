// Silence weighting of the online i-vector statistics (host side).
//
// The reference's Recognizer feeds the i-vector extractor per-frame weights
// derived from the decoder's current best path before every decoding advance
// (src/recognizer.cc:226-237, UpdateSilenceWeights; configured in
// src/model.cc:230-231 with silence weight 1e-3 and the endpoint's silence
// phones; one object per decoder segment, recreated in CleanUp,
// src/recognizer.cc:188-191).  The algorithm is Kaldi's
// OnlineSilenceWeighting (online2/online-ivector-feature.cc [K], not vendored
// in the reference): ComputeCurrentTraceback records the transition-id of
// every decoded frame on the best path (stopping where the path is unchanged),
// GetDeltaWeights turns the silence / non-silence status of the frames into
// weight changes at the feature frame rate.  This class restates it; the GPU
// applies the resulting (frame, delta) entries to the statistics.
#pragma once
#include <algorithm>
#include <utility>
#include <vector>

namespace vamd {

class SilenceWeighting {
 public:
  // silence_weight: weight of silence frames (1e-3 in the reference);
  // frame_subsampling_factor: feature frames per decoder frame (3)
  SilenceWeighting(float silence_weight = 1e-3f, int frame_subsampling_factor = 3)
      : silence_weight_(silence_weight), fss_(frame_subsampling_factor) {}

  // Best-path traceback of the decoder (without final costs): for each
  // decoded frame, the transition-id of its emitting arc and the identity of
  // that arc's source token (a token is unique per frame and state, so the
  // source state identifies it).  Frames are decoder frames of the segment.
  void ComputeCurrentTraceback(const std::vector<int>& frame_tid, const std::vector<int>& frame_tok);

  // Weight changes for feature frames, first_decoder_frame = feature frame of
  // the segment's decoder frame 0 (frame_offset * 3 in the reference).
  // is_silence_tid(tid) decides silence by the tid's phone.
  template <class F>
  void GetDeltaWeights(int num_frames_ready, int first_decoder_frame, F is_silence_tid,
                       std::vector<std::pair<int, float>>* delta);

  void Reset() { info_.clear(); }

 private:
  struct FrameInfo {
    int token = -1;          // source token of the best path's arc into this frame
    int tid = -1;            // its transition-id (-1: no traceback yet)
    float current_weight = 0.0f;  // weight already handed to the i-vector
  };
  float silence_weight_;
  int fss_;
  std::vector<FrameInfo> info_;
};

template <class F>
void SilenceWeighting::GetDeltaWeights(int num_frames_ready, int first_decoder_frame, F is_silence_tid,
                                       std::vector<std::pair<int, float>>* delta) {
  delta->clear();
  const int fs = fss_;
  const int num_decoder_frames_ready = (num_frames_ready - first_decoder_frame + fs - 1) / fs;
  const int prev_num_frames_processed = (int)info_.size();
  if ((int)info_.size() < num_decoder_frames_ready) info_.resize(num_decoder_frames_ready);
  // frames more than 100 decoder frames before the previous end keep their weights
  const int begin_frame = std::max(0, prev_num_frames_processed - 100);
  const int frames_out = (int)info_.size() - begin_frame;
  if (frames_out <= 0) return;
  std::vector<float> frame_weight(frames_out, 1.0f);
  if (info_[begin_frame].tid == -1) {
    // no traceback within the frames to output: repeat the most recent
    // weight output, or the silence weight if none
    const float w = begin_frame == 0 ? silence_weight_ : info_[begin_frame - 1].current_weight;
    for (int o = 0; o < frames_out; o++) frame_weight[o] = w;
  } else {
    for (int o = 0; o < frames_out; o++) {
      const int tid = info_[begin_frame + o].tid;
      if (tid == -1) {
        frame_weight[o] = frame_weight[o - 1];  // newer than the traceback
      } else if (is_silence_tid(tid)) {
        frame_weight[o] = silence_weight_;
      }
    }
  }
  for (int o = 0; o < frames_out; o++) {
    FrameInfo& fi = info_[begin_frame + o];
    const float old_w = fi.current_weight, new_w = frame_weight[o], diff = new_w - old_w;
    fi.current_weight = new_w;
    // the last frame is always reported (even with a zero change)
    if (diff != 0.0f || o + 1 == frames_out)
      for (int i = 0; i < fs; i++)
        delta->emplace_back(first_decoder_frame + (begin_frame + o) * fs + i, diff);
  }
}

}  // namespace vamd
