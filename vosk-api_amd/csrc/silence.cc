#include "silence.h"

#include "common.h"

namespace vamd {

void SilenceWeighting::ComputeCurrentTraceback(const std::vector<int>& frame_tid,
                                               const std::vector<int>& frame_tok) {
  const int num_frames_decoded = (int)frame_tid.size(), num_frames_prev = (int)info_.size();
  // info_ may be longer than the decoded frames: it covers every frame a
  // weight was requested for
  if (num_frames_prev < num_frames_decoded) info_.resize(num_frames_decoded);
  if (num_frames_prev > num_frames_decoded && info_[num_frames_decoded].tid != -1)
    VAMD_ERR("silence weighting: number of frames decoded decreased");
  for (int frame = num_frames_decoded - 1; frame >= 0; frame--) {
    // the traceback before an unchanged source token is unchanged too
    if (info_[frame].token == frame_tok[frame]) break;
    info_[frame].token = frame_tok[frame];
    info_[frame].tid = frame_tid[frame];
  }
}

}  // namespace vamd
