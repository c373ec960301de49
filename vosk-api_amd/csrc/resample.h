// Windowed-sinc sample-rate conversion tables (Kaldi LinearResample, used by
// the reference for inputs whose rate differs from the model's:
// src/batch_recognizer.cc:27-29 LinearResample(sr, 16000, min(sr/2, 8000), 6)
// and the feature pipeline's allow_downsample/upsample, src/model.cc:221).
// The table is built on the host; resample_kernel (kernels.hip) applies it.
#pragma once

#include <vector>

namespace vamd {

struct ResampleTable {
  int rate_in = 0, rate_out = 0;
  int in_unit = 0, out_unit = 0;  // samples per period of gcd(rate_in, rate_out)
  int taps = 0;                   // max taps over phases (rows zero-padded)
  double filter_cutoff = 0.0, window_width = 0.0;
  int num_zeros = 0;
  std::vector<int> first;         // [out_unit] first input index of phase p
  std::vector<int> ntaps;         // [out_unit]
  std::vector<float> w;           // [out_unit][taps]

  // Kaldi LinearResample::GetNumOutputSamples: outputs computable from the
  // first n_in input samples (flush: the input has ended, later samples = 0)
  long long NumOutputSamples(long long n_in, bool flush) const;
};

// cutoff <= 0: min(rate_in, rate_out) / 2 (the reference's batch setting for
// a 16 kHz model), num_zeros 6
ResampleTable BuildResampleTable(int rate_in, int rate_out, double cutoff = 0.0, int num_zeros = 6);

}  // namespace vamd
