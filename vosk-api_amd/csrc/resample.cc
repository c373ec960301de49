#include "resample.h"

#include <cmath>
#include <numeric>

#include "common.h"

namespace vamd {

namespace {
// Kaldi's FilterFunc: Hanning-windowed sinc, evaluated in float after
// double-precision trigonometry (feat/resample.cc)
float FilterFunc(double cutoff, int num_zeros, float t) {
  float window, filter;
  if (std::fabs(t) < num_zeros / (2.0 * cutoff))
    window = (float)(0.5 * (1 + std::cos(2.0 * M_PI * cutoff / num_zeros * t)));
  else
    window = 0.0f;
  if (t != 0.0f)
    filter = (float)(std::sin(2.0 * M_PI * cutoff * t) / (M_PI * t));
  else
    filter = (float)(2.0 * cutoff);
  return filter * window;
}
}  // namespace

ResampleTable BuildResampleTable(int rate_in, int rate_out, double cutoff, int num_zeros) {
  if (rate_in <= 0 || rate_out <= 0) VAMD_ERR("bad resampling rates " << rate_in << " -> " << rate_out);
  ResampleTable t;
  t.rate_in = rate_in;
  t.rate_out = rate_out;
  t.filter_cutoff = cutoff > 0 ? cutoff : 0.5 * std::min(rate_in, rate_out);
  t.num_zeros = num_zeros;
  const int g = std::gcd(rate_in, rate_out);
  t.in_unit = rate_in / g;
  t.out_unit = rate_out / g;
  t.window_width = num_zeros / (2.0 * t.filter_cutoff);
  t.first.resize(t.out_unit);
  t.ntaps.resize(t.out_unit);
  std::vector<std::vector<float>> rows(t.out_unit);
  for (int i = 0; i < t.out_unit; i++) {
    const double output_t = i / (double)rate_out;
    const double min_t = output_t - t.window_width, max_t = output_t + t.window_width;
    const int lo = (int)std::ceil(min_t * rate_in), hi = (int)std::floor(max_t * rate_in);
    t.first[i] = lo;
    t.ntaps[i] = hi - lo + 1;
    rows[i].resize(hi - lo + 1);
    for (int j = 0; j <= hi - lo; j++) {
      const double input_t = (lo + j) / (double)rate_in, delta_t = input_t - output_t;
      rows[i][j] = FilterFunc(t.filter_cutoff, num_zeros, (float)delta_t) / (float)rate_in;
    }
    t.taps = std::max(t.taps, t.ntaps[i]);
  }
  t.w.assign((size_t)t.out_unit * t.taps, 0.0f);
  for (int i = 0; i < t.out_unit; i++)
    for (int j = 0; j < t.ntaps[i]; j++) t.w[(size_t)i * t.taps + j] = rows[i][j];
  return t;
}

long long ResampleTable::NumOutputSamples(long long n_in, bool flush) const {
  const long long tick_freq = std::lcm((long long)rate_in, (long long)rate_out);
  const long long ticks_per_input = tick_freq / rate_in;
  long long interval = n_in * ticks_per_input;
  if (!flush) interval -= (long long)std::floor(window_width * tick_freq);
  if (interval <= 0) return 0;
  const long long ticks_per_output = tick_freq / rate_out;
  long long last = interval / ticks_per_output;
  if (last * ticks_per_output == interval) last--;
  return last + 1;
}

}  // namespace vamd
