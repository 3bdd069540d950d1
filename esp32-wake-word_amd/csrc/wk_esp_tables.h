// wk_esp_tables.h -- host-side tables of front-end mode A (main/esp_mfcc/mfcc.c)
// at any parameter set, built with the reference's own float formulas.
// Shared by the GPU path (wk_esp_mfcc.hip uploads them) and the host path
// (wk_host.cpp computes with them); plain C++, no HIP.
#pragma once
#include <math.h>

#include <vector>

namespace wk {
namespace esp {

// mfcc.c:133-142 (hz_to_mel takes f = 0 as 1; mel_to_hz uses the base-10 form).
inline float hz_to_mel(float f) { return 1127.0f * log1pf((f == 0.0f ? 1.0f : f) / 700.0f); }
inline float mel_to_hz(float m) { return 700.0f * (powf(10.0f, m / 2595.0f) - 1.0f); }

// create_mel_filterbank(sr, n_filters, n_fft, 0, -1) (mfcc.c:144-234) as
// dense rows [n_filters][n_fft / 2 + 1]: triangles on floor(hz / bin_width)
// bins with the reference's clamps; a degenerate triangle at the top of a
// crowded bank keeps its 0/0 (NaN) weight, as mfcc.c:224 does.
inline std::vector<float> filterbank(int sr, int n_filters, int n_fft) {
  const int nb = n_fft / 2 + 1;
  std::vector<float> fb((size_t)n_filters * nb, 0.0f);
  const float lo = hz_to_mel(0.0f), hi = hz_to_mel((float)(sr / 2));
  const float bw = (float)sr / n_fft;
  std::vector<int> bin(n_filters + 2);
  for (int i = 0; i < n_filters + 2; ++i) bin[i] = (int)floorf(mel_to_hz(lo + i * (hi - lo) / (n_filters + 1)) / bw);
  auto clamp = [nb](int v) { return v < 0 ? 0 : (v >= nb ? nb - 1 : v); };
  for (int f = 0; f < n_filters; ++f) {
    int l = clamp(bin[f]), c = clamp(bin[f + 1]), r = clamp(bin[f + 2]);
    if (l >= c) c = l + 1;
    if (c >= r) r = c + 1;
    if (r >= nb) r = nb - 1;
    float* row = fb.data() + (size_t)f * nb;
    for (int j = l; j <= c; ++j)
      if (j >= 0 && j < nb) row[j] = (float)(j - l) / (c - l);
    for (int j = c; j <= r; ++j)   // (r == c at the top of a crowded bank: 0/0, a NaN weight, as in the reference)
      if (j >= 0 && j < nb) row[j] = (float)(r - j) / (r - c);
  }
  return fb;
}

// Symmetric Hamming window, alpha 0.53836 (mfcc.c:118-120; float, the angle in double).
inline std::vector<float> window(int frame_size) {
  std::vector<float> w(frame_size);
  for (int i = 0; i < frame_size; ++i)
    w[i] = 0.53836f - (1.0f - 0.53836f) * cosf(2.0f * M_PI * i / (frame_size - 1));
  return w;
}

// DCT-II cosines [min(n_mfcc, n_filters)][n_filters] (mfcc.c:26-30 / :44-48:
// cos of the float-converted double angle) and the scales (:33, :57).
inline void dct(int n_mfcc, int n_filters, std::vector<float>& cosines, std::vector<float>& scale) {
  const int n_dct = n_mfcc < n_filters ? n_mfcc : n_filters;
  cosines.assign((size_t)n_dct * n_filters, 0.0f);
  scale.assign(n_dct, 0.0f);
  for (int k = 0; k < n_dct; ++k) {
    for (int i = 0; i < n_filters; ++i) cosines[(size_t)k * n_filters + i] = cosf(M_PI * k * (2 * i + 1) / (2.0f * n_filters));
    scale[k] = k == 0 ? sqrtf(1.0f / n_filters) : sqrtf(2.0f / n_filters);
  }
}

// mfcc.c's domain as the drop-in accepts it (esp-dsp's FFT takes powers of two
// up to its default maximum 4096): log2(n_fft), or -1 outside the domain.
inline int check_domain(int sampling_rate, int frame_size, int n_fft, int n_filters, int n_mfcc) {
  int lg = 0;
  while (lg < 31 && (1 << lg) < n_fft) ++lg;
  if (sampling_rate < 1 || frame_size < 1 || n_fft < 2 || n_fft > 4096 || (1 << lg) != n_fft || n_filters < 1 ||
      n_filters > 1024 || n_mfcc < 1)
    return -1;
  return lg;
}

}  // namespace esp
}  // namespace wk
