/*
 * esp_mfcc_oracle.c -- CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of front-end mode A, the reference's device MFCC
 * (main/esp_mfcc/mfcc.c:431-527, `extract_mfcc`).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker; the product library never links it.
 *
 * Why a restatement and not the reference file itself: mfcc.c includes
 * esp_heap_caps.h, esp_log.h, freertos/FreeRTOS.h and esp_dsp.h (ESP-IDF and
 * the un-vendored esp-dsp component, main/idf_component.yml:19).  None of them
 * exist in this image and stand-ins are not allowed, so mfcc.c is unbuildable
 * here ("Oracle").  PARITY STATUS: no reference test or fixture
 * holds mode-A MFCC values -> "parity unpinned"; this file is checked against
 * an independent numpy restatement (oracle/wk_oracle.py, mode A) instead.
 *
 * Steps, each following the reference line by line in float arithmetic:
 *   pre_emphasis      mfcc.c:66-74   y[0] = x[0], y[i] = x[i] - 0.97 x[i-1]
 *   frame_division    mfcc.c:76-108  no centring; n = (L - 320)/256 + 1
 *   apply_window      mfcc.c:110-131 symmetric Hamming, alpha 0.53836 (:460)
 *   power spectrum    mfcc.c:236-273 frame in the first 320 of 512 points,
 *                     (re^2 + im^2)/512 + 1e-12; the DFT here is exact
 *                     (double), standing in for esp-dsp's radix-2 FFT.
 *                     esp_pack = 1 restates dsps_cplx2reC_fc32's packing as
 *                     documented for esp-dsp 1.x: bins 1..255
 *                     carry 2 X[k], bin 0 carries X[0], bin 256 is zero.
 *   mel filterbank    mfcc.c:133-234 (hz_to_mel 1127 ln(1+f/700) with f=0->1,
 *                     mel_to_hz 700 (10^(m/2595) - 1) -- the reference's own
 *                     mixed definitions -- floor(hz / 31.25) bins, clamps)
 *   apply + log       mfcc.c:275-295, 496-498   ln(max(E, 1e-12))
 *   dct_ii            mfcc.c:20-64   n = 40 > 32: cos-table path, scale after sum
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static float hz_to_mel(float f) {
  if (f == 0) f = 1;
  return 1127.0f * log1pf(f / 700.0f);
}
static float mel_to_hz(float m) { return 700.0f * (powf(10.0f, m / 2595.0f) - 1.0f); }

/* [n_filters][n_fft/2+1] triangle weights (mfcc.c:144-234). */
int esp_mfcc_oracle_fbank(int sr, int n_filters, int n_fft, float* fb) {
  const int nb = n_fft / 2 + 1;
  memset(fb, 0, sizeof(float) * (size_t)n_filters * nb);
  const float lo = hz_to_mel(0.0f), hi = hz_to_mel((float)(sr / 2));
  int* bins = (int*)malloc(sizeof(int) * (n_filters + 2));
  if (!bins) return -1;
  const float bw = (float)sr / n_fft;
  for (int i = 0; i < n_filters + 2; ++i) {
    const float m = lo + i * (hi - lo) / (n_filters + 1);
    bins[i] = (int)floorf(mel_to_hz(m) / bw);
  }
  for (int i = 0; i < n_filters; ++i) {
    int l = bins[i], c = bins[i + 1], r = bins[i + 2];
    l = l < 0 ? 0 : (l >= nb ? nb - 1 : l);
    c = c < 0 ? 0 : (c >= nb ? nb - 1 : c);
    r = r < 0 ? 0 : (r >= nb ? nb - 1 : r);
    if (l >= c) c = l + 1;
    if (c >= r) r = c + 1;
    if (r >= nb) r = nb - 1;
    for (int j = l; j <= c; ++j)
      if (j >= 0 && j < nb) fb[i * nb + j] = (float)(j - l) / (c - l);
    for (int j = c; j <= r; ++j)
      if (j >= 0 && j < nb) fb[i * nb + j] = (float)(r - j) / (r - c);
  }
  free(bins);
  return 0;
}

/* Mode-A MFCC of one signal -> out[n_frames][n_mfcc] (frame-major).
 * Returns n_frames, or -1 on bad arguments / allocation failure.  `pre` is the
 * pre-emphasis coefficient: 0.97 for extract_mfcc (mfcc.c:445), 0 for
 * flow_extract_mfcc_single_frame (mfcc.c:297-427, which has none). */
int esp_mfcc_oracle_ex(const float* x, int L, int sr, int frame, int hop, int n_fft, int n_filters, int n_mfcc,
                       int esp_pack, float pre, float* out) {
  if (!x || !out || L < frame || frame <= 0 || hop <= 0 || n_fft < frame || n_filters <= 0 || n_mfcc <= 0 ||
      n_mfcc > n_filters)
    return -1;
  const int nf = (L - frame) / hop + 1, nb = n_fft / 2 + 1;
  float* y = (float*)malloc(sizeof(float) * L);
  float* win = (float*)malloc(sizeof(float) * frame);
  float* fb = (float*)malloc(sizeof(float) * (size_t)n_filters * nb);
  float* pw = (float*)malloc(sizeof(float) * nb);
  float* mel = (float*)malloc(sizeof(float) * n_filters);
  float* ct = (float*)malloc(sizeof(float) * (size_t)n_filters * n_filters);
  double* cs = (double*)malloc(sizeof(double) * n_fft);
  double* sn = (double*)malloc(sizeof(double) * n_fft);
  float* fr = (float*)malloc(sizeof(float) * frame);
  int rc = nf;
  if (!y || !win || !fb || !pw || !mel || !ct || !cs || !sn || !fr || esp_mfcc_oracle_fbank(sr, n_filters, n_fft, fb)) {
    rc = -1;
    goto done;
  }
  y[0] = x[0];
  for (int i = 1; i < L; ++i) y[i] = x[i] - pre * x[i - 1];
  for (int i = 0; i < frame; ++i) win[i] = 0.53836f - (1.0f - 0.53836f) * cosf(2.0f * M_PI * i / (frame - 1));
  for (int i = 0; i < n_fft; ++i) {
    cs[i] = cos(2.0 * M_PI * i / n_fft);
    sn[i] = sin(2.0 * M_PI * i / n_fft);
  }
  for (int k = 0; k < n_filters; ++k)
    for (int i = 0; i < n_filters; ++i) ct[k * n_filters + i] = cosf(M_PI * k * (2 * i + 1) / (2.0f * n_filters));
  for (int t = 0; t < nf; ++t) {
    for (int j = 0; j < frame; ++j) fr[j] = y[t * hop + j] * win[j];
    for (int k = 0; k < nb; ++k) {
      double re = 0.0, im = 0.0;
      for (int j = 0; j < frame; ++j) {
        const int e = (int)(((long long)j * k) % n_fft);
        re += fr[j] * cs[e];
        im -= fr[j] * sn[e];
      }
      float r = (float)re, m = (float)im;
      if (esp_pack) {
        if (k == nb - 1) r = m = 0.0f;
        else if (k > 0) r *= 2.0f, m *= 2.0f;
      }
      pw[k] = (r * r + m * m) / n_fft + 1e-12f;
    }
    for (int f = 0; f < n_filters; ++f) {
      float e = 0.0f;
      for (int k = 0; k < nb; ++k) e += pw[k] * fb[f * nb + k];
      mel[f] = logf(fmaxf(e, 1e-12f));
    }
    for (int c = 0; c < n_mfcc; ++c) {
      float s = 0.0f;
      for (int i = 0; i < n_filters; ++i) s += mel[i] * ct[c * n_filters + i];
      out[t * n_mfcc + c] = (c == 0 ? sqrtf(1.0f / n_filters) : sqrtf(2.0f / n_filters)) * s;
    }
  }
done:
  free(y); free(win); free(fb); free(pw); free(mel); free(ct); free(cs); free(sn); free(fr);
  return rc;
}

int esp_mfcc_oracle(const float* x, int L, int sr, int frame, int hop, int n_fft, int n_filters, int n_mfcc,
                    int esp_pack, float* out) {
  return esp_mfcc_oracle_ex(x, L, sr, frame, hop, n_fft, n_filters, n_mfcc, esp_pack, 0.97f, out);
}
