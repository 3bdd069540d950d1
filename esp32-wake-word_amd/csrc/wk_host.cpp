// wk_host.cpp -- libwakeword_host.so: the wake-word path on the host CPU
// (include/wakeword_host.h).  Product code for callers without a GPU
// (BASELINE config 1) and for C code written against mfcc.h; it shares no code
// path with libwakeword.so's kernels and never touches HIP, and nothing in the
// GPU library calls it.  The tables come from the same builders the GPU path
// uploads (wk_esp_tables.h for mode A) or from the same definitions (mode B).
//
//   mode A  mfcc.c:431-527 (extract_mfcc) / :297-427 (single frame): pre-emphasis
//           0.97 (:66-74), symmetric Hamming (:110-131), the frame in the first
//           min(frame, n_fft) points of an n_fft-point radix-2 complex FFT
//           (compute_power_spectrum :241-295, esp-dsp's dsps_fft2r_fc32 +
//           dsps_bit_rev_fc32 algorithm), |X|^2 / n_fft + 1e-12 with the
//           dsps_cplx2reC_fc32 packing as a flag, mel (:144-234), ln(max(E,
//           1e-12)) (:290, :496-498), DCT-II (:20-64)
//   mode B  extract_mfcc.py:137-175: torchaudio preemphasis (:171) + MFCC
//           (Spectrogram n_fft 512, win 320, hop 256, periodic Hamming centred
//           in 512, center/reflect, power 2; HTK MelScale 40, no norm;
//           ln(mel + 1e-6); ortho DCT-II, 13) + normalize_mfcc('cmvn') (:47-88)
//   CNN     wakeModel.py:4-34 LightweightKWS, fp32
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "wakeword_host.h"
#include "wk_esp_tables.h"
#include "wk_status.h"

// The error helpers of wk_status.h for this library (wk_wav.cpp reports through them too).
namespace wk {
thread_local std::string g_last_error;
wk_status invalid(const char* what) {
  g_last_error = what;
  return WK_ERR_INVALID_ARG;
}
wk_status fail(wk_status s, const char* what) {
  g_last_error = what;
  return s;
}
}  // namespace wk

namespace {

using wk::fail;

std::atomic<int> g_threads{0};   // 0 = hardware concurrency (atomic: wkh_set_threads may race a batch call)

int n_threads() {
  const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  const int t = g_threads.load(std::memory_order_relaxed);
  return t > 0 ? t : hw;
}

// Run f(begin, end) over [0, n) in contiguous chunks on up to n_threads()
// threads (the calling thread takes the first chunk).
template <class F>
void parallel_for(int64_t n, int64_t min_chunk, const F& f) {
  if (n <= 0) return;
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>(n_threads(), (n + min_chunk - 1) / min_chunk));
  if (nt == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(nt - 1);
  const int64_t per = (n + nt - 1) / nt;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t b = t * per, e = std::min(n, b + per);
    if (b < e) pool.emplace_back([&f, b, e] { f(b, e); });
  }
  f(0, std::min(n, per));
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------------------------
// Radix-2 decimation-in-time complex FFT in float (bit-reversed placement,
// log2 n butterfly stages): the algorithm of esp-dsp's dsps_fft2r_fc32 +
// dsps_bit_rev_fc32, and of the GPU path's wk_esp_mfcc_kernel.
// ---------------------------------------------------------------------------
struct Fft {
  int n = 0, lg = 0;
  std::vector<float> wr, wi;   // per stage s (half = 2^(s-1)): W_{2 half}^k, k < half, at [half - 1 + k]
  std::vector<int> rev;

  explicit Fft(int n_) : n(n_) {
    while ((1 << lg) < n) ++lg;
    wr.resize(n > 1 ? n - 1 : 1);
    wi.resize(n > 1 ? n - 1 : 1);
    for (int half = 1; half < n; half *= 2)
      for (int k = 0; k < half; ++k) {   // W_n^(k * n / (2 half)): the same float values as one W_n table
        const int e = k * (n / (2 * half));
        wr[half - 1 + k] = (float)cos(2.0 * M_PI * e / n);
        wi[half - 1 + k] = (float)-sin(2.0 * M_PI * e / n);
      }
    rev.resize(n);
    for (int j = 0; j < n; ++j) {
      int r = 0;
      for (int b = 0; b < lg; ++b) r |= ((j >> b) & 1) << (lg - 1 - b);
      rev[j] = r;
    }
  }
  // re/im hold the input in bit-reversed slots (place()); the spectrum in natural order on return.
  void place(const float* x, int nx, float* re, float* im) const {
    for (int j = 0; j < n; ++j) {
      re[rev[j]] = j < nx ? x[j] : 0.0f;
      im[rev[j]] = 0.0f;
    }
  }
  void butterflies(float* __restrict__ re, float* __restrict__ im) const {
    for (int half = 1; half < n; half *= 2) {
      const float* __restrict__ w_r = wr.data() + half - 1;
      const float* __restrict__ w_i = wi.data() + half - 1;
      for (int base = 0; base < n; base += 2 * half) {
        float* __restrict__ pr = re + base;
        float* __restrict__ pi = im + base;
        float* __restrict__ qr = re + base + half;
        float* __restrict__ qi = im + base + half;
        for (int k = 0; k < half; ++k) {
          const float tr = qr[k] * w_r[k] - qi[k] * w_i[k], ti = qr[k] * w_i[k] + qi[k] * w_r[k];
          const float a = pr[k], b = pi[k];
          qr[k] = a - tr;
          qi[k] = b - ti;
          pr[k] = a + tr;
          pi[k] = b + ti;
        }
      }
    }
  }
};

const Fft& fft_of(int n) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<Fft>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& p = cache[n];
  if (!p) p.reset(new Fft(n));
  return *p;
}

// ---------------------------------------------------------------------------
// Mode A tables (one parameter set) and one frame's computation.
// ---------------------------------------------------------------------------
struct EspTables {
  int sr, frame, n_fft, n_filters, n_mfcc, nb, n_dct;
  std::vector<float> win, dct, scale;
  std::vector<int> row_lo, row_len;   // sparse mel rows: first bin and length of each row's nonzero (or NaN) span
  std::vector<float> row_w;           // ... their weights, row after row
  std::vector<int> row_off;
};

std::unique_ptr<EspTables> make_esp_tables(int sr, int frame, int n_fft, int n_filters, int n_mfcc) {
  std::unique_ptr<EspTables> t(new EspTables);
  t->sr = sr;
  t->frame = frame;
  t->n_fft = n_fft;
  t->n_filters = n_filters;
  t->n_mfcc = n_mfcc;
  t->nb = n_fft / 2 + 1;
  t->win = wk::esp::window(frame);
  wk::esp::dct(n_mfcc, n_filters, t->dct, t->scale);
  t->n_dct = (int)t->scale.size();
  const std::vector<float> fb = wk::esp::filterbank(sr, n_filters, n_fft);
  for (int f = 0; f < n_filters; ++f) {
    int lo = -1, hi = -1;
    for (int k = 0; k < t->nb; ++k)
      if (fb[(size_t)f * t->nb + k] != 0.0f) {   // (NaN != 0: kept, as the reference sums it)
        if (lo < 0) lo = k;
        hi = k;
      }
    if (lo < 0) lo = hi = 0;
    t->row_lo.push_back(lo);
    t->row_len.push_back(hi - lo + 1);
    t->row_off.push_back((int)t->row_w.size());
    for (int k = lo; k <= hi; ++k) t->row_w.push_back(fb[(size_t)f * t->nb + k]);
  }
  return t;
}

// Tables cached per parameter set (mfcc.c rebuilds them per call; its single-
// frame variant caches its filterbank, mfcc.c:362-377).
std::shared_ptr<const EspTables> esp_tables(int sr, int frame, int n_fft, int n_filters, int n_mfcc) {
  static std::mutex mu;
  static std::vector<std::shared_ptr<const EspTables>> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& t : cache)
    if (t->sr == sr && t->frame == frame && t->n_fft == n_fft && t->n_filters == n_filters && t->n_mfcc == n_mfcc)
      return t;
  if (cache.size() >= 16) cache.erase(cache.begin());   // (a caller's shared_ptr keeps an evicted set alive)
  cache.emplace_back(make_esp_tables(sr, frame, n_fft, n_filters, n_mfcc));
  return cache.back();
}

struct EspScratch {
  std::vector<float> buf, re, im, pw, mel;
  explicit EspScratch(const EspTables& t)
      : buf(t.n_fft), re(t.n_fft), im(t.n_fft), pw(t.nb), mel(t.n_filters) {}
};

// Frame t of signal x (length L) -> out[n_mfcc].
void esp_frame(const EspTables& t, const Fft& F, const float* x, int t0, float pre, int esp_pack, EspScratch& s,
               float* out) {
  const int fl = std::min(t.frame, t.n_fft);
  for (int j = 0; j < fl; ++j) {
    const int i = t0 + j;
    const float y = i == 0 ? x[0] : x[i] - pre * x[i - 1];   // mfcc.c:66-74 (y[0] = x[0])
    s.buf[j] = y * t.win[j];
  }
  F.place(s.buf.data(), fl, s.re.data(), s.im.data());
  F.butterflies(s.re.data(), s.im.data());
  for (int k = 0; k < t.nb; ++k) {
    float r = s.re[k], m = s.im[k];
    if (esp_pack) {   // dsps_cplx2reC_fc32: bins 1..n/2-1 doubled, bin n/2 zero
      if (k == t.nb - 1) r = m = 0.0f;
      else if (k > 0) r *= 2.0f, m *= 2.0f;
    }
    s.pw[k] = (r * r + m * m) / (float)t.n_fft + 1e-12f;
  }
  for (int f = 0; f < t.n_filters; ++f) {
    const float* w = t.row_w.data() + t.row_off[f];
    const float* p = s.pw.data() + t.row_lo[f];
    float e = 0.0f;
    for (int j = 0; j < t.row_len[f]; ++j) e += p[j] * w[j];
    s.mel[f] = logf(fmaxf(e, 1e-12f));   // (fmaxf drops a NaN energy, as the reference's max does)
  }
  for (int c = 0; c < t.n_mfcc; ++c) {
    float v = 0.0f;
    if (c < t.n_dct) {
      const float* ct = t.dct.data() + (size_t)c * t.n_filters;
      for (int i = 0; i < t.n_filters; ++i) v += s.mel[i] * ct[i];
      v *= t.scale[c];
    }
    out[c] = v;   // coefficients past n_filters stay 0 (mfcc.c's calloc)
  }
}

wk_status esp_run(const float* signal, int64_t batch, int32_t L, int64_t stride, int32_t sr, int32_t frame,
                  int32_t hop, int32_t n_fft, int32_t n_filters, int32_t n_mfcc, int32_t esp_pack, float pre,
                  float* out) {
  if (wk::esp::check_domain(sr, frame, n_fft, n_filters, n_mfcc) < 0)
    return fail(WK_ERR_INVALID_ARG, "wkh_esp_mfcc: parameters outside mfcc.c's domain (n_fft a power of 2 in "
                                    "[2, 4096], 1 <= n_filters <= 1024, frame_size, n_mfcc, sampling_rate >= 1)");
  if (batch < 0 || L < frame || hop < 1 || (batch > 1 && stride < 1))
    return fail(WK_ERR_INVALID_ARG, "wkh_esp_mfcc: bad sizes (signal_len >= frame_size, hop_size >= 1)");
  if (batch > 0 && (!signal || !out)) return fail(WK_ERR_INVALID_ARG, "wkh_esp_mfcc: null pointer");
  if (batch == 0) return WK_OK;
  const std::shared_ptr<const EspTables> tp = esp_tables(sr, frame, n_fft, n_filters, n_mfcc);
  const EspTables& tab = *tp;
  const Fft& F = fft_of(n_fft);
  const int nf = (L - frame) / hop + 1;
  parallel_for(batch * nf, 64, [&](int64_t b, int64_t e) {
    EspScratch s(tab);
    for (int64_t u = b; u < e; ++u) {
      const int64_t clip = u / nf;
      const int t = (int)(u - clip * nf);
      esp_frame(tab, F, signal + clip * stride, t * hop, pre, esp_pack, s, out + u * n_mfcc);
    }
  });
  return WK_OK;
}

// ---------------------------------------------------------------------------
// Mode B (torchaudio MFCC + CMVN) at the xiaoa geometry.
// ---------------------------------------------------------------------------
constexpr int kN = 16000, kNfft = 512, kWin = 320, kHop = 256, kMels = 40, kMfcc = 13, kFrames = 63, kBins = 257;

struct ModeBTables {
  float win[kWin];                // periodic Hamming(320) (torch.hamming_window, periodic=True)
  float wsr[kBins], wsi[kBins];   // real-FFT split twiddles W512^k
  int mel_lo[kMels], mel_len[kMels];
  std::vector<float> mel_w[kMels];   // HTK triangles (MelScale, norm=None), nonzero span per filter
  float dct[kMfcc][kMels];        // create_dct(13, 40, norm='ortho')
  ModeBTables() {
    for (int n = 0; n < kWin; ++n) win[n] = (float)(0.54 - 0.46 * cos(2.0 * M_PI * n / kWin));
    for (int k = 0; k < kBins; ++k) {
      wsr[k] = (float)cos(2.0 * M_PI * k / kNfft);
      wsi[k] = (float)-sin(2.0 * M_PI * k / kNfft);
    }
    // melscale_fbanks(257, 0, 8000, 40, 16000, norm=None, mel_scale='htk')
    auto h2m = [](double f) { return 2595.0 * log10(1.0 + f / 700.0); };
    auto m2h = [](double m) { return 700.0 * (pow(10.0, m / 2595.0) - 1.0); };
    double fpt[kMels + 2];
    const double m0 = h2m(0.0), m1 = h2m(8000.0);
    for (int i = 0; i < kMels + 2; ++i) fpt[i] = m2h(m0 + (m1 - m0) * i / (kMels + 1));
    for (int m = 0; m < kMels; ++m) {
      std::vector<float> row(kBins);
      int lo = -1, hi = -1;
      for (int k = 0; k < kBins; ++k) {
        const double f = 8000.0 * k / (kBins - 1);
        const double down = (fpt[m + 2] - f) / (fpt[m + 2] - fpt[m + 1]);
        const double up = (f - fpt[m]) / (fpt[m + 1] - fpt[m]);
        const double v = std::max(0.0, std::min(down, up));
        row[k] = (float)v;
        if (v > 0.0) {
          if (lo < 0) lo = k;
          hi = k;
        }
      }
      if (lo < 0) lo = hi = 0;
      mel_lo[m] = lo;
      mel_len[m] = hi - lo + 1;
      mel_w[m].assign(row.begin() + lo, row.begin() + hi + 1);
    }
    for (int k = 0; k < kMfcc; ++k)
      for (int n = 0; n < kMels; ++n)
        dct[k][n] = (float)(cos(M_PI / kMels * (n + 0.5) * k) * sqrt(2.0 / kMels) * (k == 0 ? 1.0 / sqrt(2.0) : 1.0));
  }
};

const ModeBTables& mode_b_tables() {
  static const ModeBTables t;
  return t;
}

struct ModeBScratch {
  float y[kN];
  float re[kNfft / 2], im[kNfft / 2], z[kNfft];
  float pw[kBins];
  float mf[kMfcc][kFrames];
};

// One clip (16000 samples) -> feats[13][63].
void mode_b_clip(const ModeBTables& T, const Fft& F256, const float* x, int cmvn, ModeBScratch& s, float* feats) {
  // torchaudio.functional.preemphasis: y[i] = x[i] - 0.97 x[i-1], y[0] = x[0]
  s.y[0] = x[0];
  for (int i = 1; i < kN; ++i) s.y[i] = x[i] - 0.97f * x[i - 1];
  for (int t = 0; t < kFrames; ++t) {
    // frame t of the reflect-padded signal: samples 256 t - 160 + n, n < 320,
    // under the window (its 96-sample centring offset in the 512 is a circular
    // shift, a pure phase: |X|^2 is unchanged)
    const int i0 = kHop * t + (kNfft - kWin) / 2 - kNfft / 2;   // = 256 t - 160
    for (int n = 0; n < kWin; ++n) {
      int i = i0 + n;
      i = i < 0 ? -i : i;
      i = i > kN - 1 ? 2 * (kN - 1) - i : i;
      s.z[n] = s.y[i] * T.win[n];
    }
    // 512-point real FFT as a 256-point complex FFT of the (even, odd) pairs + the split
    for (int m = 0; m < kNfft / 2; ++m) {
      const int r = F256.rev[m];
      s.re[r] = 2 * m < kWin ? s.z[2 * m] : 0.0f;
      s.im[r] = 2 * m + 1 < kWin ? s.z[2 * m + 1] : 0.0f;
    }
    F256.butterflies(s.re, s.im);
    for (int k = 0; k <= kNfft / 2; ++k) {
      const int a = k & (kNfft / 2 - 1), b = (kNfft / 2 - k) & (kNfft / 2 - 1);
      const float zr = s.re[a], zi = s.im[a], cr = s.re[b], ci = -s.im[b];   // Z[k], conj Z[256 - k]
      const float er = 0.5f * (zr + cr), ei = 0.5f * (zi + ci);              // even part
      const float dr = 0.5f * (zr - cr), di = 0.5f * (zi - ci);              // odd part times i
      // X[k] = E + W^k (-i) D
      const float odr = di, odi = -dr;
      const float xr = er + T.wsr[k] * odr - T.wsi[k] * odi, xi = ei + T.wsr[k] * odi + T.wsi[k] * odr;
      s.pw[k] = xr * xr + xi * xi;
    }
    float lm[kMels];
    for (int m = 0; m < kMels; ++m) {
      const float* w = T.mel_w[m].data();
      const float* p = s.pw + T.mel_lo[m];
      float e = 0.0f;
      for (int j = 0; j < T.mel_len[m]; ++j) e += p[j] * w[j];
      lm[m] = logf(e + 1e-6f);
    }
    for (int k = 0; k < kMfcc; ++k) {
      float v = 0.0f;
      for (int m = 0; m < kMels; ++m) v += T.dct[k][m] * lm[m];
      s.mf[k][t] = v;
    }
  }
  for (int k = 0; k < kMfcc; ++k) {
    float* o = feats + k * kFrames;
    if (!cmvn) {
      memcpy(o, s.mf[k], sizeof(float) * kFrames);
      continue;
    }
    // normalize_mfcc('cmvn'): mean, unbiased std, std == 0 -> 1, (x - mean) / (std + 1e-8)
    double mean = 0.0;
    for (int t = 0; t < kFrames; ++t) mean += s.mf[k][t];
    mean /= kFrames;
    double var = 0.0;
    for (int t = 0; t < kFrames; ++t) var += (s.mf[k][t] - mean) * (s.mf[k][t] - mean);
    double sd = sqrt(var / (kFrames - 1));
    if (sd == 0.0) sd = 1.0;
    const double inv = 1.0 / (sd + 1e-8);
    for (int t = 0; t < kFrames; ++t) o[t] = (float)((s.mf[k][t] - mean) * inv);
  }
}

// ---------------------------------------------------------------------------
// LightweightKWS (wakeModel.py:4-34), fp32.
// ---------------------------------------------------------------------------
struct CnnScratch {
  float a0[kMfcc][kFrames + 2];   // conv1 input, zero guards at t = -1 and t = 63
  float c1[32][kFrames];
  float a1[32][31 + 2];
  float c2[64][31];
  float a2[64][15 + 2];
  float c3[128][15];
};

// conv1d(k3, p1, no bias) over guarded rows x[ci][0..T+1] (x[ci][t+1] = input t) -> y[co][T]
template <int CI, int CO, int T, int XP>
void conv_k3(const float* w, const float (*x)[XP], float (*y)[T]) {
  for (int co = 0; co < CO; ++co) {
    float acc[T] = {};
    for (int ci = 0; ci < CI; ++ci) {
      const float w0 = w[(co * CI + ci) * 3], w1 = w[(co * CI + ci) * 3 + 1], w2 = w[(co * CI + ci) * 3 + 2];
      const float* r = x[ci];
      for (int t = 0; t < T; ++t) acc[t] += w0 * r[t] + w1 * r[t + 1] + w2 * r[t + 2];
    }
    memcpy(y[co], acc, sizeof(acc));
  }
}

// ReLU -> maxpool(2) (floor) into guarded rows
template <int C, int T, int TP>
void relu_pool(const float (*y)[T], float (*o)[TP]) {
  for (int c = 0; c < C; ++c) {
    o[c][0] = 0.0f;
    for (int p = 0; p < T / 2; ++p) o[c][p + 1] = std::max(0.0f, std::max(y[c][2 * p], y[c][2 * p + 1]));
    o[c][T / 2 + 1] = 0.0f;
  }
}

float cnn_clip(const float* w, const float* feats, CnnScratch& s) {
  const float* w1 = w;                     // [32][13][3]
  const float* w2 = w1 + 32 * 13 * 3;      // [64][32][3]
  const float* w3 = w2 + 64 * 32 * 3;      // [128][64][3]
  const float* f1 = w3 + 128 * 64 * 3;     // [64][128]
  const float* f2 = f1 + 64 * 128;         // [1][64]
  for (int c = 0; c < kMfcc; ++c) {
    s.a0[c][0] = 0.0f;
    memcpy(&s.a0[c][1], feats + c * kFrames, sizeof(float) * kFrames);
    s.a0[c][kFrames + 1] = 0.0f;
  }
  conv_k3<13, 32, 63, kFrames + 2>(w1, s.a0, s.c1);
  relu_pool<32, 63, 33>(s.c1, s.a1);
  conv_k3<32, 64, 31, 33>(w2, s.a1, s.c2);
  relu_pool<64, 31, 17>(s.c2, s.a2);
  conv_k3<64, 128, 15, 17>(w3, s.a2, s.c3);
  float g[128];
  for (int c = 0; c < 128; ++c) {   // ReLU -> maxpool(2) 15 -> 7 -> AdaptiveAvgPool1d(1)
    float sum = 0.0f;
    for (int p = 0; p < 7; ++p) sum += std::max(0.0f, std::max(s.c3[c][2 * p], s.c3[c][2 * p + 1]));
    g[c] = sum / 7.0f;
  }
  float logit = 0.0f;
  for (int o = 0; o < 64; ++o) {   // classifier.0 (128 -> 64) + ReLU, classifier.2 (64 -> 1)
    float h = 0.0f;
    for (int k = 0; k < 128; ++k) h += f1[o * 128 + k] * g[k];
    logit += f2[o] * std::max(h, 0.0f);
  }
  return logit;
}

wk_status check_b(const float* audio, int64_t batch, int32_t win_len, int64_t stride, const void* out) {
  if (batch < 0) return fail(WK_ERR_INVALID_ARG, "batch < 0");
  if (win_len != kN) return fail(WK_ERR_INVALID_ARG, "mode B (torchaudio+CMVN) requires win_len == 16000");
  if (batch > 1 && stride < 1) return fail(WK_ERR_INVALID_ARG, "stride < 1");
  if (batch > 0 && (!audio || !out)) return fail(WK_ERR_INVALID_ARG, "null pointer");
  return WK_OK;
}

}  // namespace

struct wkh_model {
  std::vector<float> w;
};

extern "C" {

wk_status wkh_create(const float* weights, wkh_model** out) {
  if (!out) return fail(WK_ERR_INVALID_ARG, "wkh_create: null out");
  *out = nullptr;
  if (!weights) return fail(WK_ERR_INVALID_ARG, "wkh_create: null weights");
  wkh_model* m = new (std::nothrow) wkh_model;
  if (!m) return fail(WK_ERR_NO_MEMORY, "wkh_create: out of memory");
  m->w.assign(weights, weights + WK_NUM_WEIGHTS);
  *out = m;
  return WK_OK;
}

wk_status wkh_destroy(wkh_model* m) {
  delete m;
  return WK_OK;
}

wk_status wkh_mfcc(const float* audio, int64_t batch, int32_t win_len, int64_t stride, int32_t cmvn, float* feats) {
  const wk_status st = check_b(audio, batch, win_len, stride, feats);
  if (st != WK_OK) return st;
  const ModeBTables& T = mode_b_tables();
  const Fft& F = fft_of(kNfft / 2);
  parallel_for(batch, 4, [&](int64_t b, int64_t e) {
    std::unique_ptr<ModeBScratch> s(new ModeBScratch);
    for (int64_t i = b; i < e; ++i) mode_b_clip(T, F, audio + i * stride, cmvn, *s, feats + i * kMfcc * kFrames);
  });
  return WK_OK;
}

wk_status wkh_cnn(const wkh_model* m, const float* feats, int64_t batch, float* logits) {
  if (!m) return fail(WK_ERR_INVALID_ARG, "wkh_cnn: null model");
  if (batch < 0 || (batch > 0 && (!feats || !logits))) return fail(WK_ERR_INVALID_ARG, "wkh_cnn: bad arguments");
  parallel_for(batch, 4, [&](int64_t b, int64_t e) {
    std::unique_ptr<CnnScratch> s(new CnnScratch);
    for (int64_t i = b; i < e; ++i) logits[i] = cnn_clip(m->w.data(), feats + i * kMfcc * kFrames, *s);
  });
  return WK_OK;
}

wk_status wkh_forward(const wkh_model* m, const float* audio, int64_t batch, int32_t win_len, int64_t stride,
                      float* logits, float* feats_or_null) {
  if (!m) return fail(WK_ERR_INVALID_ARG, "wkh_forward: null model");
  const wk_status st = check_b(audio, batch, win_len, stride, logits);
  if (st != WK_OK) return st;
  const ModeBTables& T = mode_b_tables();
  const Fft& F = fft_of(kNfft / 2);
  parallel_for(batch, 4, [&](int64_t b, int64_t e) {
    std::unique_ptr<ModeBScratch> s(new ModeBScratch);
    std::unique_ptr<CnnScratch> c(new CnnScratch);
    float f[kMfcc * kFrames];
    for (int64_t i = b; i < e; ++i) {
      float* fi = feats_or_null ? feats_or_null + i * kMfcc * kFrames : f;
      mode_b_clip(T, F, audio + i * stride, 1, *s, fi);
      logits[i] = cnn_clip(m->w.data(), fi, *c);
    }
  });
  return WK_OK;
}

wk_status wkh_esp_mfcc(const float* signal, int64_t batch, int32_t signal_len, int64_t stride, int32_t sampling_rate,
                       int32_t frame_size, int32_t hop_size, int32_t n_fft, int32_t n_filters, int32_t n_mfcc,
                       int32_t esp_dsp_packing, float pre_emphasis, float* out) {
  return esp_run(signal, batch, signal_len, stride, sampling_rate, frame_size, hop_size, n_fft, n_filters, n_mfcc,
                 esp_dsp_packing ? 1 : 0, pre_emphasis, out);
}

int32_t wkh_set_threads(int32_t n) {
  if (n >= 0) g_threads.store(n, std::memory_order_relaxed);
  return n_threads();
}

const char* wkh_last_error(void) { return wk::g_last_error.c_str(); }

// ---------------------------------------------------------------------------
// mfcc.h (main/esp_mfcc/mfcc.h:10-17) on the host: same signatures, ownership
// (malloc'd block, free_mfcc) and NULL-on-error behaviour as mfcc.c, with
// esp-dsp's packing on (what mfcc.c runs).
// ---------------------------------------------------------------------------
float* extract_mfcc(const float* signal, int signal_len, int sampling_rate, int frame_size, int hop_size, int n_fft,
                    int n_filters, int n_mfcc) {
  if (!signal || signal_len < frame_size || frame_size <= 0) {   // mfcc.c:434-437
    fprintf(stderr, "E (MFCC) Invalid signal parameters\n");
    return nullptr;
  }
  if (hop_size < 1) {   // (mfcc.c:447 divides by it)
    fprintf(stderr, "E (MFCC) Invalid hop size\n");
    return nullptr;
  }
  if (wk::esp::check_domain(sampling_rate, frame_size, n_fft, n_filters, n_mfcc) < 0) {
    fprintf(stderr, "E (MFCC) unsupported configuration\n");
    return nullptr;
  }
  const int nf = (signal_len - frame_size) / hop_size + 1;
  float* out = (float*)malloc(sizeof(float) * (size_t)nf * n_mfcc);
  if (!out) {
    fprintf(stderr, "E (MFCC) Memory allocation failed\n");
    return nullptr;
  }
  if (esp_run(signal, 1, signal_len, signal_len, sampling_rate, frame_size, hop_size, n_fft, n_filters, n_mfcc, 1,
              0.97f, out) != WK_OK) {
    fprintf(stderr, "E (MFCC) %s\n", wk::g_last_error.c_str());
    free(out);
    return nullptr;
  }
  return out;
}

void free_mfcc(float* mfcc) { free(mfcc); }

// mfcc.c:297-427: one frame, no pre-emphasis -> malloc'd n_mfcc floats.
float* flow_extract_mfcc_single_frame(const float* frame, int frame_size, int sampling_rate, int n_fft, int n_filters,
                                      int n_mfcc) {
  if (!frame || frame_size <= 0 || frame_size > n_fft) {   // mfcc.c:300-303
    fprintf(stderr, "E (MFCC) Invalid frame parameters\n");
    return nullptr;
  }
  if (n_mfcc < 1 || wk::esp::check_domain(sampling_rate, frame_size, n_fft, n_filters, n_mfcc) < 0) {
    fprintf(stderr, "E (MFCC) unsupported configuration\n");
    return nullptr;
  }
  float* out = (float*)malloc(sizeof(float) * (size_t)n_mfcc);
  if (!out) return nullptr;
  if (esp_run(frame, 1, frame_size, frame_size, sampling_rate, frame_size, frame_size, n_fft, n_filters, n_mfcc, 1,
              0.0f, out) != WK_OK) {
    free(out);
    return nullptr;
  }
  return out;
}

// mfcc.c:530-553: min/max/avg over the finite entries.
void analyze_mfcc_range(float* mfcc, int size, const char* label) {
  if (!mfcc || size <= 0) return;
  float mn = INFINITY, mx = -INFINITY, sum = 0.0f;
  int valid = 0;
  for (int i = 0; i < size; i++) {
    if (!isnan(mfcc[i]) && !isinf(mfcc[i])) {
      mn = std::min(mn, mfcc[i]);
      mx = std::max(mx, mfcc[i]);
      sum += mfcc[i];
      valid++;
    }
  }
  if (valid > 0)
    printf("I (MFCC) %s MFCC Range: min=%.6f, max=%.6f, avg=%.6f, valid=%d/%d\n", label ? label : "", mn, mx,
           sum / valid, valid, size);
  else
    fprintf(stderr, "E (MFCC) %s MFCC: No valid values\n", label ? label : "");
  fflush(stdout);
}

}  // extern "C"
