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
 *
 * esp_mfcc_oracle_batch is the same computation with a float radix-2 FFT in
 * place of the exact DFT (esp-dsp's dsps_fft2r_fc32 is an in-place radix-2
 * decimation-in-time FFT with a bit-reversal pass: restated from its published
 * algorithm, not its source), sparse mel rows and a thread pool: the timed
 * mode-A CPU baseline SURVEY 8(d) asks for (bench_surfaces.py).  It agrees
 * with the DFT path to float rounding (tests/test_oracle_fft.py).
 */
#include <math.h>
#include <pthread.h>
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
  if (!x || !out || L < frame || frame <= 0 || hop <= 0 || n_fft <= 0 || n_filters <= 0 || n_mfcc <= 0) return -1;
  /* compute_power_spectrum (mfcc.c:252) copies only the first n_fft samples of
   * a longer frame; dct_ii fills n_filters coefficients and extract_mfcc's
   * calloc leaves any further ones 0 (mfcc.c:514-517) */
  const int fl = frame < n_fft ? frame : n_fft;
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
      for (int j = 0; j < fl; ++j) {
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
      if (c >= n_filters) {
        out[t * n_mfcc + c] = 0.0f;
        continue;
      }
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

/* ---- FFT-based batch path (timed CPU baseline) ---------------------------- */
typedef struct {
  int sr, frame, hop, n_fft, n_filters, n_mfcc, esp_pack, log2n;
  float pre;
  float *win, *twr, *twi, *ct;   /* window, twiddles W^k (k < n_fft/2), DCT table */
  int *rev;                      /* bit reversal */
  int *fb_lo, *fb_n;             /* sparse mel rows: first bin, count */
  float* fb_w;                   /* their weights, row after row */
} mfcc_ctx;

static void ctx_free(mfcc_ctx* c) {
  free(c->win); free(c->twr); free(c->twi); free(c->ct); free(c->rev); free(c->fb_lo); free(c->fb_n); free(c->fb_w);
}

static int ctx_init(mfcc_ctx* c, int sr, int frame, int hop, int n_fft, int n_filters, int n_mfcc, int esp_pack,
                    float pre) {
  memset(c, 0, sizeof(*c));
  int lg = 0;
  while ((1 << lg) < n_fft) ++lg;
  if ((1 << lg) != n_fft || frame > n_fft || n_mfcc > n_filters) return -1;
  c->sr = sr; c->frame = frame; c->hop = hop; c->n_fft = n_fft; c->n_filters = n_filters; c->n_mfcc = n_mfcc;
  c->esp_pack = esp_pack; c->pre = pre; c->log2n = lg;
  const int nb = n_fft / 2 + 1;
  c->win = (float*)malloc(sizeof(float) * frame);
  c->twr = (float*)malloc(sizeof(float) * (n_fft / 2));
  c->twi = (float*)malloc(sizeof(float) * (n_fft / 2));
  c->ct = (float*)malloc(sizeof(float) * (size_t)n_filters * n_filters);
  c->rev = (int*)malloc(sizeof(int) * n_fft);
  c->fb_lo = (int*)malloc(sizeof(int) * n_filters);
  c->fb_n = (int*)malloc(sizeof(int) * n_filters);
  float* fb = (float*)malloc(sizeof(float) * (size_t)n_filters * nb);
  c->fb_w = (float*)malloc(sizeof(float) * (size_t)n_filters * nb);
  if (!c->win || !c->twr || !c->twi || !c->ct || !c->rev || !c->fb_lo || !c->fb_n || !fb || !c->fb_w ||
      esp_mfcc_oracle_fbank(sr, n_filters, n_fft, fb)) {
    free(fb);
    ctx_free(c);
    return -1;
  }
  for (int i = 0; i < frame; ++i) c->win[i] = 0.53836f - (1.0f - 0.53836f) * cosf(2.0f * M_PI * i / (frame - 1));
  for (int k = 0; k < n_fft / 2; ++k) {
    c->twr[k] = (float)cos(2.0 * M_PI * k / n_fft);
    c->twi[k] = (float)-sin(2.0 * M_PI * k / n_fft);
  }
  for (int i = 0; i < n_fft; ++i) {
    int r = 0;
    for (int b = 0; b < lg; ++b) r |= ((i >> b) & 1) << (lg - 1 - b);
    c->rev[i] = r;
  }
  for (int k = 0; k < n_filters; ++k)
    for (int i = 0; i < n_filters; ++i) c->ct[k * n_filters + i] = cosf(M_PI * k * (2 * i + 1) / (2.0f * n_filters));
  int w = 0;
  for (int f = 0; f < n_filters; ++f) {
    int lo = -1, hi = -1;
    for (int k = 0; k < nb; ++k)
      if (fb[f * nb + k] != 0.0f) { if (lo < 0) lo = k; hi = k; }
    if (lo < 0) lo = hi = 0;
    c->fb_lo[f] = lo;
    c->fb_n[f] = hi - lo + 1;
    for (int k = lo; k <= hi; ++k) c->fb_w[w++] = fb[f * nb + k];
  }
  free(fb);
  return 0;
}

/* One clip -> out[n_frames][n_mfcc]; re/im: n_fft scratch each. */
static int clip_mfcc(const mfcc_ctx* c, const float* x, int L, float* re, float* im, float* pw, float* mel, float* out) {
  const int n = c->n_fft, nb = n / 2 + 1, nf = (L - c->frame) / c->hop + 1;
  for (int t = 0; t < nf; ++t) {
    const int s0 = t * c->hop;
    memset(re, 0, sizeof(float) * n);
    memset(im, 0, sizeof(float) * n);
    for (int j = 0; j < c->frame; ++j) {   /* pre-emphasis on the fly, window, bit-reversed placement */
      const int i = s0 + j;
      const float y = i == 0 ? x[0] : x[i] - c->pre * x[i - 1];
      re[c->rev[j]] = y * c->win[j];
    }
    for (int len = 2; len <= n; len <<= 1) {   /* radix-2 DIT butterflies */
      const int half = len >> 1, step = n / len;
      for (int b = 0; b < n; b += len)
        for (int k = 0; k < half; ++k) {
          const float wr = c->twr[k * step], wi = c->twi[k * step];
          const int p = b + k, q = p + half;
          const float tr = re[q] * wr - im[q] * wi, ti = re[q] * wi + im[q] * wr;
          re[q] = re[p] - tr; im[q] = im[p] - ti;
          re[p] += tr; im[p] += ti;
        }
    }
    for (int k = 0; k < nb; ++k) {
      float r = re[k], m = im[k];
      if (c->esp_pack) {
        if (k == nb - 1) r = m = 0.0f;
        else if (k > 0) r *= 2.0f, m *= 2.0f;
      }
      pw[k] = (r * r + m * m) / n + 1e-12f;
    }
    const float* w = c->fb_w;
    for (int f = 0; f < c->n_filters; ++f) {
      float e = 0.0f;
      for (int j = 0; j < c->fb_n[f]; ++j) e += pw[c->fb_lo[f] + j] * w[j];
      w += c->fb_n[f];
      mel[f] = logf(fmaxf(e, 1e-12f));
    }
    for (int q = 0; q < c->n_mfcc; ++q) {
      float s = 0.0f;
      for (int i = 0; i < c->n_filters; ++i) s += mel[i] * c->ct[q * c->n_filters + i];
      out[t * c->n_mfcc + q] = (q == 0 ? sqrtf(1.0f / c->n_filters) : sqrtf(2.0f / c->n_filters)) * s;
    }
  }
  return nf;
}

typedef struct {
  const mfcc_ctx* c;
  const float* x;
  long long first, count, stride;
  int L, nf;
  float* out;
  int rc;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  const int n = j->c->n_fft;
  float* sc = (float*)malloc(sizeof(float) * (2 * n + n / 2 + 1 + j->c->n_filters));
  if (!sc) { j->rc = -1; return NULL; }
  for (long long i = j->first; i < j->first + j->count; ++i)
    clip_mfcc(j->c, j->x + i * j->stride, j->L, sc, sc + n, sc + 2 * n, sc + 2 * n + n / 2 + 1,
              j->out + i * (long long)j->nf * j->c->n_mfcc);
  free(sc);
  j->rc = 0;
  return NULL;
}

/* Mode-A MFCC of n_clips signals (clip i at x + i*stride, L samples) ->
 * out[n_clips][n_frames][n_mfcc] on n_threads host threads.  Returns n_frames,
 * or -1. */
int esp_mfcc_oracle_batch(const float* x, long long n_clips, int L, long long stride, int sr, int frame, int hop,
                          int n_fft, int n_filters, int n_mfcc, int esp_pack, float pre, int n_threads, float* out) {
  if (!x || !out || n_clips < 0 || L < frame || frame <= 0 || hop <= 0 || n_threads < 1) return -1;
  mfcc_ctx c;
  if (ctx_init(&c, sr, frame, hop, n_fft, n_filters, n_mfcc, esp_pack, pre)) return -1;
  const int nf = (L - frame) / hop + 1;
  if (n_threads > n_clips) n_threads = n_clips > 0 ? (int)n_clips : 1;
  batch_job* jobs = (batch_job*)calloc((size_t)n_threads, sizeof(batch_job));
  pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
  int rc = nf;
  if (!jobs || !th) rc = -1;
  for (int t = 0; t < n_threads && rc >= 0; ++t) {
    const long long a = n_clips * t / n_threads, b = n_clips * (t + 1) / n_threads;
    jobs[t] = (batch_job){&c, x, a, b - a, stride, L, nf, out, -1};
    if (t > 0 && pthread_create(&th[t], NULL, batch_worker, &jobs[t])) { jobs[t].rc = -1; th[t] = 0; }
  }
  if (rc >= 0) {
    batch_worker(&jobs[0]);
    for (int t = 1; t < n_threads; ++t)
      if (th[t]) pthread_join(th[t], NULL);
    for (int t = 0; t < n_threads; ++t)
      if (jobs[t].rc) rc = -1;
  }
  free(jobs);
  free(th);
  ctx_free(&c);
  return rc;
}
