// wk_esp_mfcc.hip -- mode A (main/esp_mfcc/mfcc.c) at any parameter set.
//
// The fixed-geometry mode-A path (wk_frontend.hip: 320-sample frames, hop 256,
// 512-point FFT, 40 filters, 13 coefficients) backs wk_mfcc and the
// reference configuration of the mfcc.h shims.  mfcc.c itself takes any
// sampling rate, frame, hop, n_fft, n_filters and n_mfcc and rebuilds its
// tables per call (create_mel_filterbank :144-234, the window :110-131, the
// DCT table :37-52).  This file is that general form on the GPU:
//   host    the per-configuration tables, built once per wk_esp_mfcc object
//           with the reference's own float formulas (mel triangles on
//           floor(hz / bin_width) bins with its clamps, the symmetric Hamming
//           window alpha 0.53836, the DCT-II cosines and scales);
//   device  one workgroup per frame (grid-stride over clips x frames):
//           pre-emphasis (mfcc.c:66-74) and window on the load, frame in the
//           first min(frame, n_fft) slots of an n_fft-point complex buffer
//           (compute_power_spectrum :251-256, zero tail), radix-2 FFT in LDS
//           (bit-reversed placement, log2 n_fft butterfly stages -- the
//           algorithm of esp-dsp's dsps_fft2r_fc32 + dsps_bit_rev_fc32),
//           power (re^2 + im^2) / n_fft + 1e-12 with the dsps_cplx2reC_fc32
//           packing as a flag (parity unpinned), the mel
//           rows (sparse, NaN weights of degenerate triangles kept: :224's
//           0/0), ln(max(E, 1e-12)) (:290, :496-498), DCT-II (:20-64), the
//           first n_mfcc coefficients (zero past n_filters, as mfcc.c's calloc
//           leaves them).
// Not a hot path: it exists so that a C caller of the drop-in may use any
// parameter set mfcc.c accepts.  Domain: n_fft a power of two in [2, 4096]
// (esp-dsp's FFT refuses other lengths and its default maximum is 4096),
// frame_size >= 1 (samples past n_fft are dropped, as :252 does), hop >= 1,
// 1 <= n_filters <= 1024, n_mfcc >= 1, sampling_rate >= 1.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

#include "wk_esp_tables.h"
#include "wk_kernels.h"

struct wk_esp_mfcc {
  int32_t sr, frame, n_fft, n_filters, n_mfcc, esp_pack, device, log2n;
  float* d_win = nullptr;     // [frame] symmetric Hamming (mfcc.c:118-120)
  float2* d_tw = nullptr;     // [n_fft / 2] W^k = exp(-2 pi i k / n_fft)
  int2* d_rows = nullptr;     // [n_filters] {first weight index, first bin} ...
  int* d_rlen = nullptr;      // [n_filters] ... and the row's length
  float* d_fbw = nullptr;     // the rows' weights, back to back
  float* d_dct = nullptr;     // [min(n_mfcc, n_filters)][n_filters] cosines
  float* d_scale = nullptr;   // [min(n_mfcc, n_filters)] sqrt(1/n), sqrt(2/n)
};

namespace {

constexpr int kEspBlock = 256;

// One frame per workgroup iteration; LDS: re[n], im[n], pw[n/2+1], mel[n_filters].
__global__ __launch_bounds__(kEspBlock) void wk_esp_mfcc_kernel(
    const float* __restrict__ sig, int64_t batch, int L, int64_t stride, int hop, float pre, int frame, int n_fft,
    int log2n, int esp_pack, const float* __restrict__ win, const float2* __restrict__ tw, const int2* __restrict__ rows,
    const int* __restrict__ rlen, const float* __restrict__ fbw, int n_filters, const float* __restrict__ dct,
    const float* __restrict__ scale, int n_mfcc, int nf, float* __restrict__ out) {
  extern __shared__ float sm[];
  float* re = sm;
  float* im = re + n_fft;
  float* pw = im + n_fft;
  float* mel = pw + (n_fft / 2 + 1);
  const int tid = threadIdx.x, nb = n_fft / 2 + 1, fl = min(frame, n_fft);
  const int n_dct = min(n_mfcc, n_filters);
  for (int64_t u = blockIdx.x; u < batch * nf; u += gridDim.x) {
    const int64_t clip = u / nf;
    const int t = (int)(u - clip * nf);
    const float* x = sig + clip * stride;
    const int s0 = t * hop;
    // pre-emphasised (y[0] = x[0]), windowed samples in bit-reversed slots; zero tail
    for (int j = tid; j < n_fft; j += kEspBlock) {
      const int slot = (int)(__brev((unsigned)j) >> (32 - log2n));
      float v = 0.0f;
      if (j < fl) {
        const int i = s0 + j;
        const float y = i == 0 ? x[0] : x[i] - pre * x[i - 1];
        v = y * win[j];
      }
      re[slot] = v;
      im[slot] = 0.0f;
    }
    __syncthreads();
    // radix-2 decimation-in-time butterflies, stage by stage
    for (int s = 1; s <= log2n; ++s) {
      const int half = 1 << (s - 1), step = n_fft >> s;
      for (int b = tid; b < n_fft / 2; b += kEspBlock) {
        const int k = b & (half - 1), p = ((b >> (s - 1)) << s) + k, q = p + half;
        const float2 w = tw[k * step];
        const float tr = re[q] * w.x - im[q] * w.y, ti = re[q] * w.y + im[q] * w.x;
        const float pr = re[p], pi = im[p];
        re[q] = pr - tr;
        im[q] = pi - ti;
        re[p] = pr + tr;
        im[p] = pi + ti;
      }
      __syncthreads();
    }
    // power spectrum (mfcc.c:264-270) with the cplx2reC packing flag
    for (int k = tid; k < nb; k += kEspBlock) {
      float r = re[k], m = im[k];
      if (esp_pack) {
        if (k == nb - 1) r = m = 0.0f;
        else if (k > 0) r *= 2.0f, m *= 2.0f;
      }
      pw[k] = (r * r + m * m) / (float)n_fft + 1e-12f;
    }
    __syncthreads();
    // mel rows: E = sum_k pw[k] fb[f][k]; ln(max(E, 1e-12)) (fmaxf drops a NaN E, as the reference's does)
    for (int f = tid; f < n_filters; f += kEspBlock) {
      const int2 rw = rows[f];
      const int n = rlen[f];
      float e = 0.0f;
      for (int j = 0; j < n; ++j) e += pw[rw.y + j] * fbw[rw.x + j];
      mel[f] = logf(fmaxf(e, 1e-12f));
    }
    __syncthreads();
    // DCT-II (mfcc.c:20-64): scale after the sum; coefficients past n_filters stay 0
    float* o = out + u * (int64_t)n_mfcc;
    for (int c = tid; c < n_mfcc; c += kEspBlock) {
      float s = 0.0f;
      if (c < n_dct) {
        const float* ct = dct + (size_t)c * n_filters;
        for (int i = 0; i < n_filters; ++i) s += mel[i] * ct[i];
        s *= scale[c];
      }
      o[c] = s;
    }
    __syncthreads();
  }
}

template <typename T>
hipError_t upload(T** d, const std::vector<T>& h) {
  hipError_t e = hipMalloc(d, sizeof(T) * (h.empty() ? 1 : h.size()));
  if (e != hipSuccess) return e;
  return h.empty() ? hipSuccess : hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice);
}

void free_tables(wk_esp_mfcc* m) {
  for (void* p : {(void*)m->d_win, (void*)m->d_tw, (void*)m->d_rows, (void*)m->d_rlen, (void*)m->d_fbw, (void*)m->d_dct,
                  (void*)m->d_scale})
    if (p) (void)hipFree(p);
}

}  // namespace

using wk::hip_fail;
using wk::invalid;

extern "C" {

wk_status wk_esp_mfcc_create(int32_t sampling_rate, int32_t frame_size, int32_t n_fft, int32_t n_filters,
                             int32_t n_mfcc, int32_t esp_dsp_packing, int32_t device, wk_esp_mfcc** out) {
  if (!out) return invalid("wk_esp_mfcc_create: null out");
  *out = nullptr;
  const int lg = wk::esp::check_domain(sampling_rate, frame_size, n_fft, n_filters, n_mfcc);
  if (lg < 0)
    return invalid("wk_esp_mfcc_create: parameters outside mfcc.c's domain (n_fft a power of 2 in [2, 4096], "
                   "1 <= n_filters <= 1024, frame_size, n_mfcc, sampling_rate >= 1)");
  wk_esp_mfcc* m = new (std::nothrow) wk_esp_mfcc;
  if (!m) return WK_ERR_NO_MEMORY;
  *m = wk_esp_mfcc{sampling_rate, frame_size, n_fft, n_filters, n_mfcc, esp_dsp_packing ? 1 : 0, device, lg};
  // window (mfcc.c:118-120: alpha - (1 - alpha) cos(2 pi i / (frame - 1)), float, the angle in double)
  const std::vector<float> win = wk::esp::window(frame_size);
  std::vector<float2> tw(n_fft / 2);
  for (int k = 0; k < n_fft / 2; ++k)
    tw[k] = make_float2((float)cos(2.0 * M_PI * k / n_fft), (float)-sin(2.0 * M_PI * k / n_fft));
  // sparse mel rows: the span of each row's nonzero (or NaN) weights
  const int nb = n_fft / 2 + 1;
  const std::vector<float> fb = wk::esp::filterbank(sampling_rate, n_filters, n_fft);
  std::vector<int2> rows(n_filters);
  std::vector<int> rlen(n_filters);
  std::vector<float> fbw;
  for (int f = 0; f < n_filters; ++f) {
    int lo = -1, hi = -1;
    for (int k = 0; k < nb; ++k)
      if (fb[(size_t)f * nb + k] != 0.0f) {   // (NaN != 0: kept)
        if (lo < 0) lo = k;
        hi = k;
      }
    if (lo < 0) lo = hi = 0;
    rows[f] = make_int2((int)fbw.size(), lo);
    rlen[f] = hi - lo + 1;
    for (int k = lo; k <= hi; ++k) fbw.push_back(fb[(size_t)f * nb + k]);
  }
  // DCT-II cosines (mfcc.c:26-30 / :44-48: cos of the float-converted double angle) and scales (:33, :57)
  std::vector<float> dct, scale;
  wk::esp::dct(n_mfcc, n_filters, dct, scale);
  const wk_status s = wk::on_device(device, [&]() -> wk_status {
    hipError_t e;
    if ((e = upload(&m->d_win, win)) != hipSuccess || (e = upload(&m->d_tw, tw)) != hipSuccess ||
        (e = upload(&m->d_rows, rows)) != hipSuccess || (e = upload(&m->d_rlen, rlen)) != hipSuccess ||
        (e = upload(&m->d_fbw, fbw)) != hipSuccess || (e = upload(&m->d_dct, dct)) != hipSuccess ||
        (e = upload(&m->d_scale, scale)) != hipSuccess)
      return hip_fail(e, "wk_esp_mfcc_create: table upload");
    return WK_OK;
  });
  if (s != WK_OK) {
    (void)wk::on_device(device, [&]() -> wk_status {
      free_tables(m);
      return WK_OK;
    });
    delete m;
    return s;
  }
  *out = m;
  return WK_OK;
}

wk_status wk_esp_mfcc_run(wk_esp_mfcc* m, const float* d_signal, int64_t batch, int32_t signal_len, int64_t stride,
                          int32_t hop_size, float pre_emphasis, float* d_out, void* stream) {
  if (!m) return invalid("wk_esp_mfcc_run: null object");
  if (batch < 0 || signal_len < m->frame || hop_size < 1 || (batch > 1 && stride < 1))
    return invalid("wk_esp_mfcc_run: bad sizes (signal_len >= frame_size, hop_size >= 1)");
  if (batch > 0 && (!d_signal || !d_out)) return invalid("wk_esp_mfcc_run: null pointer");
  if (batch == 0) return WK_OK;
  const int nf = (signal_len - m->frame) / hop_size + 1;
  const size_t lds = sizeof(float) * ((size_t)2 * m->n_fft + m->n_fft / 2 + 1 + m->n_filters);
  return wk::on_device(m->device, [&]() -> wk_status {
    int cu = 256;
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, m->device);
    const int64_t units = batch * nf, cap = (int64_t)cu * 8;
    const unsigned grid = (unsigned)(units < cap ? units : cap);
    hipLaunchKernelGGL(wk_esp_mfcc_kernel, dim3(grid), dim3(kEspBlock), lds, (hipStream_t)stream, d_signal, batch,
                       signal_len, stride, hop_size, pre_emphasis, m->frame, m->n_fft, m->log2n, m->esp_pack, m->d_win,
                       m->d_tw, m->d_rows, m->d_rlen, m->d_fbw, m->n_filters, m->d_dct, m->d_scale, m->n_mfcc, nf,
                       d_out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_esp_mfcc launch");
  });
}

wk_status wk_esp_mfcc_destroy(wk_esp_mfcc* m) {
  if (!m) return WK_OK;
  (void)wk::on_device(m->device, [&]() -> wk_status {
    free_tables(m);
    return WK_OK;
  });
  delete m;
  return WK_OK;
}

}  // extern "C"
