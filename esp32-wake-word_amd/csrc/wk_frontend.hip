// wk_frontend.hip -- fused MFCC front-end for gfx950 (MI355X).
//
// Restates, per 1 s window (reference paths):
//   mode B  ml_models/src/extract_mfcc.py:171-175 (torchaudio preemphasis,
//           MFCC(n_fft 512, win 320, hop 256, 40 mel, 13 mfcc, hamming,
//           center/reflect), normalize_mfcc('cmvn') :73-80)
//   mode A  main/esp_mfcc/mfcc.c:431-527 (pre_emphasis :66-74, frame_division
//           :76-108, apply_window :110-131, compute_power_spectrum :236-273,
//           create/apply_mel_filterbank :144-234/:275-295, log :496-498,
//           dct_ii :20-64)
//
// Workgroup = 8 waves, one work unit (a clip, or a <=63-frame chunk of a clip
// in mode A) at a time, grid-stride persistent.  Three phases per unit:
//   1. FFT phase, "16 lanes per frame": each 16-lane group turns one frame
//      into its 257-bin power row.  The 512-pt real DFT is a 256-pt complex
//      DFT of (even, odd) sample pairs done as 16 x 16: an in-register DFT16
//      over the 16 values a lane holds, a per-lane twiddle, a 16x16 transpose
//      through the frame's own LDS row (pitch-17 image, two passes re/im),
//      a second in-register DFT16, then the real-FFT split with the partner
//      bin fetched by ds_bpermute.  Only 160 of the 256 complex inputs are
//      non-zero (320-sample window), so the first DFT16 runs on 10 inputs.
//   2. mel phase, "lane per frame": lane f owns frame f; wave w owns a block
//      of mel filters, so filterbank weights and bin offsets are immediates
//      in straight-line generated code (wk_tables.h); ln -> log-mel rows.
//   3. DCT (+ CMVN for mode B), lane per frame; CMVN statistics are wave
//      reductions across the 63 lanes; coalesced stores.
#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_tables.h"

using namespace wk;

namespace {

// W32^k2 = exp(-2*pi*i*k2/32), k2 = 0..8.
__device__ __forceinline__ cf w32(int k2) {
  switch (k2) {
    case 0: return {1.0f, 0.0f};
    case 1: return {0.98078528040323043f, -0.19509032201612825f};
    case 2: return {0.92387953251128674f, -0.38268343236508978f};
    case 3: return {0.83146961230254524f, -0.55557023301960218f};
    case 4: return {0.70710678118654752f, -0.70710678118654752f};
    case 5: return {0.55557023301960218f, -0.83146961230254524f};
    case 6: return {0.38268343236508978f, -0.92387953251128674f};
    case 7: return {0.19509032201612825f, -0.98078528040323043f};
    default: return {0.0f, -1.0f};
  }
}

// Pre-emphasised sample at (centred) index i, general path.
//   mode B: reflect padding of the pre-emphasised signal (torch.stft center).
//   mode A: no padding; y[0] = x[0] (mfcc.c:70).
template <bool MODE_B, typename T>
__device__ __forceinline__ float pre_general(const T* __restrict__ x, int i, int n) {
  int r = i;
  if (MODE_B) {
    r = r < 0 ? -r : r;
    r = r > n - 1 ? 2 * (n - 1) - r : r;
  }
  const float xr = sample(x, r);
  const float xm = sample(x, r > 0 ? r - 1 : 0);
  return r > 0 ? __builtin_fmaf(-0.97f, xm, xr) : xr;
}

struct LaneConst {
  float wr[10], wi[10];  // window at n = 32*n1 + 2j, +1
  cf tw[16];             // W256^(j*k1)
  cf w512;               // W512^j
};

// One frame -> its power row (bins 0..256) in LDS, by one 16-lane group.
template <bool MODE_B, bool SLOW, typename T>
__device__ __forceinline__ void fe_frame(const T* __restrict__ x, int t, int n, int j, int lane,
                                         float* __restrict__ row, const LaneConst& k, int esp_pack) {
  cf a[16];
  const int base = MODE_B ? (256 * t - 160) : (256 * t);
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) {
    const int i0 = base + 32 * n1 + 2 * j;
    float y0, y1;
    if constexpr (!SLOW) {
      const float xm = sample(x, i0 - 1), x0 = sample(x, i0), x1 = sample(x, i0 + 1);
      y0 = __builtin_fmaf(-0.97f, xm, x0);
      y1 = __builtin_fmaf(-0.97f, x0, x1);
    } else {
      y0 = pre_general<MODE_B>(x, i0, n);
      y1 = pre_general<MODE_B>(x, i0 + 1, n);
    }
    a[n1] = {y0 * k.wr[n1], y1 * k.wi[n1]};
  }
#pragma unroll
  for (int n1 = 10; n1 < 16; ++n1) a[n1] = {0.0f, 0.0f};

  dft16(a);  // A[k1] at a[dft16_out(k1)]

  // twiddle + 16x16 transpose through this frame's LDS row (pitch 17).
  cf b[16];
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) b[k1] = k1 == 0 ? a[0] : cmul(a[dft16_out(k1)], k.tw[k1]);
  cf c[16];
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) row[17 * k1 + j] = b[k1].re;
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) c[n2].re = row[17 * j + n2];
  wave_lds_sync();
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) row[17 * k1 + j] = b[k1].im;
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) c[n2].im = row[17 * j + n2];
  wave_lds_sync();

  dft16(c);  // Z[j + 16*k2] at c[dft16_out(k2)]

  // Partner Z[256 - k]: lane (16-j)&15 of this group, register 15-k2; lane 0 uses its own.
  const int src = ((lane & 48) | ((16 - j) & 15)) << 2;
  cf zq[8];
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    const cf s = c[dft16_out(15 - k2)];
    const cf own = c[dft16_out((16 - k2) & 15)];
    const float pr = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(s.re)));
    const float pi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(s.im)));
    zq[k2] = j == 0 ? own : cf{pr, pi};
  }
  wave_lds_sync();

  // Real-FFT split: U = 2 V[k] = S - i*b, U' = conj(2 V[256-k]) = S + i*b with
  // S = Z[k] + conj Z[256-k], D = Z[k] - conj Z[256-k], b = W512^k D.
#pragma unroll
  for (int k2 = 0; k2 <= 8; ++k2) {
    const cf zk = c[dft16_out(k2)];
    const cf zq_ = k2 < 8 ? zq[k2] : c[dft16_out(8)];
    const cf S = {zk.re + zq_.re, zk.im - zq_.im};
    const cf D = {zk.re - zq_.re, zk.im + zq_.im};
    const cf tw = cmul(k.w512, w32(k2));
    const cf bb = cmul(tw, D);
    const float ur = S.re + bb.im, ui = S.im - bb.re;
    const float vr = S.re - bb.im, vi = S.im + bb.re;
    float pk = __builtin_fmaf(ur, ur, ui * ui);
    float pq = __builtin_fmaf(vr, vr, vi * vi);
    const int kb = j + 16 * k2;
    if constexpr (!MODE_B) {
      // mfcc.c:267 power = |X|^2 / n_fft + 1e-12 with |X|^2 = |U|^2 / 4; the
      // esp-dsp dsps_cplx2reC_fc32 packing (mfcc.c:261) doubles bins 1..255
      // and zeroes bin 256 (parity unpinned).
      const float sk = esp_pack ? (kb == 0 ? 1.0f : 4.0f) : 1.0f;
      const float sq = esp_pack ? (kb == 0 ? 0.0f : 4.0f) : 1.0f;  // kb==0 -> upper bin is 256
      pk = __builtin_fmaf(pk, sk * (1.0f / 2048.0f), 1e-12f);
      pq = __builtin_fmaf(pq, sq * (1.0f / 2048.0f), 1e-12f);
    }
    if (k2 < 8) {
      row[kb] = pk;
      row[256 - kb] = pq;
    } else if (j == 0) {
      row[128] = pk;
    }
  }
}

template <bool MODE_B, int W>
__device__ __forceinline__ void mel_wave(const float* p, float* l) {
  if constexpr (MODE_B) melB_wave<W>(p, l); else melA_wave<W>(p, l);
}

template <bool MODE_B>
__device__ __forceinline__ void mel_dispatch(int wave, const float* p, float* l) {
  switch (wave) {
    case 0: mel_wave<MODE_B, 0>(p, l); break;
    case 1: mel_wave<MODE_B, 1>(p, l); break;
    case 2: mel_wave<MODE_B, 2>(p, l); break;
    case 3: mel_wave<MODE_B, 3>(p, l); break;
    case 4: mel_wave<MODE_B, 4>(p, l); break;
    case 5: mel_wave<MODE_B, 5>(p, l); break;
    case 6: mel_wave<MODE_B, 6>(p, l); break;
    default: mel_wave<MODE_B, 7>(p, l); break;
  }
}

// CMVN over the 63 lanes of one coefficient row (extract_mfcc.py:76-80):
// mean, unbiased std, std==0 -> 1, (x - mean) / (std + 1e-8).
__device__ __forceinline__ float cmvn_lane(float v, bool valid, int n) {
  const float mean = wave_sum(valid ? v : 0.0f) / (float)n;
  const float d = valid ? v - mean : 0.0f;
  float sd = sqrtf(wave_sum(d * d) / (float)(n - 1));
  sd = sd == 0.0f ? 1.0f : sd;
  return d / (sd + 1e-8f);
}

template <bool MODE_B, typename T>
__global__ __launch_bounds__(kFeBlock, 4) void wk_frontend_kernel(const T* __restrict__ audio, int64_t n_units,
                                                                  int n_chunks, int nf, int win_len,
                                                                  int64_t clip_stride, float* __restrict__ out,
                                                                  int esp_pack, int cmvn) {
  __shared__ __attribute__((aligned(16))) float smem[kNFramesB * kPRow + 64 * kLRow];
  float* P = smem;
  float* L = smem + kNFramesB * kPRow;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;

  LaneConst k;
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) {
    const int nn = 32 * n1 + 2 * j;
    k.wr[n1] = MODE_B ? kWinB[nn] : kWinA[nn];
    k.wi[n1] = MODE_B ? kWinB[nn + 1] : kWinA[nn + 1];
  }
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) {
    float s, cc;
    sincospif(-(float)(j * k1) / 128.0f, &s, &cc);
    k.tw[k1] = {cc, s};
  }
  {
    float s, cc;
    sincospif(-(float)j / 256.0f, &s, &cc);
    k.w512 = {cc, s};
  }
  // Frame slots: groups 0/1 (and 2/3) of a wave take frames 16 apart so their
  // pitch-17 transpose images fall in disjoint LDS banks.
  const int slot_base = 16 * (g & 1) + 32 * (g >> 1);

  for (int64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    const int64_t clip = u / n_chunks;
    const int chunk = (int)(u - clip * n_chunks);
    const T* x = audio + clip * clip_stride;
    const int f0 = chunk * kNFramesB;
    const int nfc = min(kNFramesB, nf - f0);

#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int fl = wave + 8 * r + slot_base;
      const int t = f0 + fl;
      const bool slow = MODE_B ? ((r == 0 && wave == 0) || (r == 1 && wave == 6))
                               : (chunk == 0 && r == 0 && wave == 0);
      if (fl < nfc) {
        float* row = P + fl * kPRow;
        if (slow)
          fe_frame<MODE_B, true>(x, t, win_len, j, lane, row, k, esp_pack);
        else
          fe_frame<MODE_B, false>(x, t, win_len, j, lane, row, k, esp_pack);
      }
    }
    __syncthreads();

    mel_dispatch<MODE_B>(wave, P + min(lane, nfc - 1) * kPRow, L + lane * kLRow);
    __syncthreads();

    const float* lrow = L + lane * kLRow;
    const bool valid = lane < nfc;
    const int c0 = wave < 5 ? 2 * wave : wave + 5;
    const int nc = wave < 5 ? 2 : 1;
    for (int ci = 0; ci < nc; ++ci) {
      const int cc = c0 + ci;
      const float v = dct_coef<MODE_B>(cc, lrow);
      if constexpr (MODE_B) {
        const float y = cmvn ? cmvn_lane(v, valid, nfc) : v;
        if (valid) out[clip * (13 * kNFramesB) + cc * kNFramesB + lane] = y;
      } else {
        if (valid) out[(clip * nf + f0 + lane) * 13 + cc] = v;
      }
    }
  }
}

}  // namespace

namespace wk {

hipError_t launch_frontend(bool mode_b, bool i16, const void* audio, int64_t batch, int win_len,
                           int64_t clip_stride, float* out, int esp_pack, int cmvn, int grid_cap,
                           hipStream_t stream) {
  const int nf = mode_b ? kNFramesB : (win_len - 320) / 256 + 1;
  const int n_chunks = mode_b ? 1 : (nf + kNFramesB - 1) / kNFramesB;
  const int64_t n_units = batch * n_chunks;
  if (n_units == 0) return hipSuccess;
  const int grid = (int)(n_units < grid_cap ? n_units : grid_cap);
  if (mode_b) {
    if (i16)
      hipLaunchKernelGGL((wk_frontend_kernel<true, int16_t>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const int16_t*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn);
    else
      hipLaunchKernelGGL((wk_frontend_kernel<true, float>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const float*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn);
  } else {
    if (i16)
      hipLaunchKernelGGL((wk_frontend_kernel<false, int16_t>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const int16_t*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn);
    else
      hipLaunchKernelGGL((wk_frontend_kernel<false, float>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const float*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn);
  }
  return hipGetLastError();
}

}  // namespace wk
