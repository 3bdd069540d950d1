// wk_fe_dev.h -- device code of the MFCC front-end (shared by the standalone
// front-end kernel, wk_frontend.hip, and the fused kernel, wk_fused.hip).
// See wk_frontend.hip for the algorithm and the reference citations.
#pragma once
#include "wk_common.h"
#include "wk_tables.h"

namespace wk {

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

// Raw samples of one frame-group slot, prefetched into registers one round
// ahead: x[i0], x[i0+1] for i0 = base + 32*n1 + 2j, plus x[base-1].  The
// pre-emphasis partner x[i0-1] is the previous lane's x[i0+1] (DPP row
// rotate), so it is not loaded twice.  Kept in the input type so the loads
// stay outstanding until first use.
template <typename T>
struct Raw {
  T x0[10], x1[10];
  T xb;
};

template <typename T>
__device__ __forceinline__ void load_raw(const T* __restrict__ x, int base, int j, bool act, Raw<T>& r) {
  if (act) {
#pragma unroll
    for (int n1 = 0; n1 < 10; ++n1) {
      const int i0 = base + 32 * n1 + 2 * j;
      r.x0[n1] = x[i0];
      r.x1[n1] = x[i0 + 1];
    }
    r.xb = x[base - 1];
  }
}

__device__ __forceinline__ float row_ror1(float v) {  // lane l <- lane (l-1) mod 16 of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xF, 0xF, false));
}

// LDS tables shared by the workgroup.
struct FeTables {
  const float* win;   // [320] analysis window (mode-specific)
  const float* tw;    // [15][16][2]: W256^(j*k1), k1 = 1..15
};

// One frame -> its power row (bins 0..256) in LDS, by one 16-lane group.
// SLOW = general sample path (reflect padding / first-sample rule), used only
// by the wave-rounds that hold the edge frames; it loads its own samples.
// Stage 0: pre-emphasis + window of the 320 frame samples as 160 complex
// (even, odd) pairs: lane j holds pair index 16*n1 + j, n1 = 0..9.
template <bool MODE_B, bool SLOW, typename T>
__device__ __forceinline__ void fe_stage0(const T* __restrict__ x, const Raw<T>& raw, int t, int n, int j,
                                          const FeTables& tb, cf (&a)[16]) {
  const int base = MODE_B ? (256 * t - 160) : (256 * t);
  float prev_rot = 0.0f;
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) {
    float y0, y1;
    if constexpr (!SLOW) {
      const float x0 = to_f(raw.x0[n1]), x1 = to_f(raw.x1[n1]);
      // x[i0-1]: lane j-1's x1 of this row; lane 0 takes lane 15's x1 of the previous row.
      const float rot = row_ror1(x1);
      const float xm = j != 0 ? rot : (n1 == 0 ? to_f(raw.xb) : prev_rot);
      prev_rot = rot;
      y0 = __builtin_fmaf(-0.97f, xm, x0);
      y1 = __builtin_fmaf(-0.97f, x0, x1);
    } else {
      const int i0 = base + 32 * n1 + 2 * j;
      y0 = pre_general<MODE_B>(x, i0, n);
      y1 = pre_general<MODE_B>(x, i0 + 1, n);
    }
    const float2 w = *reinterpret_cast<const float2*>(tb.win + 32 * n1 + 2 * j);
    a[n1] = {y0 * w.x, y1 * w.y};
  }
#pragma unroll
  for (int n1 = 10; n1 < 16; ++n1) a[n1] = {0.0f, 0.0f};
}

// Stages 1..4 of one frame -> its power row (bins 0..256) in LDS.
template <bool MODE_B>
__device__ __forceinline__ void fe_rest(cf (&a)[16], int j, int lane, float* __restrict__ row, const FeTables& tb,
                                        cf w512, int esp_pack) {
  dft16(a);  // A[k1] at a[dft16_out(k1)]

  // twiddle W256^(j*k1) + 16x16 transpose through this frame's LDS row (pitch 17).
  // (twiddles are applied in groups of 4 so their LDS reads do not all
  // sit in VGPRs at once; re parts go straight to the transpose image.)
  cf b[16];
  b[0] = a[0];
  row[j] = b[0].re;
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {
    const float2 w = *reinterpret_cast<const float2*>(tb.tw + ((k1 - 1) * 16 + j) * 2);
    b[k1] = cmul(a[dft16_out(k1)], cf{w.x, w.y});
    row[17 * k1 + j] = b[k1].re;
    if ((k1 & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  cf c[16];
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

  // Real-FFT split: U = 2 V[k] = S - i*b, U' = conj(2 V[256-k]) = S + i*b with
  // S = Z[k] + conj Z[256-k], D = Z[k] - conj Z[256-k], b = W512^k D.
  // Partner Z[256 - k]: lane (16-j)&15 of this group, register 15-k2 (ds_bpermute);
  // lane 0 holds its own partner in register (16-k2)&15.
  const int src = ((lane & 48) | ((16 - j) & 15)) << 2;
#pragma unroll
  for (int k2 = 0; k2 <= 8; ++k2) {
    const cf zk = c[dft16_out(k2)];
    cf zq_;
    if (k2 < 8) {
      const cf s = c[dft16_out(15 - k2)];
      const cf own = c[dft16_out((16 - k2) & 15)];
      const float pr = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(s.re)));
      const float pi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(s.im)));
      zq_ = j == 0 ? own : cf{pr, pi};
    } else {
      zq_ = c[dft16_out(8)];
    }
    const cf S = {zk.re + zq_.re, zk.im - zq_.im};
    const cf D = {zk.re - zq_.re, zk.im + zq_.im};
    const cf tw = cmul(w512, w32(k2));
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

// LDS carve (floats): twiddles | window | log-mel [40][64] | power rows [63][271].
constexpr int kTwOff = 0, kTwSize = 15 * 16 * 2;
constexpr int kWinOff = kTwOff + kTwSize, kWinSize = 320;
constexpr int kLOff = kWinOff + kWinSize, kLSize = 40 * WK_LSTRIDE;
constexpr int kPOff = kLOff + kLSize, kPSize = kNFramesB * kPRow;
constexpr int kFeLds = kPOff + kPSize;
static_assert(kFeLds * 4 <= 81920, "front-end LDS must allow 2 workgroups per CU");

// Fill the window / twiddle tables of the LDS carve (all threads of the WG).
template <bool MODE_B>
__device__ __forceinline__ void fe_init_tables(float* smem, int tid, int nthreads) {
  for (int i = tid; i < 320; i += nthreads) smem[kWinOff + i] = MODE_B ? kWinB[i] : kWinA[i];
  for (int i = tid; i < 15 * 16; i += nthreads) {
    const int k1 = i / 16 + 1, jj = i % 16;
    float sn, cs;
    sincospif(-(float)(jj * k1) / 128.0f, &sn, &cs);
    smem[kTwOff + 2 * i] = cs;
    smem[kTwOff + 2 * i + 1] = sn;
  }
}

__device__ __forceinline__ cf fe_w512(int j) {
  float sn, cs;
  sincospif(-(float)j / 256.0f, &sn, &cs);
  return {cs, sn};
}

}  // namespace wk
