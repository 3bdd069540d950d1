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
#include "wk_kernels.h"

using namespace wk;

#include "wk_fe_dev.h"

namespace {


template <bool MODE_B, typename T>
__global__ __launch_bounds__(kFeBlock, 4) void wk_frontend_kernel(const T* __restrict__ audio, int64_t n_units,
                                                                  int n_chunks, int nf, int win_len,
                                                                  int64_t clip_stride, float* __restrict__ out,
                                                                  int esp_pack, int cmvn, float pre) {
  __shared__ __attribute__((aligned(16))) float smem[kFeLdsNoWin];
  float* P = smem + kPOff;
  float* L = smem + kLOff;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;

  fe_init_tables<MODE_B, false>(smem, threadIdx.x, kFeBlock);
  const FeTables tb = {MODE_B ? kWinB : kWinA, smem + kTwOff};   // window: constant table (L1-resident)
  const TwsLds tws = {smem + kTwsOff};
  const f2 w0 = fe_split_tw(j, 0);
  // Frame slots: groups 0/1 (and 2/3) of a wave take frames 16 apart so their
  // pitch-17 transpose images fall in disjoint LDS banks.
  const int slot_base = 16 * (g & 1) + 32 * (g >> 1);
  __syncthreads();

  // Wave-round (unit u, round r) geometry: frame t (within the clip), local
  // frame fl (within the 63-frame chunk), frames in the chunk, edge flag.
  auto frame_of = [&](int64_t u, int r, int& t, int& fl, int& nfc, bool& slow, const T*& xp) {
    const int64_t clip = MODE_B ? u : u / n_chunks;   // mode B: one chunk per clip
    const int chunk = (int)(u - clip * n_chunks);
    xp = audio + clip * clip_stride;
    const int f0 = chunk * kNFramesB;
    nfc = min(kNFramesB, nf - f0);
    fl = wave + 8 * r + slot_base;
    t = f0 + fl;
    slow = MODE_B && ((r == 0 && wave == 0) || (r == 1 && wave == 6));   // holds frame 0 or 62
  };
  auto prefetch = [&](int64_t u, int r, Raw<T>& dst) {
    if (u < n_units) {
      int t, fl, nfc;
      bool slow;
      const T* xp;
      frame_of(u, r, t, fl, nfc, slow, xp);
      load_raw<MODE_B>(make_rsrc(xp, (uint32_t)win_len * sizeof(T)), MODE_B ? 256 * t - 160 : 256 * t, j, win_len,
                       fl < nfc, slow, dst);
    }
  };

  Raw<T> pf;
  prefetch(blockIdx.x, 0, pf);

  for (int64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    const int64_t clip = MODE_B ? u : u / n_chunks;
    const int chunk = (int)(u - clip * n_chunks);
    const int f0 = chunk * kNFramesB;
    const int nfc = min(kNFramesB, nf - f0);

#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
      int t, fl, nfc_r;
      bool slow;
      const T* xp;
      frame_of(u, r, t, fl, nfc_r, slow, xp);
      f2 a[16];
      if (fl < nfc) {
        fe_stage0<MODE_B>(pf, MODE_B ? 256 * t - 160 : 256 * t, win_len, j, slow, tb, a, pre);
      }
      // pf is consumed: prefetch the next wave-round, (u,1) or (u+grid,0), into it.
      prefetch(r == 0 ? u : u + gridDim.x, r ^ 1, pf);
      if (fl < nfc) fe_rest<MODE_B>(a, j, P + fl * kPRow, P + fl * kPRow + (fl & 1), tb, w0, tws, esp_pack, NoPrefetch());
    }
    wg_barrier_lds();

    mel_dispatch<MODE_B>(wave, P + min(lane, nfc - 1) * kPRow, L + lane);
    wg_barrier_lds();

    const float* lrow = L + lane;
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
                           int64_t clip_stride, float* out, int esp_pack, int cmvn, int grid_cap, float pre_emphasis,
                           hipStream_t stream) {
  const int nf = mode_b ? kNFramesB : (win_len - 320) / 256 + 1;
  const int n_chunks = mode_b ? 1 : (nf + kNFramesB - 1) / kNFramesB;
  const int64_t n_units = batch * n_chunks;
  if (n_units == 0) return hipSuccess;
  const int grid = (int)(n_units < grid_cap ? n_units : grid_cap);
  if (mode_b) {
    if (i16)
      hipLaunchKernelGGL((wk_frontend_kernel<true, int16_t>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const int16_t*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn, -pre_emphasis);
    else
      hipLaunchKernelGGL((wk_frontend_kernel<true, float>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const float*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn, -pre_emphasis);
  } else {
    if (i16)
      hipLaunchKernelGGL((wk_frontend_kernel<false, int16_t>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const int16_t*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn, -pre_emphasis);
    else
      hipLaunchKernelGGL((wk_frontend_kernel<false, float>), dim3(grid), dim3(kFeBlock), 0, stream,
                         (const float*)audio, n_units, n_chunks, nf, win_len, clip_stride, out, esp_pack, cmvn, -pre_emphasis);
  }
  return hipGetLastError();
}

}  // namespace wk
