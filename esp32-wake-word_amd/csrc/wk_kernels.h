// wk_kernels.h -- host-side launchers of the wake-word kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <string>

#include "wakeword.h"
#include "wk_status.h"

namespace wk {

// Error reporting shared by the C-ABI translation units (wk_api.hip, wk_ctc.hip;
// g_last_error, invalid and fail in wk_status.h).
wk_status hip_fail(hipError_t e, const char* what);

// Run `body` with device `dev` current; restore the caller's device.
template <typename F>
wk_status on_device(int dev, F body) {
  int old = -1;
  hipError_t e = hipGetDevice(&old);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (old != dev && (e = hipSetDevice(dev)) != hipSuccess) return hip_fail(e, "hipSetDevice");
  wk_status s = body();
  if (old != dev) (void)hipSetDevice(old);
  return s;
}

// Front-end (wk_frontend.hip).  mode_b: torchaudio+CMVN -> [B][13][63];
// otherwise esp_mfcc -> [B][n_frames][13].
hipError_t launch_frontend(bool mode_b, bool i16, const void* audio, int64_t batch, int win_len,
                           int64_t clip_stride, float* out, int esp_pack, int cmvn, int grid_cap,
                           float pre_emphasis, hipStream_t stream);   // pre_emphasis: 0.97 (mfcc.c:445), 0 = none

// Fused front-end + CNN (wk_fused.hip), mode B only.
// w = fp32 fragment-major weights (pack_fragments); wbf = bf16 conv fragments
// (pack_fragments_bf16; hi then lo parts for split bf16) for conv_mode 1
// (bf16, config 4) and 2 (split bf16, WK_PREC_BF16X3); conv_mode 0 = fp32 MFMA.
hipError_t launch_fused(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                        const uint16_t* wbf, int conv_mode, float* logits, float* feats_or_null, int grid_cap, hipStream_t stream,
                        unsigned* err,        // host-visible protocol error word (see wk_fused_kernel), may be null
                        int diag = 0);   // role isolation (-DWK_DIAG builds only): 1 = FE role only,
                                         // 2 = CNN role only; wrong logits

// The bf16-family half of launch_fused (wk_fused_xdl.hip: conv_mode 1 / 2,
// scalar-fp32 front-end); launch_fused calls it.
hipError_t launch_fused_xdl(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                            const uint16_t* wbf, int conv_mode, float* logits, float* feats_or_null, int grid_cap,
                            hipStream_t stream, unsigned* err, int diag);

// CNN on caller features (wk_fused.hip, the fused kernel's CNN role fed from
// HBM): feats [B][13][63] -> logits [B]; conv_mode as launch_fused.
hipError_t launch_cnn_fused(const float* feats, int64_t batch, const float* w, const uint16_t* wbf, int conv_mode,
                            float* logits, int grid_cap, hipStream_t stream, unsigned* err);

// int8 CNN in the device's esp-dl arithmetic (wk_int8.hip); feats [B][13][63] fp32.
constexpr int kNumInt8Weights = 3 * 13 * 32 + 3 * 32 * 64 + 3 * 64 * 128 + 128 * 64 + 64;
hipError_t launch_int8_cnn(const float* feats, int64_t batch, const int8_t* wq, float* logits, int grid_cap,
                           hipStream_t stream);
void quantize_int8_weights(const float* w, int8_t* q);

// Misc (wk_misc.hip).
hipError_t launch_synth(uint32_t seed, int64_t first, int64_t count, int n, float* out, hipStream_t stream);
hipError_t launch_normalize(const float* in, float* out, int64_t batch, int n_coef, int n_time, int method,
                            hipStream_t stream);
// The firmware's per-window CMVN over an MFCC frame stream (wk_device_cmvn).
hipError_t launch_record_front(const int16_t* tdm, int64_t n_out, int16_t* out16, float* outf, hipStream_t stream);
hipError_t launch_quantize_frames(const float* x, int64_t n, int8_t* q, hipStream_t stream);
// wk_stream_push: ring samples [pos, pos + m) mod cap, host staging ring -> mirrored device ring.
hipError_t launch_ring_ingest(const float* src, float* dst, int64_t cap, int64_t pos, int64_t m, hipStream_t stream);
hipError_t launch_device_cmvn(const void* frames, bool int8_in, int64_t n_windows, int8_t* out_i8, float* out_f,
                              hipStream_t stream);

// Offsets (floats) of each tensor inside the packed weight blob.
constexpr int kOffW1 = 0;                       // conv_layers.0.weight [32][13][3]
constexpr int kOffW2 = kOffW1 + 32 * 13 * 3;    // conv_layers.3.weight [64][32][3]
constexpr int kOffW3 = kOffW2 + 64 * 32 * 3;    // conv_layers.6.weight [128][64][3]
constexpr int kOffF1 = kOffW3 + 128 * 64 * 3;   // classifier.0.weight [64][128]
constexpr int kOffF2 = kOffF1 + 64 * 128;       // classifier.2.weight [1][64]
constexpr int kNumWeights = kOffF2 + 64;        // 40224

// Fragment-major copy of the weights for the MFMA kernels.  Per 16-row output
// tile and k-step, the 64 values lane l feeds as the A operand of
// v_mfma_f32_16x16x4_f32 (row = l&15), so a wave loads one fragment with one
// coalesced 256-byte load.
//   conv ([clip][t][ci] images): step s = 4 (tap * CB + cb) + j, lane group
//     q = l>>4 feeds ci = 16 cb + 4 q + j at that tap (Cin padded to 16);
//     taps 0 and 2 are g0, g2, tap 1 the Winograd tap G1 = (g0 + g1 + g2) / 2.
//   classifier.0 (v_mfma_f32_4x4x1_16b_f32, 16 blocks): wave w, step s feeds
//     k = 16 w + s; lane l is the output row o = l.
constexpr int kPkW1 = 0;                        // [2 tiles][12 s][64]
constexpr int kPkW2 = kPkW1 + 2 * 12 * 64;      // [4][24][64]
constexpr int kPkW3 = kPkW2 + 4 * 24 * 64;      // [8][48][64]
constexpr int kPkF1 = kPkW3 + 8 * 48 * 64;      // [8 waves][16 s][64 o]  (k = 16 w + s)
constexpr int kPkF2 = kPkF1 + 8 * 16 * 64;      // [64]
constexpr int kNumPacked = kPkF2 + 64;

// bf16 variant (WK_PREC_BF16 / BF16X3, v_mfma_f32_16x16x32_bf16): per 16-row
// tile and k-step s, lane l feeds 8 consecutive k = 32s + 8(l>>4) + j (j = 0..7)
// of row l&15 -- one 16-byte load per fragment.  k = tap*Cin_pad + ci, zero
// past 3*Cin_pad (conv1: 48 -> 2 steps).  Offsets in bf16 (uint16) units.
constexpr int kPbW1 = 0;                        // [2 tiles][2 s][64][8]   (Cin 13 padded to 16)
constexpr int kPbW2 = kPbW1 + 2 * 2 * 64 * 8;   // [4][3][64][8]
constexpr int kPbW3 = kPbW2 + 4 * 3 * 64 * 8;   // [8][6][64][8]
constexpr int kNumPackedBf16 = kPbW3 + 8 * 6 * 64 * 8;
constexpr int kBfFrag = 64 * 8;                 // bf16 elements per fragment

inline uint16_t to_bf16_rne(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// lo = true packs the split-bf16 low parts, bf16(w - bf16(w)) (WK_PREC_BF16X3).
inline uint16_t split_bf16(float x, bool lo) {
  const uint16_t h = to_bf16_rne(x);
  if (!lo) return h;
  const uint32_t u = (uint32_t)h << 16;
  float hf;
  memcpy(&hf, &u, 4);
  return to_bf16_rne(x - hf);
}

inline void pack_fragments_bf16(const float* w, uint16_t* pk, bool lo = false) {
  auto pack = [&](int off, int cout_tiles, int cin, int cin_pad, int wbase) {
    const int nsteps = (3 * cin_pad + 31) / 32;
    for (int t = 0; t < cout_tiles; ++t)
      for (int s = 0; s < nsteps; ++s)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int co = 16 * t + (l & 15), k = 32 * s + 8 * (l >> 4) + j, tap = k / cin_pad, ci = k % cin_pad;
            pk[off + ((t * nsteps + s) * 64 + l) * 8 + j] =
                tap < 3 && ci < cin ? split_bf16(w[wbase + (co * cin + ci) * 3 + tap], lo) : (uint16_t)0;
          }
  };
  pack(kPbW1, 2, 13, 16, kOffW1);
  pack(kPbW2, 4, 32, 32, kOffW2);
  pack(kPbW3, 8, 64, 64, kOffW3);
}

// Host-side packing of the WK_NUM_WEIGHTS blob into the fragment-major layouts.
inline void pack_fragments(const float* w, float* pk) {
  auto conv_blocked = [&](int off, int tiles, int cin, int cin_pad, int wbase) {
    const int cb_n = cin_pad / 16, nsteps = 12 * cb_n;
    for (int t = 0; t < tiles; ++t)
      for (int s = 0; s < nsteps; ++s)
        for (int l = 0; l < 64; ++l) {
          const int g = s >> 2, j = s & 3, tap = g / cb_n, cb = g % cb_n;
          const int co = 16 * t + (l & 15), ci = 16 * cb + 4 * (l >> 4) + j;
          float v = 0.0f;
          if (ci < cin) {
            const float* g = w + wbase + (co * cin + ci) * 3;
            // tap 1 holds the Winograd F(2,3) tap G1 = (g0 + g1 + g2) / 2; the
            // kernel forms G2 = (g0 + g2) - G1 (conv_wino_v)
            v = tap == 1 ? (float)(0.5 * ((double)g[0] + (double)g[1] + (double)g[2])) : g[tap];
          }
          pk[off + (t * nsteps + s) * 64 + l] = v;
        }
  };
  conv_blocked(kPkW1, 2, 13, 16, kOffW1);
  conv_blocked(kPkW2, 4, 32, 32, kOffW2);
  conv_blocked(kPkW3, 8, 64, 64, kOffW3);
  for (int wv = 0; wv < 8; ++wv)
    for (int s = 0; s < 16; ++s)
      for (int o = 0; o < 64; ++o) pk[kPkF1 + (wv * 16 + s) * 64 + o] = w[kOffF1 + o * 128 + 16 * wv + s];
  for (int o = 0; o < 64; ++o) pk[kPkF2 + o] = w[kOffF2 + o];
}

}  // namespace wk
