// wk_cnn_dev.h -- device helpers of the xiaoa CNN (LightweightKWS,
// ml_models/src/wakeModel.py:4-34) on the matrix cores, used by the CNN role of
// wk_fused.hip (the fused kernel and the standalone CNN kernel).
//
//   conv(13->32,k3,p1) ReLU maxpool2 -> conv(32->64) ReLU pool -> conv(64->128)
//   ReLU pool -> mean over time -> Linear(128,64) ReLU -> Linear(64,1)
//
// Each conv is an implicit GEMM D[co][t] = sum_k W[co][k] X[k][t] over
// [clip][t][ci] LDS images: fp32 by Winograd F(2,3) on v_mfma_f32_16x16x4_f32,
// bf16 / split-bf16 directly on bf16 MFMA.
#pragma once
#include "wk_common.h"


namespace wk {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_4x4x1_16b_f32: 16 independent 4 x 4 x 1 blocks, block b = lane>>2
// (A: lane 4b + i = row i, B: lane 4b + j = column j; D[r] in lane 4b + j = row r, column j).
__device__ __forceinline__ f32x4 mfma4x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float swap_adjacent(float v) {  // lane l <- lane l^1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// ReLU -> maxpool(2) (15 -> 7, floor) -> mean over the 7 pooled steps.
template <int GSTRIDE>
__device__ __forceinline__ void epi_gap(const f32x4& acc, float* __restrict__ g, int co0, int clip, int lane) {
  const int tt = lane & 15;
  const bool w = !(lane & 1) && tt <= 12;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = fmaxf(acc[r], 0.0f);
    v = fmaxf(v, swap_adjacent(v));
    float s = w ? v : 0.0f;   // 16-lane row sum by DPP butterflies
    s += dpp<0xB1>(s);
    s += dpp<0x4E>(s);
    s += dpp<0x141>(s);
    s += dpp<0x140>(s);
    if (tt == 0) {
      g[(co0 + 4 * (lane >> 4) + r) * GSTRIDE + clip] = s * (1.0f / 7.0f);
    }
  }
}

// ---- bf16 convolutions (WK_PREC_BF16 / BF16X3) -----------------------------
// Fragments hold 8 bf16 per lane (K = 32 per step): one 16-byte LDS read per
// B fragment and one 16-byte load per A fragment.  Product builds issue a step
// as gfx950's v_mfma_f32_16x16x32_bf16.  The K = 32 rule: no
// kernel that issues it may issue packed-fp32 VALU (v_pk_*_f32), which was seen
// corrupted in lanes 48-63 beside it on the same SIMD.  The bf16-family fused
// unit (wk_fused_xdl.hip) therefore runs its front-end in scalar fp32, and
// tests/test_isa_rules.py checks every kernel of the library.  Diagnostic
// one-unit builds (WK_FUSED_ONE_TU: packed front-end in every precision) issue
// the step as two CDNA3-era v_mfma_f32_16x16x16_bf16 instead.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s8 __attribute__((ext_vector_type(8)));   // one lane's A or B fragment: 8 bf16 bit patterns

template <bool K32>
__device__ __forceinline__ f32x4 mfma_bf16(s8 a, s8 b, f32x4 c) {
  if constexpr (K32)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 0, 1, 2, 3),
                                                __builtin_shufflevector(b, b, 0, 1, 2, 3), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 4, 5, 6, 7),
                                                   __builtin_shufflevector(b, b, 4, 5, 6, 7), c, 0, 0, 0);
}
// Whether a conv layer (CINP 16: conv1, 32: conv2, 64: conv3) uses the K = 32
// form: every layer in product builds, none in diagnostic one-unit builds.
template <int CINP>
constexpr bool k32_layer() {
  return !WK_FUSED_ONE_TU;
}

__device__ __forceinline__ uint32_t bf16_bits(float x) {   // round to nearest even
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// K order of the fragments (wk_kernels.h pack_fragments_bf16): lane group
// g = lane >> 4 feeds k = 32 s + 8 g + j (j = 0..7) at step s, k = tap * CINP +
// ci, so its 8 B values are 8 consecutive ci of one image row: one 16-byte
// read.  kofs = that read's element offset from the lane's t row.  CINP = 16
// (conv1): step 0 = taps 0, 1; step 1 = tap 2 in groups 0-1 and K padding in
// groups 2-3, whose weights are zero and whose B read re-reads tap 2 (finite
// data: 0 * NaN garbage would poison the accumulator).
template <int CINP, int CIP>
__device__ __forceinline__ int kofs(int s, int g) {
  if constexpr (CINP >= 32) {
    return ((32 * s) / CINP) * CIP + (32 * s) % CINP + 8 * g;
  } else {
    const int tap = 2 * s + (g >> 1);
    return (tap < 2 ? tap : 2) * CIP + 8 * (g & 1);
  }
}

// Two 16-column t-tiles of one conv layer from a bf16 [clip][t][ci] image
// (ci pitch CIP).  boff = this lane's t row (element offset), g = lane >> 4.
template <int NSTEP, int CINP, int CIP, int CHUNK = 0>
__device__ __forceinline__ void conv_pair_bf(const uint16_t* __restrict__ img, const s8 (&wf)[NSTEP], int boff_a,
                                             int boff_b, int g, f32x4& acc_a, f32x4& acc_b) {
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int off = kofs<CINP, CIP>(s, g);
    const s8 ba = *reinterpret_cast<const s8*>(img + boff_a + off);
    const s8 bb = *reinterpret_cast<const s8*>(img + boff_b + off);
    acc_a = mfma_bf16<k32_layer<CINP>()>(wf[s], ba, acc_a);
    acc_b = mfma_bf16<k32_layer<CINP>()>(wf[s], bb, acc_b);
    if (CHUNK > 0 && (s % CHUNK) == CHUNK - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// ReLU -> maxpool(2) -> the 4 pooled channels of this lane (consecutive co)
// as one 8-byte store into the next layer's bf16 [clip][t][ci] image.
template <int CIP_N, int TP_N, int TN>
__device__ __forceinline__ void epi_pool_bf(const f32x4& acc, uint16_t* __restrict__ next, int co0, int clip, int t0,
                                            int lane) {
  const int t = t0 + (lane & 15);
  const int tp = t >> 1;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x = fmaxf(acc[r], 0.0f);
    v[r] = fmaxf(x, swap_adjacent(x));
  }
  if (!(lane & 1) && tp < TN) {
    uint2 pkd;
    pkd.x = bf16_bits(v[0]) | (bf16_bits(v[1]) << 16);
    pkd.y = bf16_bits(v[2]) | (bf16_bits(v[3]) << 16);
    *reinterpret_cast<uint2*>(next + (clip * TP_N + 1 + tp) * CIP_N + co0 + 4 * (lane >> 4)) = pkd;
  }
}

// ---- split-bf16 ("bf16x3") convolutions: fp32-grade products at bf16 MFMA rate.
// x = xh + xl and w = wh + wl with xh = bf16(x), xl = bf16(x - xh) (both RNE);
// x w ~= xh wh + (xl wh + xh wl), dropping xl wl (relative 2^-16).  Each bf16
// product is exact in the fp32 accumulator, so the per-product error is
// ~2^-16 relative -- three K=32 bf16 steps (mfma_bf16) in place of eight
// v_mfma_f32_16x16x4f32 (fp32 MFMA: 1/16 the bf16 rate).  Images hold
// xh at ci and xl at ci + CINP of the same t row.  All three products chain on
// one accumulator per tile (no VALU sum of partial accumulators).
template <int NSTEP, int CINP, int CIP, int CHUNK = 0>
__device__ __forceinline__ void conv_pair_bf3(const uint16_t* __restrict__ img, const s8 (&wh)[NSTEP],
                                              const s8 (&wl)[NSTEP], int boff_a, int boff_b, int g, f32x4& acc_a,
                                              f32x4& acc_b) {
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int off = kofs<CINP, CIP>(s, g);
    const s8 ha = *reinterpret_cast<const s8*>(img + boff_a + off);
    const s8 hb = *reinterpret_cast<const s8*>(img + boff_b + off);
    const s8 la = *reinterpret_cast<const s8*>(img + boff_a + off + CINP);
    const s8 lb = *reinterpret_cast<const s8*>(img + boff_b + off + CINP);
    acc_a = mfma_bf16<k32_layer<CINP>()>(wl[s], ha, acc_a);
    acc_b = mfma_bf16<k32_layer<CINP>()>(wl[s], hb, acc_b);
    acc_a = mfma_bf16<k32_layer<CINP>()>(wh[s], la, acc_a);
    acc_b = mfma_bf16<k32_layer<CINP>()>(wh[s], lb, acc_b);
    acc_a = mfma_bf16<k32_layer<CINP>()>(wh[s], ha, acc_a);
    acc_b = mfma_bf16<k32_layer<CINP>()>(wh[s], hb, acc_b);
    if (CHUNK > 0 && (s % CHUNK) == CHUNK - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// epi_pool_bf for split images: xh (8 bytes at co) and xl (8 bytes at co + LO).
template <int CIP_N, int TP_N, int TN, int LO>
__device__ __forceinline__ void epi_pool_bf3(const f32x4& acc, uint16_t* __restrict__ next, int co0, int clip, int t0,
                                             int lane) {
  const int t = t0 + (lane & 15);
  const int tp = t >> 1;
  uint32_t h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x = fmaxf(acc[r], 0.0f);
    const float v = fmaxf(x, swap_adjacent(x));
    h[r] = bf16_bits(v);
    l[r] = bf16_bits(v - __uint_as_float(h[r] << 16));
  }
  if (!(lane & 1) && tp < TN) {
    uint16_t* p = next + (clip * TP_N + 1 + tp) * CIP_N + co0 + 4 * (lane >> 4);
    *reinterpret_cast<uint2*>(p) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    *reinterpret_cast<uint2*>(p + LO) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
  }
}

// ---- fp32 convolutions by Winograd F(2,3) (the fp32 path) ---------------
// conv1d k3 p1 (cross-correlation) for the output pair (2p, 2p+1) from the
// four input rows d_r = x[2p - 1 + r] (image rows 2p + r):
//   m0 = (d0 - d2) g0,  m1 = (d1 + d2) (g0 + g1 + g2) / 2,
//   m2 = (d2 - d1) (g0 - g1 + g2) / 2,  m3 = (d1 - d3) g2,
//   y(2p) = m0 + m1 + m2,  y(2p+1) = m1 - m2 - m3.
// Four products per input channel for two outputs instead of six: 2/3 of the
// direct form's v_mfma_f32_16x16x4f32 work (on gfx950 the fp32 MFMA shares
// the fp32 datapath with the front-end's VALU, so every MFMA cycle saved is a
// front-end cycle).  The pair is also exactly maxpool(2)'s window, so the
// epilogue pools in-lane.  MFMA columns = pairs; lane (n, q) reads rows
// 2n..2n+3 at ci = 16 cb + 4 q + j (the ci-blocked K order of conv_pair_v, so
// the same packed taps g0, G1, g2 serve; G2 is formed per step).
// boff = this lane's element of row 2n; image pitch CIP = 4 mod 8 keeps the
// stride-2 row reads conflict-free.
template <int CB, int CIP, int CHUNK = 0>
__device__ __forceinline__ void conv_wino_v(const float* __restrict__ img, const float (&w)[12 * CB], int boff,
                                            f32x4 (&m)[4]) {
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    float d[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float4 v = *reinterpret_cast<const float4*>(img + boff + r * CIP + 16 * cb);
      d[r][0] = v.x;
      d[r][1] = v.y;
      d[r][2] = v.z;
      d[r][3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // packed taps g0, G1 = (g0 + g1 + g2) / 2, g2 (pack_fragments); G2 =
      // (g0 - g1 + g2) / 2 = (g0 + g2) - G1, two VALU per step
      const float g0 = w[4 * cb + j], G1 = w[4 * (CB + cb) + j], g2 = w[4 * (2 * CB + cb) + j];
      float sg = g0 + g2;
      asm volatile("" : "+v"(sg));   // keep G2 per step: hoisted out of the caller's loops it costs a VGPR per step
      const float G2 = sg - G1;
      m[0] = mfma4(g0, d[0][j] - d[2][j], m[0]);
      m[1] = mfma4(G1, d[1][j] + d[2][j], m[1]);
      m[2] = mfma4(G2, d[2][j] - d[1][j], m[2]);
      m[3] = mfma4(g2, d[1][j] - d[3][j], m[3]);
    }
    if (CHUNK > 0 && (cb % CHUNK) == CHUNK - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// Winograd output transform + ReLU + maxpool(2): pair p -> pooled row p.
template <int CIP_N, int TP_N, int TN>
__device__ __forceinline__ void epi_wino_pool(const f32x4 (&m)[4], float* __restrict__ next, int co0, int clip, int p0,
                                              int lane) {
  const int p = p0 + (lane & 15);
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float y0 = m[0][r] + m[1][r] + m[2][r], y1 = m[1][r] - m[2][r] - m[3][r];
    v[r] = fmaxf(fmaxf(y0, y1), 0.0f);
  }
  if (p < TN) {
    *reinterpret_cast<float4*>(next + (clip * TP_N + 1 + p) * CIP_N + co0 + 4 * (lane >> 4)) =
        make_float4(v[0], v[1], v[2], v[3]);
  }
}

// conv3's tile holds two clips (columns 0-7: clip ca, 8-15: clip ca + 1; 8
// pairs each, the 8th dropped by the floor pool): pooled -> mean over the 7.
template <int GSTRIDE>
__device__ __forceinline__ void epi_wino_gap(const f32x4 (&m)[4], float* __restrict__ g, int co0, int ca, int lane) {
  const int p = lane & 7;
  const int clip = ca + ((lane >> 3) & 1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float y0 = m[0][r] + m[1][r] + m[2][r], y1 = m[1][r] - m[2][r] - m[3][r];
    float s = p < 7 ? fmaxf(fmaxf(y0, y1), 0.0f) : 0.0f;
    s += dpp<0xB1>(s);    // 8-lane sum: quad_perm xor 1, xor 2, row_half_mirror
    s += dpp<0x4E>(s);
    s += dpp<0x141>(s);
    if (p == 0) {
      g[(co0 + 4 * (lane >> 4) + r) * GSTRIDE + clip] = s * (1.0f / 7.0f);
    }
  }
}

}  // namespace wk
