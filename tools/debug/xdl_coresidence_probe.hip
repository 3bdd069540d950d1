// Minimal co-residence probe for the K = 32 question.
//
// The fused kernel's front-end values change run to run when its CNN waves
// use the K = 32 MFMA forms (v_mfma_f32_16x16x32_{bf16,f16}) on the same SIMDs,
// and not with the K = 16 pair.  This program asks whether that needs the
// fused kernel at all: one 1,024-thread workgroup per CU, waves 0-7 run a
// deterministic packed-fp32 VALU chain (v_pk_fma_f32 / v_pk_mul_f32 rotations,
// a DPP row_mirror exchange and an LDS round trip per iteration, the front-end's
// instruction mix), waves 8-15 run an MFMA stream for as long as any VALU wave
// is running.  Every wave index maps to SIMDs as in the fused kernel (two of
// each role per SIMD).  The VALU results must not depend on the MFMA form.
//
//   hipcc -O3 --offload-arch=gfx950 -o xdl_probe tools/debug/xdl_coresidence_probe.hip
//   ./xdl_probe [repeats] [iterations] [variant bits 0-31]
//
// Prints, per MFMA mode and repeat, how many VALU lanes differ from mode 0
// (no MFMA stream) and the lane histogram of the differences.
// Diagnostic tool, not product code.
#include <hip/hip_runtime.h>

#ifndef WK_PROBE_CHAINS
#define WK_PROBE_CHAINS 8   // packed-fp32 chains per VALU lane (-DWK_PROBE_CHAINS=48: ~110 VGPRs, the front-end's register range)
#endif

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 1024, kValuWaves = 8, kChains = WK_PROBE_CHAINS;
constexpr int kOutBlocks = 9;            // f32x4 outputs per VALU lane
constexpr int kLdsFloats = 24 * 1024;   // ~96 KB: one workgroup per CU

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul_swap_neg(f32x2 a, f32x2 b) {   // {-a.y * b.x, a.x * b.y}
  f32x2 d;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ f32x2 pk_fma_s(f32x2 a, f32x2 b_sgpr, f32x2 c) {   // a constant in an SGPR pair
  f32x2 d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_sgpr), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul_swap_neg_s(f32x2 a, f32x2 b_sgpr) {
  f32x2 d;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(a), "s"(b_sgpr));
  return d;
}
__device__ __forceinline__ float dpp_shr1_keep(float old, float x) {   // row_shr:1, bound_ctrl off: lane 0 of a row keeps old
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x),
                                                               0x111, 0xf, 0xf, false));
}
// The front-end's in-register DFT16 (wk_common.h: dft4 / twid16 / dft16, the
// same packed-fp32 forms), restated here so the probe stays standalone.
__device__ __forceinline__ f32x2 p_swp(f32x2 a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ f32x2 p_fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 p_twid(f32x2 v, int e) {
  constexpr float c8 = 0.92387953251128674f, s8 = 0.38268343236508978f, h = 0.70710678118654752f;
  const float W[16][2] = {{1.f, 0.f}, {c8, -s8}, {h, -h}, {s8, -c8}, {0.f, -1.f}, {-s8, -c8}, {-h, -h}, {-c8, -s8},
                          {-1.f, 0.f}, {-c8, s8}, {-h, h}, {-s8, c8}, {0.f, 1.f}, {s8, c8}, {h, h}, {c8, s8}};
  switch (e & 15) {
    case 0: return v;
    case 4: return p_swp(v) * f32x2{1.0f, -1.0f};
    case 8: return -v;
    case 12: return p_swp(v) * f32x2{-1.0f, 1.0f};
    default: return p_fma2(p_swp(v), f32x2{-W[e & 15][1], W[e & 15][1]}, v * f32x2{W[e & 15][0], W[e & 15][0]});
  }
}
__device__ __forceinline__ void p_dft4(f32x2& a0, f32x2& a1, f32x2& a2, f32x2& a3) {
  const f32x2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = p_fma2(p_swp(t3), f32x2{1.0f, -1.0f}, t1);
  a3 = p_fma2(p_swp(t3), f32x2{-1.0f, 1.0f}, t1);
}
// -i v as one packed op (the swap in op_sel, the sign from a {1, -1} constant):
// the compiler's own form of p_twid(v, 4) is two v_mov_b32 (a register-pair
// swap) with the sign folded into a later op.
__device__ __forceinline__ f32x2 p_mul_negi_pk(f32x2 v) {
  f32x2 r;
  const f32x2 c = {1.0f, -1.0f};
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(v), "v"(c));
  return r;
}
// The quarter turn -i v as the compiler builds it in sub 5 -- two v_mov_b32
// into the halves of a register pair, then a packed op reading the pair --
// written out in asm on a fixed pair (v80:v81) so the spacing is exact:
// NOP = false back to back (the bisected form), true with s_nop 7 (8 wait
// states) between the pair's writes and the packed read.  The round-6
// wait-state experiment (DESIGN.md 5.1, K = 32 rule).
template <bool NOP>
__device__ __forceinline__ f32x2 p_mul_negi_movpair(f32x2 v) {
  f32x2 r;
  const f32x2 c = {1.0f, -1.0f};
  if (NOP)
    asm volatile("v_mov_b32 v80, %1\n\tv_mov_b32 v81, %2\n\ts_nop 7\n\tv_pk_mul_f32 %0, v[80:81], %3"
                 : "=v"(r) : "v"(v.y), "v"(v.x), "v"(c) : "v80", "v81");
  else
    asm volatile("v_mov_b32 v80, %1\n\tv_mov_b32 v81, %2\n\tv_pk_mul_f32 %0, v[80:81], %3"
                 : "=v"(r) : "v"(v.y), "v"(v.x), "v"(c) : "v80", "v81");
  return r;
}
template <int KA>
__device__ __forceinline__ void p_rowgroup(f32x2 (&a)[16]) {
#pragma unroll
  for (int nb = 1; nb < 4; ++nb) a[4 * KA + nb] = p_twid(a[4 * KA + nb], nb * KA);
  p_dft4(a[4 * KA], a[4 * KA + 1], a[4 * KA + 2], a[4 * KA + 3]);
}
__device__ __forceinline__ void p_dft16(f32x2 (&a)[16]) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) p_dft4(a[nb], a[4 + nb], a[8 + nb], a[12 + nb]);
#pragma unroll
  for (int ka = 1; ka < 4; ++ka)
#pragma unroll
    for (int nb = 1; nb < 4; ++nb) a[4 * ka + nb] = p_twid(a[4 * ka + nb], nb * ka);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) p_dft4(a[4 * ka], a[4 * ka + 1], a[4 * ka + 2], a[4 * ka + 3]);
}

__device__ __forceinline__ float dpp_mirror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xf, 0xf, false));
}

// MODE 0: no MFMA stream, 1: K = 16 bf16 pair, 2: K = 32 bf16, 3: K = 32 f16,
// 4-6 K = 32 bf16 with A/B, everything, or the accumulator in AGPRs, 7 the fp32
// v_mfma_f32_16x16x4_f32, 8 the int8 v_mfma_i32_16x16x64_i8 (XDL_PROBE_MODES="0278" etc.).
// VAR bits (0 = VGPR constants, row_mirror only): 1 = SGPR-pair constants and
// the split's row_mirror -> row_shr:1 (bound_ctrl off) pair; 2 = v_log_f32 /
// v_exp_f32 and a lane select per iteration; 4 = the MFMA waves read their B
// operand from LDS and store their accumulators to LDS (the CNN role's epilogue
// stores), in their own LDS range; 32 = the VALU waves run the front-end's
// in-register DFT16 instead of the rotations; 64 = one packed-fp32 form,
// chosen by VAR >> 8: 0 v_pk_add_f32, 1 the same with neg (a subtract), 2
// v_pk_fma_f32 with a swapped source and an SGPR-pair constant, 3 v_pk_mul_f32
// by an SGPR constant's low half, 4 v_pk_fma_f32 with an SGPR-pair factor,
// 5 v_pk_fma_f32 all-VGPR; +128: the 16 ops back to back on one chain.
// 8 = each iteration adds a value loaded from global memory (a buffer load into
// VGPRs, as the front-end's audio loads) and a 64-bit LDS table read (its
// twiddles); 16 = the MFMA waves leave ~3/4 of their issue time idle
// (s_sleep between groups of MFMAs, the CNN role's MFMA share) instead of a
// dense stream.
template <int MODE>
__global__ __launch_bounds__(kThreads) void probe_kernel(int iters, int VAR, const float* __restrict__ table,
                                                         float* __restrict__ out, float* __restrict__ mout,
                                                         unsigned* __restrict__ info) {
  __shared__ float lds[kLdsFloats];
  __shared__ unsigned done;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) done = 0;
  for (int i = tid; i < 1024; i += kThreads) lds[4096 + i] = 1e-3f * (float)((i * 37) % 101) - 0.05f;   // the LDS table
  __syncthreads();
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // hwreg(HW_REG_HW_ID)
  if (lane == 0) info[blockIdx.x * 16 + wave] = (hw >> 4) & 3u;   // the wave's SIMD
  if (wave < kValuWaves) {
    // rotations by a fixed angle: norm-preserving, so a perturbation persists
    const float c = 0.99875026f, s = 0.04997917f;   // cos / sin 0.05
    const f32x2 cc = {c, c}, ss = {s, s};
    f32x2 v[kChains];
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      const float a = 0.25f + 1e-3f * (float)((blockIdx.x * 64 + lane) % 977) + 0.01f * k;
      v[k] = f32x2{a, 1.0f - a};
    }
    float* my = lds + wave * 64 * 4;
    f32x2 sum = {0.0f, 0.0f};
    f32x2 dd[16] = {};
    if (VAR & 64) {   // one packed-fp32 instruction form, form = VAR >> 8 (16 independent chains)
      const int form = VAR >> 8;
      f32x2 d[16], y[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        d[q] = f32x2{0.01f * (float)((lane * 7 + q * 3 + blockIdx.x) % 29) - 0.14f, 0.01f * (float)((lane + q * 5) % 31) - 0.15f};
        y[q] = f32x2{1e-4f * (float)((lane + q) % 13), -1e-4f * (float)((lane * 3 + q) % 11)};
      }
      const f32x2 ce = {0.00390625f, -0.00390625f}, cm = {-1.0f, 0.5f};
      const bool dep = VAR & 128;   // 128: all 16 ops on chain 0, each reading the previous one's result
      for (int it = 0; it < iters; ++it) {
        if (form == 0) {
#pragma unroll
          for (int q = 0; q < 16; ++q) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(d[dep ? 0 : q]) : "v"(d[dep ? 0 : q]), "v"(y[q]));
        } else if (form == 1) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d[dep ? 0 : q]) : "v"(d[dep ? 0 : q]), "v"(y[q]));
        } else if (form == 2) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1]" : "=v"(d[dep ? 0 : q]) : "v"(d[dep ? 0 : q]), "s"(ce), "v"(d[dep ? 0 : q]));
        } else if (form == 3) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(d[dep ? 0 : q]) : "v"(d[dep ? 0 : q]), "s"(cm));
        } else if (form == 4) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d[q]) : "v"(y[q]), "s"(cm), "v"(d[dep ? 0 : q]));
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d[dep ? 0 : q]) : "v"(d[dep ? 0 : q]), "v"(y[q]), "v"(d[dep ? 0 : q]));
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) sum += d[q];
#pragma unroll
      for (int q = 0; q < 16; ++q) dd[q] = d[q];
    } else if (VAR & 32) {   // the front-end's DFT16, scaled by 1/4 per pass (norm-preserving)
      f32x2 d[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        d[q] = f32x2{0.01f * (float)((lane * 7 + q * 3 + blockIdx.x) % 29) - 0.14f, 0.01f * (float)((lane + q * 5) % 31) - 0.15f};
      const int sub = VAR >> 8;   // 0 the DFT16; 1 its two DFT4 passes without twiddles; 2 the twiddles only;
                                  // 3 one DFT4 pass; 4 the DFT4 pass of rows only (no swapped operands: a0/a2 sums);
                                  // 5 twiddles + the row pass; 6 the column pass + twiddles;
                                  // 7-9 row group ka = sub - 6 alone (twiddles + DFT4);
                                  // 10 sub 5 with the quarter turn as one packed op;
                                  // 11 / 12 sub 5 with the quarter turn as an explicit v_mov_b32 pair
                                  // + packed read, with (11) / without (12) 8 wait states between them
      for (int it = 0; it < iters; ++it) {
        if (sub == 0) {
          p_dft16(d);
        } else if (sub == 1) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) p_dft4(d[nb], d[4 + nb], d[8 + nb], d[12 + nb]);
#pragma unroll
          for (int ka = 0; ka < 4; ++ka) p_dft4(d[4 * ka], d[4 * ka + 1], d[4 * ka + 2], d[4 * ka + 3]);
        } else if (sub == 2) {
#pragma unroll
          for (int ka = 1; ka < 4; ++ka)
#pragma unroll
            for (int nb = 1; nb < 4; ++nb) d[4 * ka + nb] = p_twid(d[4 * ka + nb], nb * ka);
        } else if (sub == 5 || sub == 6) {   // 5: twiddles then the row DFT4 pass; 6: the column pass then the twiddles
          if (sub == 6) {
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) p_dft4(d[nb], d[4 + nb], d[8 + nb], d[12 + nb]);
          }
#pragma unroll
          for (int ka = 1; ka < 4; ++ka)
#pragma unroll
            for (int nb = 1; nb < 4; ++nb) d[4 * ka + nb] = p_twid(d[4 * ka + nb], nb * ka);
          if (sub == 5) {
#pragma unroll
            for (int ka = 0; ka < 4; ++ka) p_dft4(d[4 * ka], d[4 * ka + 1], d[4 * ka + 2], d[4 * ka + 3]);
          }
        } else if (sub == 10) {   // sub 5 with the quarter-turn twiddle (ka 2, nb 2) as one packed op
#pragma unroll
          for (int ka = 1; ka < 4; ++ka)
#pragma unroll
            for (int nb = 1; nb < 4; ++nb)
              d[4 * ka + nb] = (nb * ka == 4) ? p_mul_negi_pk(d[4 * ka + nb]) : p_twid(d[4 * ka + nb], nb * ka);
#pragma unroll
          for (int ka = 0; ka < 4; ++ka) p_dft4(d[4 * ka], d[4 * ka + 1], d[4 * ka + 2], d[4 * ka + 3]);
        } else if (sub == 11 || sub == 12) {   // sub 5, the quarter turn as an explicit v_mov_b32 pair (+ s_nop 7 in 11)
#pragma unroll
          for (int ka = 1; ka < 4; ++ka)
#pragma unroll
            for (int nb = 1; nb < 4; ++nb)
              d[4 * ka + nb] = (nb * ka != 4)   ? p_twid(d[4 * ka + nb], nb * ka)
                               : sub == 11 ? p_mul_negi_movpair<true>(d[4 * ka + nb])
                                           : p_mul_negi_movpair<false>(d[4 * ka + nb]);
#pragma unroll
          for (int ka = 0; ka < 4; ++ka) p_dft4(d[4 * ka], d[4 * ka + 1], d[4 * ka + 2], d[4 * ka + 3]);
        } else if (sub == 7) {   // one row group ka = sub - 6: its twiddles, then its DFT4
          p_rowgroup<1>(d);
        } else if (sub == 8) {
          p_rowgroup<2>(d);
        } else if (sub == 9) {
          p_rowgroup<3>(d);
        } else if (sub == 3) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) p_dft4(d[nb], d[4 + nb], d[8 + nb], d[12 + nb]);
        } else {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) {
            const f32x2 t0 = d[nb] + d[8 + nb], t1 = d[nb] - d[8 + nb], t2 = d[4 + nb] + d[12 + nb], t3 = d[4 + nb] - d[12 + nb];
            d[nb] = t0 + t2;
            d[8 + nb] = t0 - t2;
            d[4 + nb] = t1 + t3;
            d[12 + nb] = t1 - t3;
          }
        }
        const float sc = sub == 2 ? 1.0f : sub >= 3 ? 0.5f : 0.25f;   // (10-12 too)   // (5, 6: one pass, x 1/2)   // keeps the norm
#pragma unroll
        for (int q = 0; q < 16; ++q) d[q] *= f32x2{sc, sc};
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) sum += d[q] * f32x2{(float)(q + 1), (float)(17 - q)};
#pragma unroll
      for (int q = 0; q < 16; ++q) dd[q] = d[q];
    } else
    for (int it = 0; it < iters; ++it) {
      if (!(VAR & 1)) {
#pragma unroll
        for (int k = 0; k < kChains; ++k) v[k] = pk_fma(v[k], cc, pk_mul_swap_neg(v[k], ss));
      } else {
#pragma unroll
        for (int k = 0; k < kChains; ++k) v[k] = pk_fma_s(v[k], cc, pk_mul_swap_neg_s(v[k], ss));
      }
      // DPP exchange (the real-FFT split's partner fetch) and an LDS round trip
      float m = dpp_mirror(v[0].x);
      if (VAR & 1) m = dpp_shr1_keep(v[kChains - 1].y, m);
      if (VAR & 2) {
        const float l = __builtin_amdgcn_logf(fabsf(m) + 1.0f);
        m = (lane & 4) ? m : m + 1e-3f * __builtin_amdgcn_exp2f(-l);
      }
      if (VAR & 8) {
        const float g = table[(it * 64 + lane) & 4095];
        const f32x2 tw = reinterpret_cast<const f32x2*>(lds + 4096)[(it + lane) & 511];
        m = fmaf(g, tw.x, m) + tw.y;
      }
      my[lane] = m;
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
      const float back = my[63 - lane];
      sum = pk_fma(f32x2{m, back}, f32x2{1.0f, 1.0f}, sum);
    }
    f32x4* o = reinterpret_cast<f32x4*>(out) + ((size_t)blockIdx.x * kValuWaves + wave) * 64 * kOutBlocks;
    if (VAR & 96) {   // the 16 complex registers, then the weighted sum
#pragma unroll
      for (int k = 0; k < 16; k += 2) o[(k / 2) * 64 + lane] = f32x4{dd[k].x, dd[k].y, dd[k + 1].x, dd[k + 1].y};
    } else {
#pragma unroll
      for (int k = 0; k < kChains && k < 16; k += 2) o[(k / 2) * 64 + lane] = f32x4{v[k].x, v[k].y, v[k + 1].x, v[k + 1].y};
    }
    o[8 * 64 + lane] = f32x4{sum.x, sum.y, 0.0f, 0.0f};
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0) atomicAdd(&done, 1u);
  } else {
    f32x4 acc[4] = {};
    s16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (short)(0x3f80 + ((lane + i) & 7));
      b[i] = (short)(0x3c00 + ((lane * 3 + i) & 7));
    }
    if (VAR & 4) {
      s16x8* dst = reinterpret_cast<s16x8*>(lds + 8192 + (wave - kValuWaves) * 1024);
      dst[lane] = b;
    }
    const int cap = 64 * iters + 4096;   // every wave leaves: bounded even if a VALU wave never signals
    if (MODE != 0) {
      for (int n = 0; n < cap; n += 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          f32x4& c = acc[j & 3];
          if (VAR & 4) {   // B from LDS (the waves' own range, beyond the VALU waves')
            const s16x8* src = reinterpret_cast<const s16x8*>(lds + 8192 + (wave - kValuWaves) * 1024);
            b = src[(lane + j) & 63];
          }
          if (MODE == 1) {
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 0, 1, 2, 3),
                                                          __builtin_shufflevector(b, b, 0, 1, 2, 3), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 4, 5, 6, 7),
                                                          __builtin_shufflevector(b, b, 4, 5, 6, 7), c, 0, 0, 0);
          } else if (MODE == 2) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                        0, 0, 0);
          } else if (MODE == 7) {   // the product's fp32 form, v_mfma_f32_16x16x4_f32 (fp32 convolutions)
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(float, (int)a[0] << 16),
                                                     __builtin_bit_cast(float, (int)b[0] << 16), c, 0, 0, 0);
          } else if (MODE == 8) {   // the int8 K = 64 form, v_mfma_i32_16x16x64_i8 (wk_int8.hip)
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            c = __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, a), __builtin_bit_cast(i32x4, b),
                                                                                __builtin_bit_cast(i32x4, c), 0, 0, 0));
          } else if (MODE == 4) {   // K = 32 bf16, A and B operands in AGPRs
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "a"(b));
          } else if (MODE == 5) {   // K = 32 bf16, A, B and the accumulator in AGPRs
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "a"(a), "a"(b));
          } else if (MODE == 6) {   // K = 32 bf16, the accumulator in AGPRs, A and B in VGPRs
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                       0, 0);
          }
        }
        if (VAR & 16) __builtin_amdgcn_s_sleep(8);
        if (VAR & 4) {   // epilogue-like stores of the accumulators
          f32x4* dst = reinterpret_cast<f32x4*>(lds + 8192 + (wave - kValuWaves) * 1024 + 256);
          dst[lane] = acc[0];
          dst[64 - 1 - lane] = acc[1];
        }
        if (__builtin_amdgcn_readfirstlane(*(volatile unsigned*)&done) >= (unsigned)kValuWaves) break;
      }
    }
    f32x4* o = reinterpret_cast<f32x4*>(mout) + ((size_t)blockIdx.x * (16 - kValuWaves) + (wave - kValuWaves)) * 64;
    o[lane] = acc[0] + acc[1] + acc[2] + acc[3];
  }
}

static void launch_mode(int mode, int var, int grid, int iters, const float* table, float* out, float* m,
                        unsigned* info) {
  switch (mode) {
    case 0: hipLaunchKernelGGL(probe_kernel<0>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 1: hipLaunchKernelGGL(probe_kernel<1>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 2: hipLaunchKernelGGL(probe_kernel<2>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 3: hipLaunchKernelGGL(probe_kernel<3>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 4: hipLaunchKernelGGL(probe_kernel<4>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 5: hipLaunchKernelGGL(probe_kernel<5>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 6: hipLaunchKernelGGL(probe_kernel<6>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 7: hipLaunchKernelGGL(probe_kernel<7>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    default: hipLaunchKernelGGL(probe_kernel<8>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 4000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus;
  const size_t nv = (size_t)grid * kValuWaves * 64 * kOutBlocks * 4, nm = (size_t)grid * 8 * 64 * 4;
  float *d_out, *d_m;
  unsigned* d_info;
  CHECK(hipMalloc(&d_out, nv * 4));
  CHECK(hipMalloc(&d_m, nm * 4));
  CHECK(hipMalloc(&d_info, (size_t)grid * 16 * 4));
  std::vector<float> ref(nv), got(nv), table(4096);
  for (int i = 0; i < 4096; ++i) table[i] = 1e-3f * (float)((i * 53) % 97) - 0.04f;
  float* d_table;
  CHECK(hipMalloc(&d_table, 4096 * 4));
  CHECK(hipMemcpy(d_table, table.data(), 4096 * 4, hipMemcpyHostToDevice));
  std::vector<unsigned> info((size_t)grid * 16);
  const int var = argc > 3 ? atoi(argv[3]) : 0;
  auto launch = [&](int mode) {
    CHECK(hipMemset(d_out, 0, nv * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    launch_mode(mode, var, grid, iters, d_table, d_out, d_m, d_info);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(got.data(), d_out, nv * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(info.data(), d_info, info.size() * 4, hipMemcpyDeviceToHost));
    return ms;
  };
  launch(0);
  ref = got;
  {   // the role placement: VALU and MFMA waves per SIMD in workgroup 0
    int cnt[4][2] = {};
    for (int w = 0; w < 16; ++w) cnt[info[w] & 3][w >= kValuWaves]++;
    printf("workgroup 0 placement (valu, mfma) per SIMD: (%d,%d) (%d,%d) (%d,%d) (%d,%d)\n", cnt[0][0], cnt[0][1],
           cnt[1][0], cnt[1][1], cnt[2][0], cnt[2][1], cnt[3][0], cnt[3][1]);
  }
  printf("valu variant %d, %d iterations\n", var, iters);
  const char* names[9] = {"none",         "k16_bf16_pair", "k32_bf16",      "k32_f16",      "k32_ab_agpr",
                          "k32_all_agpr", "k32_acc_agpr",  "f32_16x16x4",   "i8_16x16x64"};
  const char* sel = getenv("XDL_PROBE_MODES");   // e.g. "0127": the modes to run (default 0-3)
  for (int mode = 0; mode < 9; ++mode) {
    if (sel ? !strchr(sel, '0' + mode) : mode > 3) continue;
    for (int r = 0; r < reps; ++r) {
      const float ms = launch(mode);
      long diff = 0;
      int hist[64] = {}, slot[64] = {};
      const size_t per_wave = 64 * kOutBlocks * 4;
      for (size_t i = 0; i < nv; ++i)
        if (memcmp(&got[i], &ref[i], 4) != 0) {
          ++diff;
          hist[(i % per_wave) / 4 % 64]++;
          slot[((i % per_wave) / 256) * 4 + (i % 4)]++;   // the lane's output float: d[q].x/.y (float 2q, 2q + 1), then sum.x, sum.y at 32, 33
        }
      printf("mode %-14s rep %d: %.3f ms, differing values %ld", names[mode], r, ms, diff);
      if (diff) {
        printf("; by lane:");
        for (int l = 0; l < 64; ++l)
          if (hist[l]) printf(" %d:%d", l, hist[l]);
        printf("; by output float:");
        for (int l = 0; l < 4 * kOutBlocks; ++l)
          if (slot[l]) printf(" %d:%d", l, slot[l]);
      }
      printf("\n");
      fflush(stdout);
    }
  }
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_m));
  CHECK(hipFree(d_info));
  return 0;
}
