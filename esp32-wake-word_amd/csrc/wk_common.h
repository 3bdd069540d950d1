// wk_common.h -- shared device helpers for the wake-word kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wk {

constexpr int kWinSamples = 16000;   // 1 s @ 16 kHz (extract_mfcc.py:157)
constexpr int kNFramesB = 63;        // 1 + 16000/256 with center=True
constexpr int kPRow = 271;           // LDS pitch of one frame's power row (odd: lane-per-frame reads
                                     // conflict-free; >=271 so the 16x17 transpose scratch fits)
constexpr int kFeBlock = 512;        // 8 waves per front-end workgroup

// Complex values live in VGPR pairs as float2 {re, im}: the front-end's
// complex arithmetic then compiles to packed fp32 VALU (v_pk_add/mul/fma_f32,
// two lanes' worth of fp32 per issue), swaps and sign flips folded into the
// op_sel / neg modifiers.
// Diagnostic builds (and -DWK_FE_PACKED_ALL, the A/B baseline) compile the
// whole fused kernel in one translation unit (wk_fused.hip), with the packed
// front-end in every precision.
#if defined(WK_DIAG) || defined(WK_FE_PACKED_ALL)
#define WK_FUSED_ONE_TU 1
#else
#define WK_FUSED_ONE_TU 0
#endif

#if defined(WK_FE_SCALAR) && defined(WK_FUSED_TU)
// The fused kernel's bf16-family unit (wk_fused_xdl.hip): the same complex
// arithmetic as scalar fp32 pairs (v_fma/v_add/v_mul_f32; swaps and signs are
// register choices and VOP3 neg modifiers), no packed ops -- beside the bf16
// MFMAs those issue faster (wk_fused.hip header).
// WK_FE_STAGED marks this unit wherever the two units' front-end schedules
// differ, each measured in its own unit: the real-FFT split
// issued stage by stage across each group of chains and the prefetch
// placement (wk_fe_dev.h fe_rest), the round-1 frame slots (wk_fused.hip).
#define WK_FE_STAGED 1
struct __attribute__((aligned(8))) f2 {
  float x, y;
};
__device__ __forceinline__ f2 operator+(f2 a, f2 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ f2 operator-(f2 a, f2 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ f2 operator*(f2 a, f2 b) { return {a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f2 operator-(f2 a) { return {-a.x, -a.y}; }
__device__ __forceinline__ f2& operator+=(f2& a, f2 b) { return a = a + b; }
__device__ __forceinline__ f2& operator-=(f2& a, f2 b) { return a = a - b; }
__device__ __forceinline__ f2& operator*=(f2& a, f2 b) { return a = a * b; }
__device__ __forceinline__ f2 swp(f2 a) { return {a.y, a.x}; }
__device__ __forceinline__ f2 bx(f2 a) { return {a.x, a.x}; }
__device__ __forceinline__ f2 by(f2 a) { return {a.y, a.y}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return {__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)}; }
#else
#define WK_FE_STAGED 0
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 swp(f2 a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ f2 bx(f2 a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ f2 by(f2 a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
#endif
__device__ __forceinline__ f2 sub_ib(f2 a, f2 b) { return fma2(swp(b), f2{1.0f, -1.0f}, a); }  // a - i b
__device__ __forceinline__ f2 add_ib(f2 a, f2 b) { return fma2(swp(b), f2{-1.0f, 1.0f}, a); }  // a + i b

// a * w, w = {c, s} a runtime twiddle: v_pk_mul + one v_pk_fma whose second
// operand is w swizzled to {-s, s} by op_sel/neg_lo (the compiler would
// build that pair with two extra VALU ops).
__device__ __forceinline__ f2 cmul2(f2 a, f2 w) {
#if defined(WK_FE_SCALAR) && defined(WK_FUSED_TU)
  return {__builtin_fmaf(-a.y, w.y, a.x * w.x), __builtin_fmaf(a.x, w.y, a.y * w.x)};
#endif
  const f2 t = a * bx(w);
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
// cmul2 in two phases, t = cmul2_a(a, w) then cmul2_b(a, w, t), for a group
// of independent products issued phase by phase (WK_FE_STAGED): the same
// operations as cmul2, so the same bits.
__device__ __forceinline__ f2 cmul2_a(f2 a, f2 w) { return a * bx(w); }
__device__ __forceinline__ f2 cmul2_b(f2 a, f2 w, f2 t) {
#if defined(WK_FE_SCALAR) && defined(WK_FUSED_TU)
  return {__builtin_fmaf(-a.y, w.y, t.x), __builtin_fmaf(a.x, w.y, t.y)};
#else
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
#endif
}
// a * w for a compile-time constant w.
__device__ __forceinline__ f2 cmulc(f2 a, f2 w) { return fma2(swp(a), f2{-w.y, w.y}, a * f2{w.x, w.x}); }

// W16^e = exp(-2*pi*i*e/16).
__device__ __forceinline__ f2 w16(int e) {
  constexpr float c8 = 0.92387953251128674f, s8 = 0.38268343236508978f, h = 0.70710678118654752f;
  switch (e & 15) {
    case 0: return {1.f, 0.f};
    case 1: return {c8, -s8};
    case 2: return {h, -h};
    case 3: return {s8, -c8};
    case 4: return {0.f, -1.f};
    case 5: return {-s8, -c8};
    case 6: return {-h, -h};
    case 7: return {-c8, -s8};
    case 8: return {-1.f, 0.f};
    case 9: return {-c8, s8};
    case 10: return {-h, h};
    case 11: return {-s8, c8};
    case 12: return {0.f, 1.f};
    case 13: return {s8, c8};
    case 14: return {h, h};
    default: return {c8, s8};
  }
}

__device__ __forceinline__ f2 swap_mul(f2 v, f2 s) { return swp(v) * s; }
// v * W16^e with the quarter turns folded (e is a constant after unrolling).
__device__ __forceinline__ f2 twid16(f2 v, int e) {
  switch (e & 15) {
    case 0: return v;
    case 4: return swap_mul(v, f2{1.0f, -1.0f});    // -i v
    case 8: return -v;
    case 12: return swap_mul(v, f2{-1.0f, 1.0f});   // i v
    default: return cmulc(v, w16(e));
  }
}

// In-place 4-point forward DFT (8 packed ops).
__device__ __forceinline__ void dft4(f2& a0, f2& a1, f2& a2, f2& a3) {
  const f2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = sub_ib(t1, t3);
  a3 = add_ib(t1, t3);
}

// In-register 16-point forward DFT (radix 4x4).  Input a[n] natural order;
// output A[k] lands in a[4*(k&3) + (k>>2)] (use dft16_out()).  Inputs known to
// be zero at compile time fold away (built with -fno-signed-zeros).
__device__ __forceinline__ void dft16(f2 (&a)[16]) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) dft4(a[nb], a[4 + nb], a[8 + nb], a[12 + nb]);
#pragma unroll
  for (int ka = 1; ka < 4; ++ka)
#pragma unroll
    for (int nb = 1; nb < 4; ++nb) a[4 * ka + nb] = twid16(a[4 * ka + nb], nb * ka);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) dft4(a[4 * ka], a[4 * ka + 1], a[4 * ka + 2], a[4 * ka + 3]);
}
__device__ __forceinline__ constexpr int dft16_out(int k) { return 4 * (k & 3) + (k >> 2); }

// Wave-scope ordering of LDS traffic between lanes of one wave: LDS ops of a
// wave execute in order, so only the compiler must be kept from moving them.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// then s_barrier.  Unlike __syncthreads() it does not drain vmcnt, so global
// loads issued as prefetch stay in flight across it.
__device__ __forceinline__ void wg_barrier_lds() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int CTRL> __device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 64 lanes, result in every lane.  Within each 16-lane row the
// butterflies are DPP (quad_perm xor1, xor2, row_half_mirror, row_mirror);
// the four row sums are combined through SGPRs (v_readlane) -- no LDS
// round trips (a __shfl_xor reduction is six dependent ds_bpermute).
// Must be called with all 64 lanes active.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// Buffer-resource loads: base in SGPRs, per-lane byte offset in one VGPR, a
// wave-uniform byte offset in an SGPR -- no 64-bit VGPR address per load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// Natural log for the log-mel stage: v_log_f32 (log2, ~1 ulp; arguments are
// >= 1e-12, never denormal) times ln 2, instead of the ~20-instruction libm
// expansion.  Differs from torch.log by ~1e-7 relative (parity tolerance
// of the features is 5e-4).
__device__ __forceinline__ float wk_logf(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(int16_t v) { return (float)v * (1.0f / 32768.0f); }

template <typename T> __device__ __forceinline__ float sample(const T* p, int64_t i);
template <> __device__ __forceinline__ float sample<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float sample<int16_t>(const int16_t* p, int64_t i) {
  return (float)p[i] * (1.0f / 32768.0f);
}

// Diagnostic builds only (-DWK_DIAG, tools/debug): per-phase s_memtime
// cycle sums.  Device helpers take an optional WkStamps* (WK_SP_PARAM) and
// mark phase ends with WK_FE_HIT(k); product builds compile all of it away.
#ifdef WK_DIAG
struct WkStamps {
  unsigned long long st[16];
  unsigned long long tl;
  __device__ void init() {
    for (int k = 0; k < 16; ++k) st[k] = 0;
    tl = __builtin_amdgcn_s_memtime();
  }
  __device__ void hit(int k) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    st[k] += t - tl;
    tl = t;
  }
};
#define WK_SP_PARAM , WkStamps* stp = nullptr
#define WK_FE_HIT(k) do { if (stp) stp->hit(k); } while (0)
#else
#define WK_SP_PARAM
#define WK_FE_HIT(k) do {} while (0)
#endif

}  // namespace wk
