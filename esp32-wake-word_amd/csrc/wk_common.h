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

struct cf {
  float re, im;
};

__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
  return {__builtin_fmaf(a.re, b.re, -a.im * b.im), __builtin_fmaf(a.re, b.im, a.im * b.re)};
}

// cos / -sin of 2*pi*e/16 (forward-DFT twiddle W16^e = exp(-2*pi*i*e/16)).
__device__ __forceinline__ cf w16(int e) {
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

// v * W16^e with the trivial quarter turns folded (e is a constant after unrolling).
__device__ __forceinline__ cf twid16(cf v, int e) {
  switch (e & 15) {
    case 0: return v;
    case 4: return {v.im, -v.re};
    case 8: return {-v.re, -v.im};
    case 12: return {-v.im, v.re};
    default: return cmul(v, w16(e));
  }
}

// In-place 4-point forward DFT.
__device__ __forceinline__ void dft4(cf& a0, cf& a1, cf& a2, cf& a3) {
  const cf t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = csub(a1, a3);
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = {t1.re + t3.im, t1.im - t3.re};  // t1 - i t3
  a3 = {t1.re - t3.im, t1.im + t3.re};  // t1 + i t3
}

// In-register 16-point forward DFT (radix 4x4).  Input a[n] natural order;
// output A[k] lands in a[4*(k&3) + (k>>2)] (use dft16_out()).  Inputs known to
// be zero at compile time fold away (built with -fno-signed-zeros).
__device__ __forceinline__ void dft16(cf (&a)[16]) {
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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Buffer-resource loads: base in SGPRs, per-lane byte offset in one VGPR, a
// wave-uniform byte offset in an SGPR -- no 64-bit VGPR address per load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(int16_t v) { return (float)v * (1.0f / 32768.0f); }

template <typename T> __device__ __forceinline__ float sample(const T* p, int64_t i);
template <> __device__ __forceinline__ float sample<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float sample<int16_t>(const int16_t* p, int64_t i) {
  return (float)p[i] * (1.0f / 32768.0f);
}

}  // namespace wk
