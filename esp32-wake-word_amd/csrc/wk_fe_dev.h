// wk_fe_dev.h -- device code of the MFCC front-end (shared by the standalone
// front-end kernel, wk_frontend.hip, and the fused kernel, wk_fused.hip).
// See wk_frontend.hip for the algorithm and the reference citations.
#pragma once
#include "wk_common.h"
#include "wk_tables.h"

namespace wk {

// W32^k2 = exp(-2*pi*i*k2/32), k2 = 0..8.
__device__ __forceinline__ f2 w32(int k2) {
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

// Raw samples of one frame-group slot, prefetched into registers one round
// ahead (buffer loads: clip base in SGPRs, out-of-range reads return 0):
// x0[n1] = x[r(i0)], x1[n1] = x[r(i0+1)] for i0 = base + 32*n1 + 2j, with
// r() the reflection of torch.stft's centre padding (mode B) -- identity
// except on the two edge frames.  The pre-emphasis partner of each sample is
// a neighbouring lane's value (DPP row rotate), so it is not loaded twice;
// xb covers the one partner outside the slot (lane 0: x[r(base-1)], lane 15:
// x[r(i0(9,15)+2)]).  Kept in the input type so the loads stay outstanding
// until first use.
template <typename T>
struct Raw {
  T x0[10], x1[10];
  T xb;
};

template <typename T> __device__ __forceinline__ T raw_ld(__amdgpu_buffer_rsrc_t r, int idx);
template <> __device__ __forceinline__ float raw_ld<float>(__amdgpu_buffer_rsrc_t r, int idx) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, 0));
}
template <> __device__ __forceinline__ int16_t raw_ld<int16_t>(__amdgpu_buffer_rsrc_t r, int idx) {
  return (int16_t)__builtin_amdgcn_raw_buffer_load_b16(r, idx * 2, 0, 0);
}

// The adjacent pair x[idx], x[idx + 1] as one 8-byte (fp32) / 4-byte (int16)
// load: half the load instructions of two raw_ld (the front-end's loads are
// issue-bound: 8 front-end waves per CU share one load path).
template <typename T> __device__ __forceinline__ void raw_ld2(__amdgpu_buffer_rsrc_t r, int idx, T& a, T& b);
template <> __device__ __forceinline__ void raw_ld2<float>(__amdgpu_buffer_rsrc_t r, int idx, float& a, float& b) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, idx * 4, 0, 0);
  a = __uint_as_float(v[0]);   // (not __builtin_bit_cast of a vector element: miscompiled to v[0] for both)
  b = __uint_as_float(v[1]);
}
template <> __device__ __forceinline__ void raw_ld2<int16_t>(__amdgpu_buffer_rsrc_t r, int idx, int16_t& a,
                                                            int16_t& b) {
  const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(r, idx * 2, 0, 0);
  a = (int16_t)(v & 0xFFFFu);
  b = (int16_t)(v >> 16);
}

// Reflect index i of the centred (padded) signal of length n into [0, n).
__device__ __forceinline__ int refl_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i > n - 1 ? 2 * (n - 1) - i : i;
}

// GENERAL (wave-uniform) = this wave-round holds an edge frame: per-lane
// reflected indices.  Otherwise the 21 loads share one offset VGPR.
template <bool MODE_B, typename T>
__device__ __forceinline__ void load_raw(__amdgpu_buffer_rsrc_t rs, int base, int j, int n, bool act, bool general,
                                         Raw<T>& r) {
  if (!act) return;
  if (!general) {
    const int v0 = base + 2 * j;
#pragma unroll
    for (int n1 = 0; n1 < 10; ++n1) raw_ld2<T>(rs, v0 + 32 * n1, r.x0[n1], r.x1[n1]);
    r.xb = raw_ld<T>(rs, base - 1);   // mode A frame 0: index -1 -> 0 (y[0] = x[0], mfcc.c:70)
  } else {
#pragma unroll
    for (int n1 = 0; n1 < 10; ++n1) {
      const int i0 = base + 32 * n1 + 2 * j;
      r.x0[n1] = raw_ld<T>(rs, MODE_B ? refl_idx(i0, n) : i0);
      r.x1[n1] = raw_ld<T>(rs, MODE_B ? refl_idx(i0 + 1, n) : i0 + 1);
    }
    const int ib = j == 15 ? base + 32 * 9 + 32 : base - 1;
    r.xb = raw_ld<T>(rs, MODE_B ? refl_idx(ib, n) : ib);
  }
}

// Part k (0..3) of load_raw: rows n1 with pf_part(n1) == k (and xb with part
// 0), so a round's prefetch can be spread over the round instead of issued as
// one burst (eight waves issuing 11 loads each at once filled the TA FIFOs and
// stalled issue).  The edge-frame (GENERAL) form is issued whole with part 0.
// The packed unit front-loads the parts (rows 0-3, 4-6, 7-8, 9) and issues
// them earlier in the round (fe_rest); the scalar unit issues rows 3k..3k+2.
__device__ __forceinline__ constexpr int pf_part(int n1) {
  return WK_FE_STAGED ? n1 / 3 : (n1 < 4 ? 0 : n1 < 7 ? 1 : n1 < 9 ? 2 : 3);
}
template <bool MODE_B, typename T>
__device__ __forceinline__ void load_raw_part(__amdgpu_buffer_rsrc_t rs, int base, int j, int n, bool act,
                                              bool general, Raw<T>& r, int part) {
  if (!act) return;
  if (general) {
    if (part == 0) load_raw<MODE_B, T>(rs, base, j, n, act, true, r);
    return;
  }
  const int v0 = base + 2 * j;
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1)
    if (pf_part(n1) == part) raw_ld2<T>(rs, v0 + 32 * n1, r.x0[n1], r.x1[n1]);
  if (part == 0) r.xb = raw_ld<T>(rs, base - 1);
}

struct NoPrefetch {
  __device__ __forceinline__ void operator()(int) const {}
};

__device__ __forceinline__ float row_ror1(float v) {  // lane l <- lane (l-1) mod 16 of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_rol1(float v) {  // lane l <- lane (l+1) mod 16 of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x12F, 0xF, 0xF, false));
}

// LDS tables shared by the workgroup (fe_init_tables).
struct FeTables {
  const float* win;   // [320] analysis window, odd rows n1 negated in lanes j >= 8 (kWinB / kWinA)
  const float* tw;    // [16 slots][16 lanes][2]: W256^(j * (s ^ (j & 8)))
};

// Split twiddles tws(k2, j) = fe_split_tw(j, k2), k2 = 1..7: the [7][16] f2 table in LDS.
struct TwsLds {
  const float* p;
  __device__ __forceinline__ f2 operator()(int k2, int j) const {
    return *reinterpret_cast<const f2*>(p + ((k2 - 1) * 16 + j) * 2);
  }
};

// The real-FFT split pairs bin k = j + 16 k2 (lane j, register k2) with bin
// 256 - k (lane (16 - j) & 15).  After the one-pass transpose of fe_rest the
// lanes j >= 8 hold (-1)^k2 Z[k]; when a lane and its partner hold their
// values with opposite signs, S and D of the split trade places, and the
// twiddle -conj(W) in place of W restores |U|^2 and |U'|^2 exactly:
//   D - i(-conj W) S = i conj(W) (S - i W D),  D + i(-conj W) S = -i conj(W) (S + i W D).
__device__ __forceinline__ bool fe_split_flip(int j, int k2) {
  return j == 8 || (j >= 1 && j <= 7 && !(k2 & 1)) || (j >= 9 && (k2 & 1));
}
__device__ __forceinline__ f2 fe_split_tw(int j, int k2) {   // W512^(j + 16 k2), or -conj of it
  float sn, cs;
  sincospif(-(float)(j + 16 * k2) / 256.0f, &sn, &cs);
  return fe_split_flip(j, k2) ? f2{-cs, sn} : f2{cs, sn};
}
__device__ __forceinline__ void fe_init_tws(float* tws, int tid, int nthreads) {
  for (int i = tid; i < 7 * 16; i += nthreads) {
    const f2 w = fe_split_tw(i % 16, i / 16 + 1);
    tws[2 * i] = w.x;
    tws[2 * i + 1] = w.y;
  }
}

// Stage 0: pre-emphasis + window of the 320 frame samples as 160 complex
// (even, odd) pairs: lane j holds pair index 16*n1 + j, n1 = 0..9.
//   y[i] = x[i] - 0.97 x[i-1], y[0] = x[0]   (torchaudio preemphasis / mfcc.c:66-74)
// On reflected rows (mode B edge frames) y(i0) = x[r] - 0.97 x[r-1] pairs
// each sample with the NEXT one: own x1 for y0, the next lane's x0 for y1.
template <bool MODE_B, typename T>
__device__ __forceinline__ void fe_stage0(const Raw<T>& raw, int base, int n, int j, bool general,
                                          const FeTables& tb, f2 (&a)[16], float pre = -0.97f WK_SP_PARAM) {
  // All ten window pairs are read up front: issued one per iteration they
  // each exposed a full LDS round trip (the edge-frame branch kept the
  // compiler from hoisting them).
  f2 w[10];
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) w[n1] = *reinterpret_cast<const f2*>(tb.win + 32 * n1 + 2 * j);
  float prev_rot = 0.0f;
  float y0[10], y1[10];
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) {
    const float x0 = to_f(raw.x0[n1]), x1 = to_f(raw.x1[n1]);
    // x[i0-1]: lane j-1's x1 of this row; lane 0 takes lane 15's x1 of the previous row.
    // DPP row rotates read other lanes: they must execute with the whole row
    // active, so they are materialised (asm barrier) before any lane select.
    float rot = row_ror1(x1);
    asm volatile("" : "+v"(rot));
    const float xm = j != 0 ? rot : (n1 == 0 ? to_f(raw.xb) : prev_rot);
    prev_rot = rot;
    y0[n1] = __builtin_fmaf(pre, xm, x0);   // pre = -0.97 (0 for mfcc.c's single-frame variant)
    y1[n1] = __builtin_fmaf(pre, x0, x1);
  }
  // The windowed pairs are formed in each branch, so the two paths merge on
  // a[] (register pairs) rather than on y0/y1 (merging the halves cost ~15
  // v_mov per round to re-pair them on the common path).
  if (MODE_B && general) {   // wave-uniform: the two reflected edge frames only
#pragma unroll
    for (int n1 = 0; n1 < 10; ++n1) {
      const float x0 = to_f(raw.x0[n1]), x1 = to_f(raw.x1[n1]);
      const int i0 = base + 32 * n1 + 2 * j;
      float nx = row_rol1(x0);
      float nx1 = row_rol1(to_f(raw.x0[n1 + 1 < 10 ? n1 + 1 : 9]));
      asm volatile("" : "+v"(nx), "+v"(nx1));
      const float xn = j != 15 ? nx : (n1 < 9 ? nx1 : to_f(raw.xb));
      const bool reflected = i0 < 0 || i0 > n - 1;
      const float r0 = __builtin_fmaf(pre, x1, x0), r1 = __builtin_fmaf(pre, xn, x1);
      const float g0 = reflected ? r0 : (i0 == 0 ? x0 : y0[n1]);
      const float g1 = reflected ? r1 : y1[n1];
      a[n1] = f2{g0, g1} * w[n1];
    }
  } else {
#pragma unroll
    for (int n1 = 0; n1 < 10; ++n1) a[n1] = f2{y0[n1], y1[n1]} * w[n1];
  }
#pragma unroll
  for (int n1 = 10; n1 < 16; ++n1) a[n1] = f2{0.0f, 0.0f};
}

// Stages 1..4 of one frame -> its power row (bins 0..256) in LDS.  All
// complex arithmetic is packed fp32 (see f2 in wk_common.h).
// xs: 8-byte aligned transpose scratch of 270 floats inside the frame's row
// (row + 0 or row + 1; kPRow = 271).
// w0: fe_split_tw(j, 0); tws(k2, j): fe_split_tw(j, k2), k2 = 1..7.
// pf(k), k = 0..3, is called at four points of the round (prefetch parts);
// pf(-1) just before the round's first write into the row.
//
// 256-point complex FFT of the 160 (even, odd) sample pairs, four-step 16 x 16:
//   Z[k1 + 16 k2] = sum_n2 W16^(n2 k2) W256^(n2 k1) sum_n1 W16^(n1 k1) z[16 n1 + n2]
// with lane j = n2 for the first DFT16 and lane kc = k1 for the second.
// One-pass transpose of {re, im} pairs: with h = j & 8 the lanes j >= 8 hold
// their first-pass outputs in slot order k1 ^ 8 (their window rows n1 odd are
// negated: A[k1 ^ 8] = sum_n1 (-1)^n1 W16^(n1 k1) a[n1]), so every lane's
// slots 0-7 are the 8x8 blocks on the diagonal ((n2, k1) in the same half)
// and slots 8-15 the off-diagonal blocks.  Each half is 128 complex values;
// element (n2, k1) of the diagonal half sits at f2 index 17 (n2 & 7) + k1,
// of the other at 17 (n2 & 7) + (k1 ^ 8): lane-uniform immediate offsets for
// the writes (base 17 (j & 7) + h, offset s) and the reads (base kc or kc ^ 8,
// offset 17 s), each 16 lanes on 16 distinct 8-byte bank pairs, and 135
// f2 = 270 floats, inside the frame's own row.  Per round: 8 ds_write2_b64 +
// 8 ds_read2_b64 (the re / im two-pass transpose was 16 write2 + 32 reads).
// The second DFT16 then sees its inputs rotated by 8 in lanes kc >= 8, which
// multiplies Z[kc + 16 k2] by (-1)^k2 there; fe_split_tw absorbs the sign.
template <bool MODE_B, typename PF, typename TWS>
__device__ __forceinline__ void fe_rest(f2 (&a)[16], int j, float* __restrict__ row, float* __restrict__ xs,
                                        const FeTables& tb, f2 w0, const TWS& tws, int esp_pack,
                                        const PF& pf WK_SP_PARAM) {
  pf(0);
  dft16(a);  // slot s: A[s ^ (j & 8)] at a[dft16_out(s)]
  WK_FE_HIT(2);

  // twiddle W256^(n2 k1), n2 = j, k1 = s ^ (j & 8); each half is twiddled
  // just before it is written (fewer live registers)
  f2* x2 = reinterpret_cast<f2*>(xs);
  const int wb = 17 * (j & 7) + (j & 8);
  auto tw = [&](int s) { return cmul2(a[dft16_out(s)], *reinterpret_cast<const f2*>(tb.tw + (s * 16 + j) * 2)); };
  f2 b[8];
  if constexpr (!WK_FE_STAGED) pf(1);
#pragma unroll
  for (int s = 0; s < 8; ++s) b[s] = tw(s);
  pf(-1);   // the first write into this frame's LDS row follows (fused kernel: wait until the row is free)
#pragma unroll
  for (int s = 0; s < 8; ++s) x2[wb + s] = b[s];
  WK_FE_HIT(3);
  if constexpr (WK_FE_STAGED) pf(1);
  f2 c[16];
  wave_lds_sync();
#pragma unroll
  for (int s = 0; s < 8; ++s) c[s] = x2[j + 17 * s];
  // The packed unit issues prefetch parts 1-3 one step earlier than the
  // scalar unit (part 1 before the twiddles, part 2 after these reads, part 3
  // before the second DFT16 rather than after it): the loads get ~1 k more
  // cycles to land before the next round needs them; with the front-loaded
  // parts, fp32 +1.5 % (profiles/r06u..r06x); the scalar unit
  // measured -0.5 to 0 % with the earlier parts 2-3.
  if constexpr (!WK_FE_STAGED) pf(2);
#pragma unroll
  for (int s = 8; s < 16; ++s) b[s - 8] = tw(s);
  wave_lds_sync();
#pragma unroll
  for (int s = 8; s < 16; ++s) x2[wb + s - 8] = b[s - 8];
  wave_lds_sync();
#pragma unroll
  for (int s = 8; s < 16; ++s) c[s] = x2[(j ^ 8) + 17 * (s - 8)];
  wave_lds_sync();
  WK_FE_HIT(4);

  if constexpr (WK_FE_STAGED) {
    pf(2);
    dft16(c);  // +-Z[j + 16*k2] at c[dft16_out(k2)]
    pf(3);
  } else {
    pf(3);
    dft16(c);
  }
  WK_FE_HIT(5);

  // Real-FFT split, k = j + 16*k2 (k2 = 0..7), with the partner Z[256 - k]:
  //   S = Z[k] + conj Z[256-k],  D = Z[k] - conj Z[256-k],  bb = W512^k D,
  //   U = 2 X[k] = S - i bb,  U' = conj(2 X[256-k]) = S + i bb
  // (mode B folds the 1/4 of |X|^2 = |U|^2/4 into the filterbank weights).
  // {|U|^2, |U'|^2} is one packed pair: {Ux, U'x}^2 + {Uy, U'y}^2.
  // Partner: lane (16-j)&15 of this group, register 15-k2, fetched by two DPP
  // row moves (row_mirror: j <- 15-j, then row_shr:1: j <- j-1), no LDS trip;
  // lane 0 holds its own partner in register (16-k2)&15.  The twiddle is one
  // value per (lane, k2) (w0 / tws), sign-adjusted by fe_split_tw.
  f2 sc0 = {1.0f, 1.0f}, sc = {1.0f, 1.0f};
  if constexpr (!MODE_B) {
    // mfcc.c:267 power = |X|^2 / n_fft + 1e-12 = |U|^2 / 2048 + 1e-12; the
    // esp-dsp dsps_cplx2reC_fc32 packing (mfcc.c:261) doubles bins 1..255
    // (x4 in power) and zeroes bin 256 (parity unpinned).
    const float e = esp_pack ? 4.0f / 2048.0f : 1.0f / 2048.0f;
    sc = f2{e, e};
    sc0 = esp_pack ? (j == 0 ? f2{1.0f / 2048.0f, 0.0f} : sc) : sc;  // j==0, k2==0: bins 0 and 256
  }
  {
    // bin 128 (k2 = 8, column 0): X[128] = conj Z[128], so |U|^2 = 4 |Z[128]|^2.
    const f2 z = c[dft16_out(8)];
    float p128 = 4.0f * __builtin_fmaf(z.x, z.x, z.y * z.y);
    if constexpr (!MODE_B) p128 = __builtin_fmaf(p128, sc.x, 1e-12f);
    if (j == 0) row[128] = p128;
  }
  // The eight k2 chains are ~20 dependent packed ops each; run them G at a
  // time, stage by stage, so independent ops fill each other's latency
  // (left to itself the scheduler emitted them back to back, one chain at a
  // time, with s_nop between dependent v_pk ops).
  // WK_FE_STAGED (the bf16-family unit's scalar front-end, wk_common.h) also
  // issues the group's DPP moves and each chain stage across the group: the
  // same operations per value, bit-identical, bf16 +0.8 % (profiles/
  // r06m_staged_ab.txt); the packed fp32 unit measured -0.1 % with it, so
  // it keeps the per-chain order.
  constexpr int G = 3;
#pragma unroll
  for (int k0 = 0; k0 < 8; k0 += G) {
    f2 S[G], D[G], pw[G];
#if WK_FE_STAGED
    // the partners' row_mirror moves of the group first, then their row_shr
    // moves (a DPP read of a VGPR written by the previous VALU op waits 2 states)
    float mx[G], my[G];
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) {
        const f2 sv = c[dft16_out(15 - k0 - t)];
        mx[t] = dpp<0x140>(sv.x);
        my[t] = dpp<0x140>(sv.y);
      }
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > 7) continue;
      const f2 zk = c[dft16_out(k2)];
      const f2 own = c[dft16_out((16 - k2) & 15)];
      f2 zq;
      zq.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.x), __float_as_int(mx[t]), 0x111, 0xF, 0xF, false));
      zq.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.y), __float_as_int(my[t]), 0x111, 0xF, 0xF, false));
      S[t] = fma2(zq, f2{1.0f, -1.0f}, zk);
      D[t] = fma2(zq, f2{-1.0f, 1.0f}, zk);
    }
#else
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > 7) continue;
      const f2 zk = c[dft16_out(k2)];
      const f2 sv = c[dft16_out(15 - k2)];
      const f2 own = c[dft16_out((16 - k2) & 15)];
      // row_mirror (lane j <- 15 - j), then row_shr:1 (lane j <- j - 1) with
      // bound_ctrl off: lane 0 has no source and keeps `old` = its own
      // partner register -- no lane select.
      f2 zq;
      zq.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.x), __float_as_int(dpp<0x140>(sv.x)),
                                                        0x111, 0xF, 0xF, false));
      zq.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.y), __float_as_int(dpp<0x140>(sv.y)),
                                                        0x111, 0xF, 0xF, false));
      S[t] = fma2(zq, f2{1.0f, -1.0f}, zk);
      D[t] = fma2(zq, f2{-1.0f, 1.0f}, zk);
    }
#endif
#if WK_FE_STAGED
    // the G chains issued stage by stage (the same operations per value)
    f2 wt[G], tt[G], bb[G], uvx[G], uvy[G], sq[G];
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) {
        wt[t] = k0 + t == 0 ? w0 : tws(k0 + t, j);
        tt[t] = cmul2_a(D[t], wt[t]);
      }
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) bb[t] = cmul2_b(D[t], wt[t], tt[t]);
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) {
        uvx[t] = fma2(by(bb[t]), f2{1.0f, -1.0f}, bx(S[t]));
        uvy[t] = fma2(bx(bb[t]), f2{-1.0f, 1.0f}, by(S[t]));
      }
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) sq[t] = uvy[t] * uvy[t];
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > 7) continue;
      pw[t] = fma2(uvx[t], uvx[t], sq[t]);
      if constexpr (!MODE_B) pw[t] = fma2(pw[t], k2 == 0 ? sc0 : sc, f2{1e-12f, 1e-12f});
    }
#else
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > 7) continue;
      const f2 bb = cmul2(D[t], k2 == 0 ? w0 : tws(k2, j));
      const f2 uvx = fma2(by(bb), f2{1.0f, -1.0f}, bx(S[t]));
      const f2 uvy = fma2(bx(bb), f2{-1.0f, 1.0f}, by(S[t]));
      pw[t] = fma2(uvx, uvx, uvy * uvy);
      if constexpr (!MODE_B) pw[t] = fma2(pw[t], k2 == 0 ? sc0 : sc, f2{1e-12f, 1e-12f});
    }
#endif
    // the group's low bins first, then its high bins: same-base stores 16
    // dwords apart, back to back, which the compiler pairs into ds_write2_b32
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) row[j + 16 * (k0 + t)] = pw[t].x;
#pragma unroll
    for (int t = 0; t < G; ++t)
      if (k0 + t <= 7) row[256 - j - 16 * (k0 + t)] = pw[t].y;
  }
  WK_FE_HIT(6);
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
  return d * (1.0f / (sd + 1e-8f));   // wave-uniform reciprocal
}

// Two independent coefficient rows at once (interleaved reductions).
__device__ __forceinline__ void cmvn_lane2(float& v0, float& v1, bool valid, int n) {
  const float m0 = wave_sum(valid ? v0 : 0.0f) / (float)n;
  const float m1 = wave_sum(valid ? v1 : 0.0f) / (float)n;
  const float d0 = valid ? v0 - m0 : 0.0f;
  const float d1 = valid ? v1 - m1 : 0.0f;
  float s0 = sqrtf(wave_sum(d0 * d0) / (float)(n - 1));
  float s1 = sqrtf(wave_sum(d1 * d1) / (float)(n - 1));
  s0 = s0 == 0.0f ? 1.0f : s0;
  s1 = s1 == 0.0f ? 1.0f : s1;
  v0 = d0 * (1.0f / (s0 + 1e-8f));
  v1 = d1 * (1.0f / (s1 + 1e-8f));
}

// LDS carve (floats): twiddles | split twiddles | log-mel [40][64] | power
// rows [63][271] | window.  The standalone front-end stops before the window
// (it reads the window from the constant table: kFeLdsNoWin keeps two
// workgroups per CU); the fused kernel copies it to LDS.
constexpr int kTwOff = 0, kTwSize = 16 * 16 * 2;
constexpr int kTwsOff = kTwOff + kTwSize, kTwsSize = 7 * 16 * 2;
constexpr int kLOff = kTwsOff + kTwsSize, kLSize = 40 * WK_LSTRIDE;
constexpr int kPOff = kLOff + kLSize, kPSize = kNFramesB * kPRow;
constexpr int kFeLdsNoWin = kPOff + kPSize;
constexpr int kWinOff = (kFeLdsNoWin + 1) & ~1, kWinSize = 320;
constexpr int kFeLds = kWinOff + kWinSize;
static_assert(kFeLdsNoWin * 4 <= 81920, "standalone front-end LDS must allow 2 workgroups per CU");
static_assert(kLOff % 4 == 0, "log-mel rows are read with ds_read_b128");
static_assert(kPOff % 2 == 0 && kPRow % 2 == 1 && kPRow >= 271,
              "row f's transpose scratch is row + (f & 1): 8-byte aligned, 270 floats");

// Fill the twiddle tables (and the window, WIN) of the LDS carve (all threads of the WG).
template <bool MODE_B, bool WIN>
__device__ __forceinline__ void fe_init_tables(float* smem, int tid, int nthreads) {
  if (WIN)
    for (int i = tid; i < 320; i += nthreads) smem[kWinOff + i] = MODE_B ? kWinB[i] : kWinA[i];
  for (int i = tid; i < 16 * 16; i += nthreads) {
    const int s = i / 16, jj = i % 16, k1 = s ^ (jj & 8);
    float sn, cs;
    sincospif(-(float)(jj * k1) / 128.0f, &sn, &cs);
    smem[kTwOff + 2 * i] = cs;
    smem[kTwOff + 2 * i + 1] = sn;
  }
  fe_init_tws(smem + kTwsOff, tid, nthreads);
}

}  // namespace wk
