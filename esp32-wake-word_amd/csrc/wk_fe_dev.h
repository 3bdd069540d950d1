// wk_fe_dev.h -- device code of the MFCC front-end (shared by the standalone
// front-end kernel, wk_frontend.hip, and the fused kernel, wk_fused.hip).
// See wk_frontend.hip for the algorithm and the reference citations.
#pragma once
#include "wk_common.h"
#include "wk_tables.h"

#ifndef WK_SPLIT_G
#define WK_SPLIT_G 3   // real-FFT split chains interleaved per group (fe_rest)
#endif
#ifndef WK_SPLIT_MIRROR
#define WK_SPLIT_MIRROR 0   // 1: second-pass columns placed so real-FFT split partners are row mirrors (one DPP)
#endif
#ifndef WK_TW_GROUP
#define WK_TW_GROUP 0   // >0: fence the twiddle LDS reads into groups of this many (0 = compiler schedules; measured equal)
#endif

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

// Part k (0..3) of load_raw: rows n1 in [3k, 3k+3) (and xb with part 0), so
// a round's prefetch can be spread over the round instead of issued as one
// burst (eight waves issuing 11 loads each at once filled the TA FIFOs and
// stalled issue).  The edge-frame (GENERAL) form is issued whole with part 0.
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
    if (n1 / 3 == part) raw_ld2<T>(rs, v0 + 32 * n1, r.x0[n1], r.x1[n1]);
  if (part == 0) r.xb = raw_ld<T>(rs, base - 1);
}

// Column k1 of the second DFT16 pass held by lane j of a 16-lane group.
// Plain: k1 = j; the split partner column 16 - k1 then sits in lane 16 - j
// (two DPP moves).  Mirrored (WK_SPLIT_MIRROR): columns 1-7 in lanes 1-7,
// 9-15 in lanes 8-14, 0 in lane 0, 8 in lane 15 -- the partner of the column
// in lane j is in lane 15 - j (DPP row_mirror), and the two self-partnered
// columns 0 and 8 sit in lanes 0 and 15.
__device__ __forceinline__ constexpr int fe_kcol(int j) {
  return WK_SPLIT_MIRROR ? (j < 8 ? j : (j == 15 ? 8 : j + 1)) : j;
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

// LDS tables shared by the workgroup.
struct FeTables {
  const float* win;   // [320] analysis window (mode-specific)
  const float* tw;    // [15][16][2]: W256^(j*k1), k1 = 1..15
  const float* tws;   // [7][16][2]: W512^(fe_kcol(j) + 16*k2), k2 = 1..7 (TWS kernels only), else null
};

// Fill the combined split twiddles of FeTables::tws (all threads of the WG).
__device__ __forceinline__ void fe_init_tws(float* tws, int tid, int nthreads);

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
// pf(k), k = 0..3, is called at four points of the round (prefetch parts);
// pf(-1) just before the round's first write into `row`.
// TWS: the split's twiddle W512^k, k = kc + 16 k2, is one table value per
// (lane, k2) (tb.tws) instead of W512^kc x the constant W32^k2 -- one complex
// multiply instead of two; bin 128 comes from |Z[128]|^2 directly.
template <bool MODE_B, typename PF = NoPrefetch, bool TWS = false>
__device__ __forceinline__ void fe_rest(f2 (&a)[16], int j, int lane, float* __restrict__ row, const FeTables& tb,
                                        f2 w512, int esp_pack, const PF& pf = PF() WK_SP_PARAM) {
  pf(0);
#ifndef WK_ABL_NODFT   // WK_ABL_*: timing ablations of tools/debug (wrong results)
  dft16(a);  // A[k1] at a[dft16_out(k1)]
#endif
  WK_FE_HIT(2);

  // twiddle W256^(j*k1) + 16x16 transpose through this frame's LDS row (pitch 17).
  // (twiddles are applied in groups of 4 so their LDS reads do not all
  // sit in VGPRs at once; re parts go straight to the transpose image.)
  f2 b[16];
  pf(-1);   // the first write into this frame's LDS row follows (fused kernel: wait until the row is free)
  b[0] = a[0];
  row[j] = b[0].x;
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {
#ifdef WK_ABL_NOTW
    const f2 w = f2{0.5f, 0.25f};
#else
    const f2 w = *reinterpret_cast<const f2*>(tb.tw + ((k1 - 1) * 16 + j) * 2);
#endif
    b[k1] = cmul2(a[dft16_out(k1)], w);
    row[17 * k1 + j] = b[k1].x;
    if (WK_TW_GROUP > 0 && (k1 % (WK_TW_GROUP > 0 ? WK_TW_GROUP : 1)) == WK_TW_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
  }
  WK_FE_HIT(3);
  pf(1);
  f2 c[16];
#ifdef WK_ABL_NOTRANS
  const int kc = fe_kcol(j);
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) c[n2] = b[n2];
#else
  const int kc = fe_kcol(j);   // the column this lane transforms in the second pass
  // The reads are single-dword (volatile: not merged into ds_read2_b32, whose
  // two consecutive destination registers hold two elements' re parts and
  // cost ~24 v_mov per round to re-pair as {re, im}); each lands in its half
  // of c[n2] directly.
  typedef const volatile __attribute__((address_space(3))) float lds_cvf;
  lds_cvf* vrow = (lds_cvf*)(row + 17 * kc);
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) c[n2].x = vrow[n2];
  wave_lds_sync();
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) row[17 * k1 + j] = b[k1].y;
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) c[n2].y = vrow[n2];
  wave_lds_sync();
#endif
  WK_FE_HIT(4);

  pf(2);
#ifndef WK_ABL_NODFT
  dft16(c);  // Z[j + 16*k2] at c[dft16_out(k2)]
#endif
  pf(3);
  WK_FE_HIT(5);

  // Real-FFT split, k = j + 16*k2 (k2 = 0..8), with the partner Z[256 - k]:
  //   S = Z[k] + conj Z[256-k],  D = Z[k] - conj Z[256-k],  bb = W512^k D,
  //   U = 2 X[k] = S - i bb,  U' = conj(2 X[256-k]) = S + i bb
  // (mode B folds the 1/4 of |X|^2 = |U|^2/4 into the filterbank weights).
  // {|U|^2, |U'|^2} is one packed pair: {Ux, U'x}^2 + {Uy, U'y}^2.
  // Partner: lane (16-j)&15 of this group, register 15-k2, fetched by two DPP
  // row moves (row_mirror: j <- 15-j, then row_ror:1: j <- j-1), no LDS trip;
  // lane 0 holds its own partner in register (16-k2)&15.
#ifdef WK_SPLIT_BPERMUTE
  const int src = ((lane & 48) | ((16 - j) & 15)) << 2;
#endif
  f2 sc0 = {1.0f, 1.0f}, sc = {1.0f, 1.0f};
  if constexpr (!MODE_B) {
    // mfcc.c:267 power = |X|^2 / n_fft + 1e-12 = |U|^2 / 2048 + 1e-12; the
    // esp-dsp dsps_cplx2reC_fc32 packing (mfcc.c:261) doubles bins 1..255
    // (x4 in power) and zeroes bin 256 (parity unpinned).
    const float e = esp_pack ? 4.0f / 2048.0f : 1.0f / 2048.0f;
    sc = f2{e, e};
    sc0 = esp_pack ? (j == 0 ? f2{1.0f / 2048.0f, 0.0f} : sc) : sc;  // j==0, k2==0: bins 0 and 256
  }
  // The nine k2 chains are ~20 dependent packed ops each; run them WK_SPLIT_G
  // at a time, stage by stage, so independent ops fill each other's latency
  // (left to itself the scheduler emitted them back to back, one chain at a
  // time, with s_nop between dependent v_pk ops).
#ifdef WK_ABL_NOSPLIT
  row[j] = c[0].x + c[1].y + c[5].x + c[9].y + c[13].x;
  return;
#endif
  constexpr int G = WK_SPLIT_G;
  constexpr int K2MAX = TWS ? 7 : 8;
  if constexpr (TWS) {
    // bin 128 (k2 = 8, column 0): X[128] = conj Z[128], so |U|^2 = 4 |Z[128]|^2.
    const f2 z = c[dft16_out(8)];
    float p128 = 4.0f * __builtin_fmaf(z.x, z.x, z.y * z.y);
    if constexpr (!MODE_B) p128 = __builtin_fmaf(p128, sc.x, 1e-12f);
    if (j == 0) row[128] = p128;
  }
#pragma unroll
  for (int k0 = 0; k0 <= K2MAX; k0 += G) {
    f2 S[G], D[G], pw[G];
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > K2MAX) continue;
      const f2 zk = c[dft16_out(k2)];
      f2 zq;
      if (k2 < 8) {
        const f2 sv = c[dft16_out(15 - k2)];
        const f2 own = c[dft16_out((16 - k2) & 15)];
#if WK_SPLIT_MIRROR
        // lane 15 - j holds the partner column; lanes 0 (column 0) and 15
        // (column 8) are their own partners: registers (16 - k2) & 15 / 15 - k2.
        const float pr = dpp<0x140>(sv.x);
        const float pi = dpp<0x140>(sv.y);
        zq = j == 0 ? own : (j == 15 ? sv : f2{pr, pi});
#else
#ifdef WK_SPLIT_BPERMUTE
        const float pr = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(sv.x)));
        const float pi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(sv.y)));
        zq = j == 0 ? own : f2{pr, pi};
#else
        // row_mirror (lane j <- 15 - j), then row_shr:1 (lane j <- j - 1) with
        // bound_ctrl off: lane 0 has no source and keeps `old` = its own
        // partner register -- no lane select.
        zq.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.x), __float_as_int(dpp<0x140>(sv.x)),
                                                          0x111, 0xF, 0xF, false));
        zq.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(own.y), __float_as_int(dpp<0x140>(sv.y)),
                                                          0x111, 0xF, 0xF, false));
#endif
#endif
      } else {
        zq = c[dft16_out(8)];
      }
      S[t] = fma2(zq, f2{1.0f, -1.0f}, zk);
      D[t] = fma2(zq, f2{-1.0f, 1.0f}, zk);
    }
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (TWS || k2 > 8) continue;
      if (k2 == 8) D[t] = swp(D[t]) * f2{1.0f, -1.0f};   // W32^8 = -i
      else if (k2 > 0) D[t] = cmulc(D[t], w32(k2));
    }
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > K2MAX) continue;
      f2 wk = w512;
      if (TWS && k2 > 0) wk = *reinterpret_cast<const f2*>(tb.tws + ((k2 - 1) * 16 + j) * 2);
      const f2 bb = cmul2(D[t], wk);
      const f2 uvx = fma2(by(bb), f2{1.0f, -1.0f}, bx(S[t]));
      const f2 uvy = fma2(bx(bb), f2{-1.0f, 1.0f}, by(S[t]));
      pw[t] = fma2(uvx, uvx, uvy * uvy);
      if constexpr (!MODE_B) pw[t] = fma2(pw[t], k2 == 0 ? sc0 : sc, f2{1e-12f, 1e-12f});
    }
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const int k2 = k0 + t;
      if (k2 > K2MAX) continue;
      const int kb = kc + 16 * k2;
      if (k2 < 8) {
        row[kb] = pw[t].x;
        row[256 - kb] = pw[t].y;
      } else if (j == 0) {
        row[128] = pw[t].x;
      }
    }
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

__device__ __forceinline__ f2 fe_w512(int j) {
  float sn, cs;
  sincospif(-(float)j / 256.0f, &sn, &cs);
  return f2{cs, sn};
}
__device__ __forceinline__ f2 fe_w512_lane(int j) { return fe_w512(fe_kcol(j)); }   // W512^k1 of the lane's column

__device__ __forceinline__ void fe_init_tws(float* tws, int tid, int nthreads) {
  for (int i = tid; i < 7 * 16; i += nthreads) {
    const int k2 = i / 16 + 1, jj = i % 16;
    float sn, cs;
    sincospif(-(float)(fe_kcol(jj) + 16 * k2) / 256.0f, &sn, &cs);
    tws[2 * i] = cs;
    tws[2 * i + 1] = sn;
  }
}

}  // namespace wk
