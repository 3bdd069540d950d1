// wk_ctc.hip -- the GRU-CTC head (ml_models/ctc.py) on gfx950.
//
//   audio -> log-mel 80 + global z-score (ctc.py:82-107)
//         -> Linear 80->128 + LayerNorm + ReLU (ctc.py:125-130)
//         -> 2-layer bidirectional GRU, H = 128 (ctc.py:133-140)
//         -> Linear 256->V, log_softmax (ctc.py:143-152)
//         -> greedy CTC decode (ctc.py:453-471)
//
// Kernels:
//   ctc_logmel_fft2_kernel reflect-padded frames x periodic Hann(400) -> 400-point
//                         real DFT (two frames per complex 20 x 20 four-step FFT)
//                         -> power -> HTK mel -> ln(+1e-8), fused; optionally the
//                         z-score's per-pass partial sums.
//   ctc_zstats_kernel     {mean, 1/std} per utterance from those partials.
//   ctc_zscore_kernel     one block per utterance, two-pass mean / unbiased std.
//   ctc_encoder_kernel    Linear 80->128 as fp32 MFMA tiles of 16 rows, LayerNorm
//                         by in-register + 16-lane shuffle sums.
//   ctc_gemm_nt_kernel    the GEMMs that materialise a [rows][N] tensor (the fp32
//                         parity mode's input projections and output layer, the
//                         fp16 A/B path's projections): 128 x 128 MFMA block
//                         tiles over LDS-staged K chunks, fp32 or fp16 operands,
//                         fp32 accumulate.
//   ctc_gru_kernel        persistent recurrence: one 768-thread block per
//                         (16 utterances, direction); W_hh lives in VGPRs as
//                         fp32 MFMA A fragments (2 of the 24 16-row tiles per
//                         wave); per step 16x16x4 MFMAs against h (LDS), gate
//                         pre-activations through LDS, gates + state update.
//   ctc_argmax_kernel     one wave per row: bias, max/argmax (first index),
//                         log-sum-exp, optional log_softmax output.
//   ctc_argmax_only_kernel  the same argmax when no log-probs are asked for:
//                         persistent, bias in LDS, a row's loads issued a row
//                         ahead, no exp.
//   ctc_greedy_kernel     one wave per utterance: drop blanks, collapse repeats.
#include <float.h>
#include <stdlib.h>
#include <string.h>

#include <math.h>
#include <type_traits>
#include <functional>
#include <algorithm>
#include <vector>

#include <hip/hip_fp16.h>

#include "wk_cnn_dev.h"
#include "wk_kernels.h"

using namespace wk;

namespace {

constexpr int kNfft = 400, kHop = 160, kBins = kNfft / 2 + 1, kMels = 80, kH = 128;

// ---------------------------------------------------------------------------
// X1: log-mel.  The 400-point DFT is 20 x 20 four-step (n = 20 n1 + n2,
// k = k1 + 20 k2), each DFT-20 4 x DFT-5 + constant twiddles + 5 x DFT-4 in
// packed fp32 (ctc_logmel_fft2_kernel below).
// ---------------------------------------------------------------------------
// W20^e = exp(-2 pi i e / 20).
__constant__ constexpr float kW20c[20] = {1.000000000e+00f, 9.510565163e-01f, 8.090169944e-01f, 5.877852523e-01f, 3.090169944e-01f, 0.000000000e+00f, -3.090169944e-01f, -5.877852523e-01f, -8.090169944e-01f, -9.510565163e-01f, -1.000000000e+00f, -9.510565163e-01f, -8.090169944e-01f, -5.877852523e-01f, -3.090169944e-01f, 0.000000000e+00f, 3.090169944e-01f, 5.877852523e-01f, 8.090169944e-01f, 9.510565163e-01f};
__constant__ constexpr float kW20s[20] = {0.000000000e+00f, -3.090169944e-01f, -5.877852523e-01f, -8.090169944e-01f, -9.510565163e-01f, -1.000000000e+00f, -9.510565163e-01f, -8.090169944e-01f, -5.877852523e-01f, -3.090169944e-01f, 0.000000000e+00f, 3.090169944e-01f, 5.877852523e-01f, 8.090169944e-01f, 9.510565163e-01f, 1.000000000e+00f, 9.510565163e-01f, 8.090169944e-01f, 5.877852523e-01f, 3.090169944e-01f};
__device__ __forceinline__ f2 w20(int e) { return f2{kW20c[e % 20], kW20s[e % 20]}; }

// In-register DFT-5 (forward), natural order in and out.
__device__ __forceinline__ void dft5(f2& x0, f2& x1, f2& x2, f2& x3, f2& x4) {
  constexpr float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
  constexpr float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
  const f2 t1 = x1 + x4, t2 = x2 + x3, t3 = x1 - x4, t4 = x2 - x3;
  const f2 a1 = fma2(f2{c2, c2}, t2, fma2(f2{c1, c1}, t1, x0));
  const f2 a2 = fma2(f2{c1, c1}, t2, fma2(f2{c2, c2}, t1, x0));
  const f2 b1 = fma2(f2{s2, s2}, t4, f2{s1, s1} * t3);   // Y1 = a1 - i b1, Y4 = a1 + i b1
  const f2 b2 = fma2(f2{-s1, -s1}, t4, f2{s2, s2} * t3); // Y2 = a2 - i b2, Y3 = a2 + i b2
  x0 = x0 + t1 + t2;
  x1 = sub_ib(a1, b1);
  x4 = add_ib(a1, b1);
  x2 = sub_ib(a2, b2);
  x3 = add_ib(a2, b2);
}

// In-register DFT-20 (forward): x[0..19] natural order -> X[k] in x[k].
// n = 4 m + r: DFT-5 over m per r, twiddle W20^(r ka), DFT-4 over r per ka;
// X[ka + 5 kb] comes out of the DFT-4 of column ka at position kb.
__device__ __forceinline__ void dft20(f2 (&x)[20]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) dft5(x[r], x[4 + r], x[8 + r], x[12 + r], x[16 + r]);   // B[r][ka] at x[4 ka + r]
#pragma unroll
  for (int r = 1; r < 4; ++r)
#pragma unroll
    for (int ka = 1; ka < 5; ++ka) x[4 * ka + r] = cmulc(x[4 * ka + r], w20(r * ka));
  f2 y[20];
#pragma unroll
  for (int ka = 0; ka < 5; ++ka) {
    f2 b0 = x[4 * ka], b1 = x[4 * ka + 1], b2 = x[4 * ka + 2], b3 = x[4 * ka + 3];
    dft4(b0, b1, b2, b3);
    y[ka] = b0;
    y[ka + 5] = b1;
    y[ka + 10] = b2;
    y[ka + 15] = b3;
  }
#pragma unroll
  for (int k = 0; k < 20; ++k) x[k] = y[k];
}


// ---------------------------------------------------------------------------
// X1, two frames per complex FFT (round 3).  The 400-point DFT of a real frame
// wastes half of a complex FFT, so a lane group runs one complex four-step FFT
// on z = x_a + i x_b of two frames and separates the spectra afterwards:
// X_a[k] = (Z[k] + conj Z[400-k]) / 2, X_b[k] = (Z[k] - conj Z[400-k]) / (2i).
// Lane (g = lane / 20, q = lane % 20) of a wave owns frame pair g (rows
// 6 ps + 2 g, + 1; lanes 60-63 idle):
//   stage 1: lane (g, n2 = q): DFT-20 over n1 of z[20 n1 + n2] -> A[n2][k1],
//            all 20 k1 (no conjugate symmetry for a complex input);
//   stage 2: lane (g, k1 = q): twiddle W400^(n2 k1), DFT-20 over n2 ->
//            Z[k1 + 20 k2] in v[k2];
//   exchange: the partner of bin k1 + 20 k2 is 400 - k1 - 20 k2 =
//            (20 - k1) + 20 (19 - k2) in lane 20 - k1 (k1 > 0), or
//            20 (20 - k2) in the lane itself (k1 = 0): every lane publishes
//            v[10..19] (lane 0 also v[0]) and reads its partner's, one LDS
//            round trip;
//   power:   |Z[k] + conj Z'|^2 and |Z[k] - conj Z'|^2 for k = q + 20 k2,
//            k2 = 0..9 (bin 200 by lane 0), stored as {P_a, P_b} pairs; the
//            1/4 of the separation rides in the mel weights (exact);
//   mel:     straight-line per-lane windows (weights in registers), one
//            8-byte read per pair and tap feeding two FMAs, then ln(+1e-8).
// One 12-wave workgroup per CU (3 waves per SIMD), the tables once per CU.
// LDS pitches (see the per-access notes) keep the stage-1 writes, stage-2
// reads and pair-power writes free of bank conflicts.
// ---------------------------------------------------------------------------
constexpr int kF2Waves = 12, kF2Pairs = 3;
constexpr int kTwPitch = 21;    // twiddle rows (float2): stage-2 reads, lane = k1
constexpr int kMelW1 = 8, kMelW2 = 7;   // mel windows: mels 0-63 <= 8 bins, mels 64-79 <= 14 = 2 x 7 (host-checked)
constexpr int kA2Pitch = 25;    // A[g][n2][k1] rows (float2): 25 = 1 mod 8 -> stage-2 lane groups start 40 banks apart
constexpr int kE2Pitch = 11;   // exchange rows (float2): 22 dwords -> 20 partner rows on distinct banks
                                // (pitch 12 put them on 8 bank pairs: 24 p mod 64 has period 8)
constexpr int kP2Pitch = 212;   // pair-power rows (float2): 2 x 212 = 40 mod 64 banks between lane groups
static_assert(kF2Pairs * kP2Pitch <= kF2Pairs * 20 * kA2Pitch, "power rows alias the A region");
static_assert(kF2Pairs * 20 * kE2Pitch <= kF2Pairs * 20 * kA2Pitch, "exchange rows alias the A region");
struct CtcFft2Lds {
  float win[kNfft];
  f2 tw[20][kTwPitch];
  f2 w[kF2Waves][kF2Pairs * 20 * kA2Pitch];   // per wave: A, then the exchange, then the power rows
};

// Passes (6 rows each) are dealt to the waves in contiguous ranges of R
// (wave W takes passes [W R, W R + R)), so a wave walks its rows in order: the
// (utterance, frame) of its rows advance by addition, with one division per
// range rather than per pass.
//
// STATS (wk_ctc_transcribe, fp16 mode, T >= 6): the features stay un-normalised
// and each wave also leaves, per utterance its range touches, the sums of
// (x - K) and (x - K)^2 over that utterance's log-mel values x in its rows, with
// K = ln(1e-8) the floor of x (so a silent utterance sums to exactly 0): lanes
// keep running sums while the utterance lasts and reduce them across the wave
// only when it changes (2-3 times per range instead of once per pass).  Slot
// part[W MS + j] holds the range's j-th utterance; ctc_zstats_kernel folds the
// slots into each utterance's mean and 1/std, which the encoder applies as it
// loads.
__device__ __forceinline__ float row16_sum(float v) {   // every lane: the sum over its 16-lane row (DPP)
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v;
}
__device__ __forceinline__ float sum_rows4(float v);
template <bool STATS>
__global__ __launch_bounds__(kF2Waves * 64, 1) void ctc_logmel_fft2_kernel(const float* __restrict__ audio, int64_t stride,
                                                                            int n_valid, int n_pad, int T, int64_t rows,
                                                                            const float* __restrict__ win_g,
                                                                            const float* __restrict__ tw_g,
                                                                            const float* __restrict__ melw,
                                                                            const int* __restrict__ melws,
                                                                            float* __restrict__ feats,
                                                                            int64_t R, int MS,
                                                                            float2* __restrict__ part) {
  __shared__ CtcFft2Lds L;
  constexpr int NT = kF2Waves * 64;
  for (int i = threadIdx.x; i < kNfft; i += NT) L.win[i] = win_g[i];
  for (int i = threadIdx.x; i < 400; i += NT) L.tw[i / 20][i % 20] = f2{tw_g[2 * i], tw_g[2 * i + 1]};
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (buffer resources)
  const int g = lane / 20, q = lane - 20 * (lane / 20);   // pair slot (3 = idle lanes 60-63), n2 / k1
  f2* A = L.w[wv];
  typedef volatile __attribute__((address_space(3))) f2 vlf2;
#define LM_R(p, i) (*(const vlf2*)((p) + (i)))
#define LM_W(p, i, val) (*(vlf2*)((p) + (i)) = (val))
  constexpr int kRowsPerPass = 2 * kF2Pairs;
  const int64_t passes = (rows + kRowsPerPass - 1) / kRowsPerPass;
  const int64_t wid = (int64_t)blockIdx.x * kF2Waves + wv;
  const int64_t p_beg = wid * R, p_end = p_beg + R < passes ? p_beg + R : passes;
  const int nv_min = n_valid < n_pad ? n_valid : n_pad;
  // The lane's 20 samples x[20 n1 + q] of one frame (row) of pass ps_; idle
  // lanes and rows past the end read utterance 0's first samples (nothing
  // they compute is stored).  Wave-uniform paths, exactly 20 loads each.
  auto load_one = [&](bool live, int b, int t, float (&raw)[20]) {
    const float* xa = audio + (int64_t)(live ? b : 0) * stride;
    const int p0 = live ? t * kHop - kNfft / 2 : 0;
    if (__all(p0 >= 0 && p0 + kNfft <= nv_min)) {
      const float* xp = xa + p0 + q;
#pragma unroll
      for (int n1 = 0; n1 < 20; ++n1) raw[n1] = xp[20 * n1];
    } else {
#pragma unroll
      for (int n1 = 0; n1 < 20; ++n1) {
        int p = p0 + 20 * n1 + q;
        p = p < 0 ? -p : p;
        p = p > n_pad - 1 ? 2 * (n_pad - 1) - p : p;
        const bool in = p < n_valid;
        const float x = xa[in ? p : 0];
        raw[n1] = in ? x : 0.0f;
      }
    }
  };
  // The pass to load next: its first row (utterance lb, frame lt; wave-
  // uniform) advances by 6 per pass.  Frame a of the lane group's pair is row
  // 2 g after it, frame b the next row (t + 1, or frame 0 of the next utterance).
  int64_t lrow = p_beg * kRowsPerPass;
  int lb = (int)((unsigned)(lrow < rows ? lrow : 0) / (unsigned)T);   // rows < 2^31 (host check)
  int lt = (int)(lrow < rows ? lrow : 0) - lb * T;
  auto load_pair = [&](bool pass_live, float (&ra_)[20], float (&rb_)[20]) {
    const int64_t row = lrow + 2 * g;
    const bool live_a = g < kF2Pairs && pass_live && row < rows;
    const bool live_b = live_a && row + 1 < rows;
    int ba = lb, ta = lt + 2 * g;
    while (ta >= T) {   // (once at most for T >= 5)
      ta -= T;
      ++ba;
    }
    const bool wrap = ta + 1 == T;
    load_one(live_a, ba, ta, ra_);
    load_one(live_b, wrap ? ba + 1 : ba, wrap ? 0 : ta + 1, rb_);
    lrow += kRowsPerPass;
    lt += kRowsPerPass;
    while (lt >= T) {
      lt -= T;
      ++lb;
    }
  };
  // the lane's mel windows: mel `lane` (kMelW1 taps from bin ws1) and half
  // `lane & 1` of mel 64 + lane / 2 (kMelW2 taps from ws2; lanes >= 32: zero weights)
  float mw1[kMelW1], mw2[kMelW2];
#pragma unroll
  for (int j = 0; j < kMelW1; ++j) mw1[j] = melw[lane * kMelW1 + j];
#pragma unroll
  for (int j = 0; j < kMelW2; ++j) mw2[j] = melw[64 * kMelW1 + lane * kMelW2 + j];
  const int ws1 = melws[lane], ws2 = melws[64 + lane];
  float ra[20], rb[20];
  int ta_cur = lt;   // frame index of the current pass's first row in its utterance
  load_pair(p_beg < p_end, ra, rb);
  const bool lact = g < kF2Pairs;
  // STATS: the lane's running sums for the current utterance ({x, y}: its two
  // filters), and the slot of the next one to flush
  f2 s_run = {0.0f, 0.0f}, q_run = {0.0f, 0.0f};
  int seg = 0;
  auto flush = [&]() {   // (wave-uniform) reduce the running sums over the wave into the next slot
    float t0 = sum_rows4(row16_sum(s_run.x + s_run.y));
    float t1 = sum_rows4(row16_sum(q_run.x + q_run.y));
    if (lane == 0) part[wid * MS + seg] = make_float2(t0, t1);
    ++seg;
    s_run = f2{0.0f, 0.0f};
    q_run = f2{0.0f, 0.0f};
  };
  for (int64_t ps = p_beg; ps < p_end; ++ps) {
    const int ta_pass = ta_cur;
    ta_cur = lt;   // (the next pass's, before load_pair advances it)
    // stage 1: lane (g, n2 = q): DFT-20 over n1 of z[20 n1 + n2] = w (x_a + i x_b)
    f2 v[20];
    {
      // All twenty window reads first (one LDS wait), then the products; the
      // memory clobber after them keeps the next pass's loads behind the
      // products.  (A clobber per product had serialised the window reads:
      // twenty LDS round trips per pass, each waited for.)
      float wn[20];
#pragma unroll
      for (int n1 = 0; n1 < 20; ++n1) wn[n1] = L.win[20 * n1 + q];
#pragma unroll
      for (int n1 = 0; n1 < 20; ++n1) {
        v[n1] = f2{ra[n1], rb[n1]} * f2{wn[n1], wn[n1]};
        asm volatile("" ::"v"(v[n1].x), "v"(v[n1].y));
      }
      asm volatile("" ::: "memory");   // ahead of the next pass's loads
    }
    load_pair(ps + 1 < p_end, ra, rb);
    dft20(v);
    // A rows: lane (g, q) writes A[g][q][0..19]; pitch 25 float2 = 50 dwords:
    // 50 i mod 64 over 32 lanes is 2 x (25 i mod 32), all distinct
    if (lact) {
#pragma unroll
      for (int k1 = 0; k1 < 20; ++k1) LM_W(A, (g * 20 + q) * kA2Pitch + k1, v[k1]);
    }
    wave_lds_sync();
    // stage 2: lane (g, k1 = q) gathers column k1: lane groups g start at
    // 40 g x 25 = 40 g mod 64 dwords, so half-waves touch disjoint banks
    // (software-pipelined in chunks of four: the reads of chunk c + 1 issue
    // before chunk c's twiddle products, so only the first chunk's reads are
    // waited for in full)
    if (lact) {
      constexpr int CK = 4;
      f2 ab[2][CK], tb[2][CK];
      auto ldc = [&](int c, int b) {
#pragma unroll
        for (int k = 0; k < CK; ++k) {
          ab[b][k] = LM_R(A, (g * 20 + CK * c + k) * kA2Pitch + q);
          tb[b][k] = L.tw[q][CK * c + k];
        }
      };
      ldc(0, 0);
#pragma unroll
      for (int c = 0; c < 20 / CK; ++c) {
        if (c + 1 < 20 / CK) ldc(c + 1, (c + 1) & 1);
#pragma unroll
        for (int k = 0; k < CK; ++k) v[CK * c + k] = cmul2(ab[c & 1][k], tb[c & 1][k]);
      }
    }
    dft20(v);   // Z[q + 20 k2] in v[k2]
    // exchange (the A reads of this wave are done: one wave's LDS ops complete in order)
    f2* E = A;
    if (lact) {
      f2* e = E + (g * 20 + q) * kE2Pitch;
#pragma unroll
      for (int j = 0; j < 10; ++j) LM_W(e, j, v[10 + j]);
      if (q == 0) e[10] = v[0];
    }
    wave_lds_sync();
    // partner values pp[k2] = Z[400 - q - 20 k2]: lane 20 - q's v[19 - k2]
    // (= its published slot 9 - k2), or for q = 0 the lane's own v[20 - k2]
    // (slots shifted by one, slot 10 = v[0])
    f2 pp[10];
    {
      const f2* base = E + (g * 20 + (q == 0 ? 0 : 20 - q)) * kE2Pitch + (q == 0 ? 1 : 0);
#pragma unroll
      for (int k2 = 0; k2 < 10; ++k2) pp[k2] = LM_R(base, 9 - k2);
    }
    wave_lds_sync();
    // pair powers {|Z + conj Z'|^2, |Z - conj Z'|^2} = 4 {P_a, P_b}; row pitch
    // 212 float2: lane groups 40 banks apart, conflict-free 8-byte writes
    f2* PW = A;
    if (lact) {
      f2* pr = PW + g * kP2Pitch + q;
#pragma unroll
      for (int k2 = 0; k2 < 10; ++k2) {
        const f2 sa = f2{v[k2].x + pp[k2].x, v[k2].y - pp[k2].y};   // Z + conj Z'
        const f2 sb = f2{v[k2].x - pp[k2].x, v[k2].y + pp[k2].y};   // Z - conj Z'
        LM_W(pr, 20 * k2, (f2{__builtin_fmaf(sa.x, sa.x, sa.y * sa.y), __builtin_fmaf(sb.x, sb.x, sb.y * sb.y)}));
      }
      if (q == 0) {   // bin 200 is its own partner: 4 {Re^2, Im^2}
        const f2 z = v[10];
        pr[200] = f2{4.0f * z.x * z.x, 4.0f * z.y * z.y};
      }
    }
    wave_lds_sync();
    // pair powers -> HTK mel -> ln(+1e-8), straight-line: lane l takes mel l
    // over a fixed window of kMelW1 bins, and lanes 0-31 the halves of mel
    // 64 + l / 2 over kMelW2 bins each (summed by a DPP swap); weights (x 1/4,
    // zero outside the filter) and window starts are per-lane registers, so a
    // tap is three 8-byte power reads (one per pair, immediate offsets) and
    // three packed FMAs, with no per-lane trip count
    {
      const f2* p1 = PW + ws1;
      const f2* p2 = PW + ws2;
      f2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f}, a2 = {0.0f, 0.0f};
      f2 c0 = {0.0f, 0.0f}, c1 = {0.0f, 0.0f}, c2 = {0.0f, 0.0f};
      typedef const volatile __attribute__((address_space(3))) f2 vf2;
#define LM_RD(p, i) (*(vf2*)((p) + (i)))
      // Software-pipelined one tap ahead: the volatile reads issue in source
      // order, so tap j + 1's six reads are written before tap j's FMAs (in two
      // separate loops the second set's reads had been issued one at a time,
      // each waited for: ~21 serial LDS round trips per pass).
      f2 x1[2][3], x2[2][3];
      auto ld = [&](int j, int b) {
        if (j < kMelW1) {
          x1[b][0] = LM_RD(p1, j);
          x1[b][1] = LM_RD(p1, kP2Pitch + j);
          x1[b][2] = LM_RD(p1, 2 * kP2Pitch + j);
        }
        if (j < kMelW2) {
          x2[b][0] = LM_RD(p2, j);
          x2[b][1] = LM_RD(p2, kP2Pitch + j);
          x2[b][2] = LM_RD(p2, 2 * kP2Pitch + j);
        }
      };
      static_assert(kMelW1 >= kMelW2, "the first window is the longer one");
      ld(0, 0);
#pragma unroll
      for (int j = 0; j < kMelW1; ++j) {
        if (j + 1 < kMelW1) ld(j + 1, (j + 1) & 1);
        const int b = j & 1;
        a0 = fma2(x1[b][0], f2{mw1[j], mw1[j]}, a0);
        a1 = fma2(x1[b][1], f2{mw1[j], mw1[j]}, a1);
        a2 = fma2(x1[b][2], f2{mw1[j], mw1[j]}, a2);
        if (j < kMelW2) {
          c0 = fma2(x2[b][0], f2{mw2[j], mw2[j]}, c0);
          c1 = fma2(x2[b][1], f2{mw2[j], mw2[j]}, c1);
          c2 = fma2(x2[b][2], f2{mw2[j], mw2[j]}, c2);
        }
      }
#undef LM_RD
      float cv[6] = {c0.x, c0.y, c1.x, c1.y, c2.x, c2.y};
#pragma unroll
      for (int f = 0; f < 6; ++f)   // + the other half (lane ^ 1)
        cv[f] += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, cv[f]), 0xB1, 0xF, 0xF, false));
      // stores through a resource over the pass's rows: rows past the end
      // fall outside num_records, and lanes 1, 3, ... of the second set (odd
      // halves) and 32-63 aim past it too -- no branch per frame
      const int64_t r0 = ps * kRowsPerPass;
      const int64_t nr = rows - r0 < kRowsPerPass ? rows - r0 : kRowsPerPass;
      const __amdgpu_buffer_rsrc_t fr = make_rsrc(feats + r0 * kMels, (uint32_t)(nr > 0 ? nr : 0) * kMels * 4);
      const float av[6] = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y};
      const bool half0 = lane < 2 * (kMels - 64) && (lane & 1) == 0;
      const int o2 = half0 ? 4 * (64 + (lane >> 1)) : 0x40000000;
      float la[6], lc[6];
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        la[f] = wk_logf(av[f] + 1e-8f);
        lc[f] = wk_logf(cv[f] + 1e-8f);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, la[f]), fr, 4 * (f * kMels + lane), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, lc[f]), fr, o2 + 4 * f * kMels, 0, 0);
      }
      if constexpr (STATS) {
        // rows r0 .. r0 + nr - 1; those from bnd on belong to the next utterance
        const int bnd = T - ta_pass;
        const float m2 = half0 ? 1.0f : 0.0f;   // the second filter set counts once per mel (even lanes 0-30)
        const float kLogFloor = wk_logf(1e-8f);   // bit-identical to a silent bin's value
        // per frame P = {x - K, (y - K) m2} for the lane's two filters
        const f2 pm = {1.0f, m2}, pk = {-kLogFloor, -kLogFloor * m2};
        if (ta_pass == 0 && ps != p_beg) flush();   // the previous pass ended an utterance
        if (bnd >= 6 && nr == 6) {   // the common pass: one utterance, all rows live
#pragma unroll
          for (int f = 0; f < 6; ++f) {
            const f2 P = fma2(f2{la[f], lc[f]}, pm, pk);
            s_run = s_run + P;
            q_run = fma2(P, P, q_run);
          }
        } else {
#pragma unroll
          for (int f = 0; f < 6; ++f) {
            if (f == bnd && f < nr) flush();   // (wave-uniform) the utterance ends inside this pass
            const f2 P = fma2(f2{la[f], lc[f]}, pm, pk);
            if (f < nr) {   // wave-uniform
              s_run = s_run + P;
              q_run = fma2(P, P, q_run);
            }
          }
        }
        if (ps + 1 == p_end) flush();   // the range's last utterance
      }
    }
    wave_lds_sync();
  }
}

// Sum over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (a row's four 16-lane
// groups), in every lane: gfx950's v_permlane16/32_swap exchange rows in the
// VALU (with both operands the same register, the two results are the
// lane's and its partner's values), no LDS round trip as __shfl_xor costs.
__device__ __forceinline__ float sum_rows4(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// Global z-score of one utterance per block (ctc.py:101-104: mean, unbiased
// std, applied only when std > 0).  Up to kZsCache float4 per thread stay in
// registers between the two reductions and the write-back, so the utterance
// is read from HBM once (it was read three times: 0.27 ms per 4096
// utterances); longer utterances (> 32,768 values, T > 409) re-read.
// The sums are double: a constant utterance (digital silence: every value
// ln(1e-8)) then has mean = its value and std = 0 exactly, and stays
// un-normalised.  (torch's float std of a constant tensor is rounding noise
// -- 1.9e-6 for 301 x 80 values of ln(1e-8) -- so ctc.py's `std() > 0` passes
// and its output is that noise's quotient; the build takes the exact reading,
// as ctc_zstats_kernel does on the one-call path.)
constexpr int kZsCache = 8;
__global__ __launch_bounds__(1024) void ctc_zscore_kernel(float* __restrict__ feats, int64_t n_per) {
  __shared__ double red[16];
  __shared__ double bc;
  float* f = feats + (int64_t)blockIdx.x * n_per;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto block_sum = [&](double v) -> double {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[w] = v;
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
      for (int i = 0; i < 16; ++i) s += red[i];
      bc = s;
    }
    __syncthreads();
    const double r = bc;
    __syncthreads();
    return r;
  };
  const int64_t n4 = n_per / 4;
  if (n_per % 4 == 0 && n4 <= 1024 * kZsCache && ((uintptr_t)f & 15) == 0) {
    float4* f4 = reinterpret_cast<float4*>(f);
    float4 v[kZsCache];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kZsCache; ++k) {
      const int64_t i = tid + 1024 * k;
      v[k] = i < n4 ? f4[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      s += ((double)v[k].x + (double)v[k].y) + ((double)v[k].z + (double)v[k].w);
    }
    const double mean = block_sum(s) / (double)n_per;
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < kZsCache; ++k) {
      if (tid + 1024 * k < n4) {
        const double a = v[k].x - mean, b = v[k].y - mean, c = v[k].z - mean, d = v[k].w - mean;
        q += (a * a + b * b) + (c * c + d * d);
      }
    }
    const double sd = sqrt(block_sum(q) / (double)(n_per - 1));
    if (!(sd > 0.0)) return;   // ctc.py:101-104: only when std > 0
    const float mf = (float)mean, inv = (float)(1.0 / sd);
#pragma unroll
    for (int k = 0; k < kZsCache; ++k) {
      const int64_t i = tid + 1024 * k;
      if (i < n4) f4[i] = make_float4((v[k].x - mf) * inv, (v[k].y - mf) * inv, (v[k].z - mf) * inv, (v[k].w - mf) * inv);
    }
    return;
  }
  double s = 0.0;
  for (int64_t i = tid; i < n_per; i += 1024) s += (double)f[i];
  const double mean = block_sum(s) / (double)n_per;
  double q = 0.0;
  for (int64_t i = tid; i < n_per; i += 1024) {
    const double d = (double)f[i] - mean;
    q += d * d;
  }
  const double sd = sqrt(block_sum(q) / (double)(n_per - 1));
  if (!(sd > 0.0)) return;
  const float mf = (float)mean, inv = (float)(1.0 / sd);
  for (int64_t i = tid; i < n_per; i += 1024) f[i] = (f[i] - mf) * inv;
}

// The z-score's statistics for wk_ctc_transcribe: one wave per utterance
// folds the log-mel waves' {S, Q} slots for it (ctc_logmel_fft2_kernel<true>:
// wave w's range of R passes starts in utterance 6 w R / T, its j-th slot is
// that utterance + j) in double into zs[b] = {mean, 1/std} (unbiased std,
// ctc.py:101-104), or {0, 1} when std is 0 (no normalisation).  Needs T >= 6:
// a pass then spans at most two utterances.  The partials are float sums, so
// Q - S m carries ~1e-6 of
// Q's size in rounding: a variance at or below 1e-5 of the mean square (a
// constant utterance, silent or not, lands there) is recomputed exactly from
// the utterance's raw rows, two passes in double -- a constant utterance then
// gets std 0 exactly and stays un-normalised, as ctc.py:104's `std() > 0` test
// leaves it.
__global__ __launch_bounds__(256) void ctc_zstats_kernel(const float2* __restrict__ part, const float* __restrict__ feats,
                                                         int64_t batch, int T, int64_t R, int MS,
                                                         float2* __restrict__ zs) {
  // one wave per utterance: lane i takes the waves w0 + i, + 64, ... whose ranges hold its rows
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= batch) return;   // (wave-uniform)
  const int64_t r0 = b * T, w0 = r0 / 6 / R, w1 = (r0 + T - 1) / 6 / R;
  double S = 0.0, Q = 0.0;
  for (int64_t w = w0 + lane; w <= w1; w += 64) {
    const int64_t first = w * R * 6 / T;   // the utterance of the range's first row
    const float2 v = part[w * MS + (b - first)];
    S += v.x;
    Q += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    S += __shfl_xor(S, o, 64);
    Q += __shfl_xor(Q, o, 64);
  }
  const double n = (double)T * kMels;
  double m = S / n, var = (Q - S * m) / (n - 1.0);
  m += (double)wk_logf(1e-8f);   // S, Q are sums of x - ln(1e-8)
  // (Q == 0: every value is the floor ln(1e-8), digital silence: std 0 as it stands)
  if (Q > 0.0 && var <= 1e-5 * (Q / n)) {   // (wave-uniform) within the partials' rounding: exact two-pass statistics
    const float* f = feats + r0 * kMels;
    const int64_t cnt = (int64_t)T * kMels;
    double s1 = 0.0;
    for (int64_t i = lane; i < cnt; i += 64) s1 += (double)f[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s1 += __shfl_xor(s1, o, 64);
    m = s1 / n;
    double s2 = 0.0;
    for (int64_t i = lane; i < cnt; i += 64) {
      const double d = (double)f[i] - m;
      s2 += d * d;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    var = s2 / (n - 1.0);
  }
  const float sd = var > 0.0 ? (float)sqrt(var) : 0.0f;
  if (lane == 0) zs[b] = sd > 0.0f ? make_float2((float)m, 1.0f / sd) : make_float2(0.0f, 1.0f);
}

// ---------------------------------------------------------------------------
// X2a: encoder Linear(80,128) + LayerNorm(128) + ReLU, one wave per row
// ---------------------------------------------------------------------------
// OT = float, or __half in fp16 mode (the next GEMM's operand, written directly).
__device__ __forceinline__ void st_out(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_out(__half* p, float v) { *p = __float2half(v); }

// Linear 80 -> 128 on the matrix cores: a wave takes 16 rows at a time, D =
// x[16 rows][80] . W^T as 8 column tiles x 20 K-steps of v_mfma_f32_16x16x4f32
// (B fragments from an LDS copy of W laid out [k-step][tile][lane], so each
// read is one conflict-free ds_read_b32).  The lane then holds rows 4 (l>>4) + i
// of column 16 ct + (l & 15): LayerNorm's row sums are 8 in-register adds and
// a 16-lane shuffle reduction.  (Was one wave per row on the VALU: 1.19 ms per
// 4096 utterances.)
template <typename OT>
__global__ __launch_bounds__(256) void ctc_encoder_kernel(const float* __restrict__ in, int64_t rows,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, OT* __restrict__ out) {
  constexpr int KS = kMels / 4, CT = kH / 16;           // 20 K-steps, 8 column tiles
  __shared__ float wf[KS][CT][64];                      // B[k = 4 s + (l>>4)][col = 16 ct + (l&15)] = W[col][k]
  __shared__ float pb[3][kH];                           // bias, gamma, beta
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < KS * CT * 64; i += 256) {
    const int st = i / (CT * 64), ct = (i / 64) % CT, l = i & 63;
    wf[st][ct][l] = w[(16 * ct + (l & 15)) * kMels + 4 * st + (l >> 4)];
  }
  for (int i = tid; i < kH; i += 256) {
    pb[0][i] = bias[i];
    pb[1][i] = gamma[i];
    pb[2][i] = beta[i];
  }
  __syncthreads();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t nblk = (rows + 15) / 16;
  for (int64_t blk = (int64_t)blockIdx.x * 4 + wv; blk < nblk; blk += (int64_t)gridDim.x * 4) {
    const int64_t r0 = blk * 16;
    const int64_t ra = r0 + li;                          // this lane's A row
    float xa[KS];
#pragma unroll
    for (int st = 0; st < KS; ++st) xa[st] = ra < rows ? in[ra * kMels + 4 * st + lg] : 0.0f;
    f32x4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[ct] = mfma4(xa[st], wf[st][ct][lane], acc[ct]);
    float mean[4], rs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s1 = 0.0f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        acc[ct][i] += pb[0][16 * ct + li];
        s1 += acc[ct][i];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s1 += __shfl_xor(s1, o, 64);
      mean[i] = s1 * (1.0f / kH);
      float s2 = 0.0f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const float d = acc[ct][i] - mean[i];
        s2 = __builtin_fmaf(d, d, s2);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s2 += __shfl_xor(s2, o, 64);
      rs[i] = 1.0f / sqrtf(s2 * (1.0f / kH) + 1e-5f);   // biased variance, as nn.LayerNorm
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = r0 + 4 * lg + i;
      if (r < rows) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int col = 16 * ct + li;
          st_out(out + r * kH + col,
                 fmaxf(__builtin_fmaf((acc[ct][i] - mean[i]) * rs[i], pb[1][col], pb[2][col]), 0.0f));
        }
      }
    }
  }
}

// fp16 mode (precision 1, "fp16 GEMM operands"): the same Linear 80 -> 128 +
// LayerNorm + ReLU on v_mfma_f32_16x16x32_f16 -- K = 80 in 3 steps (the last
// half zero), 24 MFMAs of 16 cycles per 16 rows instead of 160 fp32 MFMAs of 32
// (the fp32 kernel above ran at ~1/5 of the HBM rate).  W is the A operand and
// the rows the B operand, so a lane ends with 4 consecutive output columns of
// one row per column tile: LayerNorm's sums are in-lane plus two shuffles, and
// each tile leaves as one 8-byte store.  W fragments come from LDS per block
// (24 KB; keeping them in VGPRs would cost 96 registers and the occupancy).
typedef _Float16 h8e __attribute__((ext_vector_type(8)));
// Output rows are time-major (row t B + b for input row b T + t): the fp16
// path keeps every [rows][.] tensor after the encoder in that order, so that a
// GRU step's 16 utterances are 16 adjacent rows of the gate inputs and outputs.
// NORM (wk_ctc_transcribe): the input rows are raw log-mel; each is z-scored
// with its utterance's zs = {mean, 1/std} (ctc_zstats_kernel) as it is loaded.
template <bool NORM>
__global__ __launch_bounds__(256) void ctc_encoder16_kernel(const float* __restrict__ in, int64_t rows,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int B, int T,
                                                            const float2* __restrict__ zs, __half* __restrict__ out) {
  constexpr int KS = 3, CT = kH / 16;
  __shared__ __attribute__((aligned(16))) h8e wf[KS][CT][64];   // A[col 16 ct + (l&15)][k = 32 s + 8 (l>>4) + j]
  __shared__ __attribute__((aligned(16))) float pb[3][kH];      // bias, gamma, beta
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < KS * CT * 64; i += 256) {
    const int st = i / (CT * 64), ct = (i / 64) % CT, l = i & 63;
    h8e v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * st + 8 * (l >> 4) + j;
      v[j] = (_Float16)(k < kMels ? w[(16 * ct + (l & 15)) * kMels + k] : 0.0f);
    }
    wf[st][ct][l] = v;
  }
  for (int i = tid; i < kH; i += 256) {
    pb[0][i] = bias[i];
    pb[1][i] = gamma[i];
    pb[2][i] = beta[i];
  }
  __syncthreads();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t nblk = (rows + 15) / 16;
  // Loads and stores go through buffer resources (rows past the end read 0 /
  // drop), so the loop has no branch: the next block's rows are loaded before
  // this block's compute and stores, and the compiler's vmcnt waits for those
  // loads only, not for the stores behind them (with guarded accesses it
  // waited for everything: ~60 % of wave-cycles were waits, PMC).
  const __amdgpu_buffer_rsrc_t irs = make_rsrc(in, (uint32_t)(rows * kMels * 4));   // < 2^31 B (host check)
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(out, (uint32_t)(rows * kH * 2));
  // 1 blocks of input rows in flight per wave (a block's compute is
  // far shorter than the HBM latency)
  float4 xr[1][KS][2];
  auto load_blk = [&](int64_t blk, float4 (&x)[KS][2]) __attribute__((always_inline)) {
    const int64_t r = blk * 16 + li;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int k0 = 32 * st + 8 * lg;
      const int off = r < rows && k0 < kMels ? (int)(r * kMels + k0) * 4 : 0x7FFFFFE0;   // past num_records: 0
      x[st][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(irs, off, 0, 0));
      x[st][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(irs, off + 16, 0, 0));
    }
  };
  const int64_t G = (int64_t)gridDim.x * 4;
  auto body = [&](int64_t blk, float4 (&x)[KS][2]) __attribute__((always_inline)) {
    const int64_t r = blk * 16 + li;   // this lane's row
    const int rr = r < rows ? (int)r : 0;   // rows < 2^31 (host check)
    const int ub = rr / T, ut = rr - ub * T;
    h8e xb[KS];
    if constexpr (NORM) {
      const float2 z = zs[ub];
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const float4 a = x[st][0], b = x[st][1];
        xb[st] = h8e{(_Float16)((a.x - z.x) * z.y), (_Float16)((a.y - z.x) * z.y), (_Float16)((a.z - z.x) * z.y),
                     (_Float16)((a.w - z.x) * z.y), (_Float16)((b.x - z.x) * z.y), (_Float16)((b.y - z.x) * z.y),
                     (_Float16)((b.z - z.x) * z.y), (_Float16)((b.w - z.x) * z.y)};
      }
    } else {
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const float4 a = x[st][0], b = x[st][1];
        xb[st] = h8e{(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
                     (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
      }
    }
    load_blk(blk + 1 * G, x);   // the block 1 ahead into this slot (past the end: zeros, unused)
    f32x4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = *reinterpret_cast<const f32x4*>(&pb[0][16 * ct + 4 * lg]);   // + bias
    int wl = lane;
    asm volatile("" : "+v"(wl));   // W fragments re-read per block, not hoisted into 96 VGPRs
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[st][ct][wl], xb[st], acc[ct], 0, 0, 0);
    // acc[ct][i] = row r, column 16 ct + 4 lg + i; the row's 128 columns are in lanes li + 16 q
    float s1 = 0.0f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) s1 += (acc[ct][0] + acc[ct][1]) + (acc[ct][2] + acc[ct][3]);
    s1 = sum_rows4(s1);
    const float mean = s1 * (1.0f / kH);
    float s2 = 0.0f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = acc[ct][i] - mean;
        s2 = __builtin_fmaf(d, d, s2);
      }
    s2 = sum_rows4(s2);
    const float rs = 1.0f / sqrtf(s2 * (1.0f / kH) + 1e-5f);   // biased variance, as nn.LayerNorm
    const int orow = r < rows ? (ut * B + ub) * (kH * 2) : 0x7FFFFE00;   // time-major output row (bytes); past the end: dropped
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int c0 = 16 * ct + 4 * lg;
      const f32x4 g = *reinterpret_cast<const f32x4*>(&pb[1][c0]);
      const f32x4 bt = *reinterpret_cast<const f32x4*>(&pb[2][c0]);
      _Float16 y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = (_Float16)fmaxf(__builtin_fmaf((acc[ct][i] - mean) * rs, g[i], bt[i]), 0.0f);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, y), ors,
                                            orow + c0 * 2, 0, 0);
    }
  };
  int64_t blk = (int64_t)blockIdx.x * 4 + wv;
#pragma unroll
  for (int u = 0; u < 1; ++u) load_blk(blk + u * G, xr[u]);
  for (; blk < nblk; blk += 1 * G) {
#pragma unroll
    for (int u = 0; u < 1; ++u) {
      if (blk + u * G >= nblk) break;   // (wave-uniform)
      body(blk + u * G, xr[u]);
    }
  }
}

// ---------------------------------------------------------------------------
// X2b: GRU recurrence (one layer, both directions)
//   r = s(Wir x + bir + Whr h + bhr), z = s(Wiz x + biz + Whz h + bhz),
//   n = tanh(Win x + bin + r (Whn h + bhn)), h' = (1 - z) n + z h
// gi = x W_ih^T for both directions comes precomputed: [B][T][768] (dir*384 + gate*128 + u).
// ---------------------------------------------------------------------------
constexpr int kGruBatch = 16, kGruWaves = 12, kGruThreads = 64 * kGruWaves;
constexpr int kHP = 17;   // LDS pitch of [unit][batch] images (conflict-free for consecutive units)

// Gate activations on the transcendental unit: v_exp_f32 + v_rcp_f32 (~1 ulp
// each) instead of an IEEE division and libm tanhf -- the gate math, not the
// MFMAs, bounded a recurrence step.  tanh(x) = 1 - 2 / (e^2x + 1): exact limits
// at +-inf, absolute error ~1e-7 near 0.
__device__ __forceinline__ float sigm(float v) { return __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }
__device__ __forceinline__ float tanh_fast(float v) { return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(__expf(2.0f * v) + 1.0f), 1.0f); }

__global__ __launch_bounds__(kGruThreads) void ctc_gru_kernel(const float* __restrict__ gi, const float* __restrict__ whh_pk,
                                                              const float* __restrict__ bih, const float* __restrict__ bhh,
                                                              int64_t B, int T, float* __restrict__ out) {
  __shared__ float hs[2][kH * kHP];
  __shared__ float gh[3 * kH * kHP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dir = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * kGruBatch;
  // W_hh fragments: this wave's tiles 2w, 2w+1 (rows 16 tile .. +15), k-step s covers k = 4s..4s+3.
  float wa[32], wb[32];
  {
    const float* p = whh_pk + ((size_t)dir * 24 + 2 * wave) * 32 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      wa[s] = p[s * 64];
      wb[s] = p[(32 + s) * 64];
    }
  }
  for (int i = tid; i < kH * kHP; i += kGruThreads) hs[0][i] = 0.0f;   // h0 = 0
  __syncthreads();
  const float* bi = bih + dir * 3 * kH;
  const float* bh = bhh + dir * 3 * kH;
  int cur = 0;
  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    // gh = W_hh h  (MFMA: A = W rows, B = h[k][n], D rows = gate rows, cols = batch)
    {
      f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
      const float* hb = hs[cur] + (lane >> 4) * kHP + (lane & 15);
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const float hv = hb[4 * s * kHP];
        acc_a = mfma4(wa[s], hv, acc_a);
        acc_b = mfma4(wb[s], hv, acc_b);
      }
      const int ra = 32 * wave + 4 * (lane >> 4), col = lane & 15;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gh[(ra + r) * kHP + col] = acc_a[r];
        gh[(ra + 16 + r) * kHP + col] = acc_b[r];
      }
    }
    __syncthreads();
    // gates: element e -> (batch n = e / 128, unit u = e % 128): coalesced gi / out rows
    for (int e = tid; e < kGruBatch * kH; e += kGruThreads) {
      const int n = e >> 7, u = e & (kH - 1);
      const int64_t b = b0 + n;
      float hn = 0.0f;
      if (b < B) {
        const float* g = gi + ((size_t)b * T + t) * (6 * kH) + dir * 3 * kH;
        const float r = sigm(g[u] + bi[u] + gh[u * kHP + n] + bh[u]);
        const float z = sigm(g[kH + u] + bi[kH + u] + gh[(kH + u) * kHP + n] + bh[kH + u]);
        const float c = tanh_fast(g[2 * kH + u] + bi[2 * kH + u] + r * (gh[(2 * kH + u) * kHP + n] + bh[2 * kH + u]));
        const float hp = hs[cur][u * kHP + n];
        hn = __builtin_fmaf(z, hp - c, c);   // (1 - z) c + z h
        out[((size_t)b * T + t) * (2 * kH) + dir * kH + u] = hn;
      }
      hs[cur ^ 1][u * kHP + n] = hn;
    }
    cur ^= 1;
    __syncthreads();
  }
}

// fp16-operand variant (precision 1, config 5): W_hh and h enter
// v_mfma_f32_16x16x16_f16 as fp16, gate pre-activations accumulate in fp32,
// gates and the state update stay fp32.  A fragment of tile tl, k-step s:
// lane l holds W[16 tl + (l & 15)][16 s + 4 (l >> 4) + j], j = 0..3; the B
// fragment is h16[batch = l & 15][16 s + 4 (l >> 4) + j] from LDS (one b64 read).
//
// Wave w computes the r, z and n tiles of the same 16 units (tiles w, 8 + w,
// 16 + w), so a lane's three accumulators hold gh_r, gh_z, gh_n of units
// 16 w + 4 (l >> 4) + i (i = 0..3) for batch slot l & 15: the gates, the state
// update and the fp32 state itself stay in its registers.  A step is 24 MFMAs,
// the gate math for 4 elements, one 8-byte LDS write of the new fp16 state and
// one barrier per wave.  (The previous layout -- 32 consecutive gate rows per
// wave, gh and the fp32 state through LDS, 12 waves -- issued ~2.6x the
// instructions per step and needed two barriers.)
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
constexpr int kH16P = kH + 8;   // LDS pitch (halves) of the fp16 state image [batch][unit]: 16-byte rows, conflict-free B reads
constexpr int kGru16Waves = kH / 16, kGru16Threads = 64 * kGru16Waves;
constexpr int kGtP = 3 * kH + 8;   // LDS pitch (halves) of a gate-input tile row: 16-byte aligned
constexpr int kGruPf = 2;

__global__ __launch_bounds__(kGru16Threads, 4) void ctc_gru16_kernel(const __half* __restrict__ gi, const h4* __restrict__ whh_pk,
                                                                  const float* __restrict__ bih,
                                                                  const float* __restrict__ bhh, int64_t B, int T,
                                                                  __half* __restrict__ out) {   // fp16: the next GEMM's operand
  __shared__ __attribute__((aligned(16))) _Float16 h16[2][kGruBatch * kH16P];
  __shared__ __attribute__((aligned(16))) _Float16 gt[2][kGruBatch * kGtP];   // gate-input tiles
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dir = blockIdx.y;
  const int n = lane & 15;                    // batch slot
  const int u0 = 16 * wave + 4 * (lane >> 4); // the lane's units u0 .. u0 + 3
  const int64_t b = (int64_t)blockIdx.x * kGruBatch + n;
  const bool live = b < B;
  h4 wr[8], wz[8], wn[8];
  {
    const h4* p = whh_pk + (size_t)dir * 24 * 8 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      wr[s] = p[((0 * 8 + wave) * 8 + s) * 64];
      wz[s] = p[((1 * 8 + wave) * 8 + s) * 64];
      wn[s] = p[((2 * 8 + wave) * 8 + s) * 64];
    }
  }
  for (int i = tid; i < kGruBatch * kH16P; i += kGru16Threads) h16[0][i] = (_Float16)0.0f;
  const float* bi = bih + dir * 3 * kH;
  const float* bh = bhh + dir * 3 * kH;
  // Biases in LDS, [gate term][unit] (b_ir + b_hr, b_iz + b_hz, b_in, b_hn):
  // read per step as four 16-byte loads (in VGPRs they pushed the kernel over
  // the 128 registers of 4 waves per SIMD).
  __shared__ f32x4 gbias[4][kH / 4];
  if (tid < kH) {
    float* gbf = reinterpret_cast<float*>(&gbias[0][0]);
    gbf[tid] = bi[tid] + bh[tid];
    gbf[kH + tid] = bi[kH + tid] + bh[kH + tid];
    gbf[2 * kH + tid] = bi[2 * kH + tid];
    gbf[3 * kH + tid] = bh[2 * kH + tid];
  }
  float h[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // Gate inputs: a step's [16 rows][384] fp16 block of gi (this direction's
  // half of 16 adjacent time-major rows) is loaded cooperatively, 16 bytes per
  // thread and two chunks per thread (chunks past the 768 read out of range),
  // kGruPf steps ahead into a register ring, written to an LDS tile one step
  // ahead, and read back per lane (3 x 8 bytes).  The buffer resource is the
  // step's block itself: rows past B fall outside num_records and read 0, the
  // step index is clamped, so every load is unconditional and there is no
  // per-lane branch.  (Per-lane 8-byte loads from gi -- 32-byte pieces per
  // row and wave -- were the recurrence's largest cost.)
  const int64_t b0 = (int64_t)blockIdx.x * kGruBatch;
  const int nrow = (int)(B - b0 < kGruBatch ? B - b0 : kGruBatch);
  const int gc0 = tid, gc1 = tid + kGru16Threads;   // 16-byte chunks: row c / 48, column c % 48
  const int gvo0 = (gc0 / 48) * (12 * kH) + dir * (6 * kH) + (gc0 % 48) * 16;
  const int gvo1 = gc1 < 16 * 48 ? (gc1 / 48) * (12 * kH) + dir * (6 * kH) + (gc1 % 48) * 16 : 0x40000000;
  uint4 gv0[kGruPf], gv1[kGruPf];
  auto load_gates = [&](int slot, int step) {
    const int st = step < T ? step : T - 1;
    const int t = dir == 0 ? st : T - 1 - st;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(gi + ((int64_t)t * B + b0) * (6 * kH), (uint32_t)nrow * (12 * kH));
    gv0[slot] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, gvo0, 0, 0));
    gv1[slot] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, gvo1, 0, 0));
  };
  auto stage_gates = [&](int slot, int buf) {   // ring slot -> LDS tile
    *reinterpret_cast<uint4*>(&gt[buf][(gc0 / 48) * kGtP + (gc0 % 48) * 8]) = gv0[slot];
    if (gc1 < 16 * 48) *reinterpret_cast<uint4*>(&gt[buf][(gc1 / 48) * kGtP + (gc1 % 48) * 8]) = gv1[slot];
  };
  const int64_t dstep = dir == 0 ? B : -B;   // out is time-major (row t B + b)
  // Outputs: the new fp16 state of a step is already the [16 rows][128 units]
  // image h16[cur] after the step's barrier; in the next step threads 0-255
  // copy it out as one 16-byte load + store each (a row's 256 bytes by 16
  // lanes) instead of every lane storing 8 bytes (32-byte pieces per row).
  const int yn = (tid >> 4) & 15, yc = tid & 15;
  const bool ylive = tid < 256 && (int64_t)blockIdx.x * kGruBatch + yn < B;
  __half* yq = out + ((int64_t)(dir == 0 ? 0 : T - 1) * B + (ylive ? (int64_t)blockIdx.x * kGruBatch + yn : 0)) * (2 * kH) +
               dir * kH + 8 * yc;
  auto store_y = [&](int buf) {
    if (ylive) *reinterpret_cast<uint4*>(yq) = *reinterpret_cast<const uint4*>(&h16[buf][yn * kH16P + 8 * yc]);
    yq += dstep * (2 * kH);
  };
#pragma unroll
  for (int j = 0; j < kGruPf; ++j) load_gates(j, j);
  stage_gates(0, 0);
  load_gates(0, kGruPf);
  __syncthreads();
  int cur = 0;
  for (int step0 = 0; step0 < T; step0 += kGruPf) {
#pragma unroll
  for (int j = 0; j < kGruPf; ++j) {
    const int step = step0 + j;
    if (step >= T) break;
    f32x4 ar = {0, 0, 0, 0}, az = {0, 0, 0, 0}, an = {0, 0, 0, 0};
    {
      const _Float16* hb = h16[cur] + n * kH16P + 4 * (lane >> 4);
      h4 hv[8];   // all eight B fragments first: one LDS wait
#pragma unroll
      for (int s = 0; s < 8; ++s) hv[s] = *reinterpret_cast<const h4*>(hb + 16 * s);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        ar = __builtin_amdgcn_mfma_f32_16x16x16f16(wr[s], hv[s], ar, 0, 0, 0);
        az = __builtin_amdgcn_mfma_f32_16x16x16f16(wz[s], hv[s], az, 0, 0, 0);
        an = __builtin_amdgcn_mfma_f32_16x16x16f16(wn[s], hv[s], an, 0, 0, 0);
      }
    }
    if (step > 0) store_y(cur);   // the previous step's outputs
    const _Float16* gp = &gt[step & 1][n * kGtP + u0];
    const h4 gr = *reinterpret_cast<const h4*>(gp), gz = *reinterpret_cast<const h4*>(gp + kH),
             gc = *reinterpret_cast<const h4*>(gp + 2 * kH);
    // next step's gates into the other tile, then refill that ring slot
    stage_gates((j + 1) % kGruPf, (step + 1) & 1);
    load_gates((j + 1) % kGruPf, step + 1 + kGruPf);
    int bq = u0 >> 2;
    asm volatile("" : "+v"(bq));   // re-read per step, not hoisted into 16 VGPRs
    const f32x4 b_r = gbias[0][bq], b_z = gbias[1][bq], bi_c = gbias[2][bq], bh_c = gbias[3][bq];
    h4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float hn = 0.0f;
      if (live) {
        const float r = sigm((float)gr[i] + ar[i] + b_r[i]);
        const float z = sigm((float)gz[i] + az[i] + b_z[i]);
        const float c = tanh_fast((float)gc[i] + bi_c[i] + r * (an[i] + bh_c[i]));
        hn = __builtin_fmaf(z, h[i] - c, c);   // (1 - z) c + z h
      }
      h[i] = hn;
      o[i] = (_Float16)hn;
    }
    *reinterpret_cast<uint2*>(&h16[cur ^ 1][n * kH16P + u0]) = __builtin_bit_cast(uint2, o);
    cur ^= 1;
    __syncthreads();
  }
  }
  store_y(cur);   // the last step's outputs
}

// ---------------------------------------------------------------------------
// fp16 recurrence with the input projection fused in (precision 1, config 5):
// gi = x W_ih^T is computed inside the persistent recurrence from the layer's
// input rows x (time-major [T][B][DIN] fp16: the encoder output, or layer 0's
// [fwd | bwd] outputs), so neither a projection GEMM nor the [rows][768] gate
// inputs (1.9 GB written and read back per layer at config 5) exist.
//
// A workgroup owns 32 utterances (two 16-row tiles) of one direction, one
// workgroup per CU (8 waves, 2 per SIMD, up to 256 VGPRs each): wave w owns
// units 16 w .. 16 w + 15 of the r, z and n gates for both row tiles, as in
// ctc_gru16_kernel.  Its 48 rows of W_hh and W_ih are A fragments of
// v_mfma_f32_16x16x32_f16 (k-steps of 32): W_hh and W_ih k < 128 in VGPRs
// (2 x 48 registers), layer 1's W_ih k >= 128 in an LDS image in fragment
// order (96 KB per workgroup).
//
// Gate pre-activations arrive pre-scaled for the exp2 unit: the r and z rows
// of both weights and their biases carry -log2(e), the n rows (x-part and
// h-part, b_in and b_hn) 2 log2(e), so r = 1 / (1 + 2^a), z likewise, and
// tanh(v) = 1 - 2 / (2^v' + 1) take no scaling multiply.  Rows past B read 0
// as x and their state is never stored (each utterance's recurrence is its
// own), so the gate math runs on every lane unmasked.
//
// One step (one barrier), per wave:
//   memory: the previous step's outputs (16-byte pieces of the state image),
//     the x rows of step t + 2 into the LDS tile the previous step's x-part
//     read (from a 2-step register ring of 16-byte loads), the ring refilled;
//   h-part of step t, tile 0 (12 MFMAs onto the x-part accumulators of r and
//     z; n's h-part apart, b_hn as its initial accumulator);
//   h-part of tile 1 (12 MFMAs), interleaved with tile 0's gate math;
//   x-part of step t + 1 (2 tiles x 3 gates x DIN/32 MFMAs on the staged x
//     tile, biases as the initial accumulator), independent of the state,
//     interleaved with tile 1's gate math;
//   the new fp16 state into the other state image, barrier.
// The interleave is fixed at compile time by sched_group_barrier, so the
// matrix pipe and the gate VALU overlap inside each wave instead of taking
// turns (phase stamps of the unscheduled form: the gate + x-part phase took
// the sum of its MFMA and VALU times).
// ---------------------------------------------------------------------------
constexpr int kGxRows = 32;                       // utterances per workgroup
// Row pitch of the state image and the x tile: 144 halves = 18 16-byte slots
// (rows 2 slots apart mod 16).  A ds_read_b128 serves its lanes in the groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): with the B-fragment pattern
// (row n = lane & 15, slot 4 s + lane / 16) a pitch of 1 slot mod 16 (136
// halves) put two lanes of each group on one bank window (PMC: 47 % of the
// kernel's LDS cycles were conflicts, ~42 % each from these two reads), 2 mod
// 16 puts all 16 on distinct windows (MI355X_MICROARCH.md, LDS lane groups).
constexpr int kGxHP = kH + 16;
constexpr int kGxWaves = 8, kGxThreads = 64 * kGxWaves;
typedef _Float16 h8x __attribute__((ext_vector_type(8)));
constexpr float kNegLog2e = -1.4426950408889634f, kTwoLog2e = 2.8853900817779268f;
constexpr int kVpm0 = 2;   // VALU per MFMA beside tile 1's h-part (1 and 3 measured equal, 4: -2 %)

// One element of the GRU cell on pre-scaled pre-activations (see above):
// ar = -log2e (r pre-activation), az likewise, gn = 2 log2e (W_in x + b_in),
// an = 2 log2e (W_hn h + b_hn); returns h' = (1 - z) n + z h.
__device__ __forceinline__ float gru_cell(float ar, float az, float gn, float an, float h) {
  const float r = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(ar));
  const float z = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(az));
  const float c = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(__builtin_fmaf(r, an, gn)) + 1.0f), 1.0f);
  return __builtin_fmaf(z, h - c, c);
}

template <int DIN>
__global__ __launch_bounds__(kGxThreads, 1) void ctc_gru16x_kernel(const __half* __restrict__ x,
                                                                  const h8x* __restrict__ wih_pk,
                                                                  const h8x* __restrict__ whh_pk,
                                                                  const float* __restrict__ bih,
                                                                  const float* __restrict__ bhh, int64_t B, int T,
                                                                  __half* __restrict__ out) {
  constexpr int KX = DIN / 32;                 // x-part k-steps
  constexpr int KXR = KX < 4 ? KX : 4;         // of which in VGPRs (k < 128)
  constexpr int KXL = KX - KXR;                // in LDS (layer 1: k >= 128)
  constexpr int XP = DIN + 16;                 // x tile pitch (halves): see kGxHP
  constexpr int XCH = kGxRows * DIN / 8;       // 16-byte chunks per x tile
  constexpr int XPT = (XCH + kGxThreads - 1) / kGxThreads;   // per thread
  // VALU per MFMA beside the x-part: the rest of the ~2 x 54 gate instructions
  constexpr int VPM1 = (108 - 12 * kVpm0 + 6 * KX - 1) / (6 * KX) > 0 ? (108 - 12 * kVpm0 + 6 * KX - 1) / (6 * KX) : 1;
  __shared__ __attribute__((aligned(16))) _Float16 h16[2][kGxRows * kGxHP];
  __shared__ __attribute__((aligned(16))) _Float16 xt[2][kGxRows * XP];
  __shared__ __attribute__((aligned(16))) h8x wl[KXL > 0 ? 3 * kGxWaves * KXL * 64 : 1];
  __shared__ f32x4 gbias[4][kH / 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dir = blockIdx.y;
  const int n = lane & 15, lg = lane >> 4;
  const int u0 = 16 * wave + 4 * lg;
  const int64_t b0 = (int64_t)blockIdx.x * kGxRows;
  const int nrow = (int)(B - b0 < kGxRows ? B - b0 : kGxRows);
  // weights (pre-scaled on the host): W_hh and W_ih k < 128 in VGPRs, [dir][gate][wave][ks][lane]
  h8x wr[4], wz[4], wn[4];
  h8x xr[KXR], xz[KXR], xn[KXR];
  {
    const h8x* p = whh_pk + (size_t)dir * 3 * kGxWaves * 4 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      wr[s] = p[((0 * kGxWaves + wave) * 4 + s) * 64];
      wz[s] = p[((1 * kGxWaves + wave) * 4 + s) * 64];
      wn[s] = p[((2 * kGxWaves + wave) * 4 + s) * 64];
    }
    const h8x* q = wih_pk + (size_t)dir * 3 * kGxWaves * KX * 64 + lane;
#pragma unroll
    for (int s = 0; s < KXR; ++s) {
      xr[s] = q[((0 * kGxWaves + wave) * KX + s) * 64];
      xz[s] = q[((1 * kGxWaves + wave) * KX + s) * 64];
      xn[s] = q[((2 * kGxWaves + wave) * KX + s) * 64];
    }
    if constexpr (KXL > 0) {   // k >= 128 -> LDS, [gate][wave][ks - KXR][lane]
      for (int i = tid; i < 3 * kGxWaves * KXL * 64; i += kGxThreads) {
        const int l = i & 63, ks = (i >> 6) % KXL, gw = (i >> 6) / KXL;
        wl[i] = wih_pk[(size_t)dir * 3 * kGxWaves * KX * 64 + ((size_t)gw * KX + KXR + ks) * 64 + l];
      }
    }
  }
  for (int i = tid; i < kGxRows * kGxHP; i += kGxThreads) h16[0][i] = (_Float16)0.0f;
  if (tid < kH) {   // scaled biases: -log2e (b_ir + b_hr), -log2e (b_iz + b_hz), 2 log2e b_in, 2 log2e b_hn
    const float* bi = bih + dir * 3 * kH;
    const float* bh = bhh + dir * 3 * kH;
    float* gbf = reinterpret_cast<float*>(&gbias[0][0]);
    gbf[tid] = kNegLog2e * (bi[tid] + bh[tid]);
    gbf[kH + tid] = kNegLog2e * (bi[kH + tid] + bh[kH + tid]);
    gbf[2 * kH + tid] = kTwoLog2e * bi[2 * kH + tid];
    gbf[3 * kH + tid] = kTwoLog2e * bh[2 * kH + tid];
  }
  // x rows of a step: 32 adjacent time-major rows, XCH 16-byte chunks, a
  // register ring kXPf steps deep, then the LDS tile of that step's parity
  constexpr int kXPf = 2;
  uint4 xv[kXPf][XPT];
  auto load_x = [&](int slot, int step) {
    const int st = step < T ? step : T - 1;
    const int t = dir == 0 ? st : T - 1 - st;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(x + ((int64_t)t * B + b0) * DIN, (uint32_t)nrow * DIN * 2);
#pragma unroll
    for (int c = 0; c < XPT; ++c) {
      const int ch = tid + c * kGxThreads;
      xv[slot][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, ch < XCH ? 16 * ch : 0x40000000, 0, 0));
    }
  };
  static_assert(XCH % kGxThreads == 0, "x tile chunks divide over the threads (no guarded LDS write)");
  auto stage_x = [&](int slot, int buf) {
#pragma unroll
    for (int c = 0; c < XPT; ++c) {
      const int ch = tid + c * kGxThreads;
      *reinterpret_cast<uint4*>(&xt[buf][(ch / (DIN / 8)) * XP + (ch % (DIN / 8)) * 8]) = xv[slot][c];
    }
  };
  __syncthreads();   // gbias
  int bq = u0 >> 2;
  asm volatile("" : "+v"(bq));
  const f32x4 b_r = gbias[0][bq], b_z = gbias[1][bq], b_n = gbias[2][bq], b_hn = gbias[3][bq];
  // x-part of one step from the x tile `buf` into g[tile][gate] (bias as the initial accumulator)
  // The operands of k-step s + 1 (the two x-tile B fragments and, for layer
  // 1's k >= 128, the three W_ih A fragments from LDS) are read before k-step
  // s's MFMAs, so each step's reads have the previous step's MFMAs to land
  // behind (read one at a time, each had been waited for in full).
  auto xpart = [&](int buf, f32x4 (&g)[2][3]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      g[q][0] = b_r;
      g[q][1] = b_z;
      g[q][2] = b_n;
    }
    h8x xb[2][2], wa[2][3];
    auto ldx = [&](int s, int st) {
#pragma unroll
      for (int q = 0; q < 2; ++q) xb[st][q] = *reinterpret_cast<const h8x*>(&xt[buf][(16 * q + n) * XP + 32 * s + 8 * lg]);
      if (s >= KXR) {
        const int sl = s - KXR;
#pragma unroll
        for (int gt = 0; gt < 3; ++gt) wa[st][gt] = wl[((gt * kGxWaves + wave) * (KXL > 0 ? KXL : 1) + sl) * 64 + lane];
      }
    };
    ldx(0, 0);
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      if (s + 1 < KX) ldx(s + 1, (s + 1) & 1);
      const int st = s & 1;
      const h8x ar = s < KXR ? xr[s < KXR ? s : 0] : wa[st][0];
      const h8x az = s < KXR ? xz[s < KXR ? s : 0] : wa[st][1];
      const h8x an = s < KXR ? xn[s < KXR ? s : 0] : wa[st][2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        g[q][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ar, xb[st][q], g[q][0], 0, 0, 0);
        g[q][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(az, xb[st][q], g[q][1], 0, 0, 0);
        g[q][2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(an, xb[st][q], g[q][2], 0, 0, 0);
      }
    }
  };
  // Outputs (time-major rows t B + b, [fwd | bwd] halves): thread (row yn,
  // chunk yc) stores 16 bytes of the state image per step through a buffer
  // resource over the step's 32 rows, so rows past B fall outside num_records
  // and are dropped -- no branch in the loop, and the compiler's vmcnt for the
  // x-ring stays exact (a guarded store had made it wait for every store).
  const int yn = tid >> 4, yc = tid & 15;     // 512 threads = 32 rows x 16 chunks of the state image
  const int yoff = yn * (2 * kH * 2) + dir * (kH * 2) + 16 * yc;
  auto store_y = [&](int buf, int step_done, bool any) {   // the state after step step_done
    const int t = dir == 0 ? step_done : T - 1 - step_done;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(out + ((int64_t)t * B + b0) * (2 * kH), any ? (uint32_t)nrow * (2 * kH * 2) : 0u);
    const uint4 v = *reinterpret_cast<const uint4*>(&h16[buf][yn * kGxHP + 8 * yc]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rs, yoff, 0, 0);
  };
  // prologue: x_0 and x_1 staged, x_2 / x_3 in the ring, gx of step 0
  load_x(0, 0);
  load_x(1, 1);
  stage_x(0, 0);
  stage_x(1, 1);
  load_x(0, 2);
  load_x(1, 3);
  __syncthreads();
  f32x4 ga[2][3], gb[2][3];   // x-parts of the even / odd steps
  xpart(0, ga);
  __syncthreads();   // x_0's tile is rewritten (with x_2) during step 0
  float h[2][4] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
  int cur = 0;
  auto step_body = [&](int step, f32x4 (&g)[2][3], f32x4 (&gn)[2][3], int slot) {
    // memory work of the step (independent of the MFMAs): x rows of step + 2
    // into the tile the previous step's x-part read, the previous step's
    // outputs (none at step 0), the ring slot refilled
    stage_x(slot, step & 1);
    store_y(cur, step - 1, step > 0);
    load_x(slot, step + 2 + kXPf);
    h8x hv[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const _Float16* hb = h16[cur] + (16 * q + n) * kGxHP + 8 * lg;
#pragma unroll
      for (int s = 0; s < 4; ++s) hv[q][s] = *reinterpret_cast<const h8x*>(hb + 32 * s);
    }
    __builtin_amdgcn_sched_barrier(0);
    // h-part of this step onto the x-part (n's h-part apart, b_hn as its initial accumulator)
    f32x4 anh[2] = {b_hn, b_hn};
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        g[q][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[s], hv[q][s], g[q][0], 0, 0, 0);
        g[q][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wz[s], hv[q][s], g[q][1], 0, 0, 0);
        anh[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wn[s], hv[q][s], anh[q], 0, 0, 0);
      }
    // gate math of both tiles (tile 0 beside tile 1's h-part, tile 1 beside
    // the x-part of the next step; the last step's x-part reads a stale tile
    // and is discarded)
    h4 o[2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float hn = gru_cell(g[q][0][i], g[q][1][i], g[q][2][i], anh[q][i], h[q][i]);
        h[q][i] = hn;
        o[q][i] = (_Float16)hn;
      }
    xpart((step + 1) & 1, gn);
    constexpr int kHp = 12;           // h-part MFMAs per tile in this region
    __builtin_amdgcn_sched_group_barrier(0x008, kHp, 0);  // tile 0's h-part
#pragma unroll
    for (int i = 0; i < kHp; ++i) {                       // tile 1's h-part || tile 0's gates
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, kVpm0, 0);
    }
    // x-part || tile 1's gates: the LDS operands of k-step s + 1 (0x100: DS
    // reads) are placed ahead of k-step s's six MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // (KXR >= 1: k-step 0's A fragments are in VGPRs)
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      if (s + 1 < KXR) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      } else if (s + 1 < KX) {
        __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, VPM1, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<uint2*>(&h16[cur ^ 1][(16 * q + n) * kGxHP + u0]) = __builtin_bit_cast(uint2, o[q]);
    }
    cur ^= 1;
    __syncthreads();
  };
  for (int step = 0; step < T; step += 2) {
    step_body(step, ga, gb, 0);
    if (step + 1 < T) step_body(step + 1, gb, ga, 1);
  }
  store_y(cur, T - 1, true);   // the last step's outputs
}

// ---------------------------------------------------------------------------
// X2c / X3: bias + log_softmax + argmax, one wave per row; greedy collapse
// ---------------------------------------------------------------------------
// Online softmax state of one lane: running max (first index on ties, as
// torch.max) and the sum of exp rescaled to it.
struct SoftmaxAcc {
  float mx = -INFINITY, s = 0.0f;
  int arg = 0x7fffffff;
  __device__ __forceinline__ void push(float y, int v) {
    if (y > mx) {
      s = s * __expf(mx - y) + 1.0f;
      mx = y;
      arg = v;
    } else {
      s += __expf(y - mx);
    }
  }
};

template <typename LT> struct Vec;
template <> struct Vec<__half> { static constexpr int N = 8; };
template <> struct Vec<float> { static constexpr int N = 4; };

// tm_B > 0: logits rows are time-major (t tm_B + b); log_probs stays [b][t].
template <typename LT>
__global__ __launch_bounds__(256) void ctc_argmax_kernel(const LT* __restrict__ logits, const float* __restrict__ bias,
                                                         int64_t rows, int V, float* __restrict__ log_probs,
                                                         int* __restrict__ best, int tm_B = 0, int T = 0) {
  constexpr int NV = Vec<LT>::N;   // elements per 16-byte load
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;   // wave-uniform
  const LT* x = logits + r * V;
  SoftmaxAcc acc;
  if (V % NV == 0) {   // rows are 16-byte aligned: one 16-byte load per lane per step
    for (int c = lane; c < V / NV; c += 64) {
      LT e[NV];
      float bb[NV];
      *reinterpret_cast<uint4*>(e) = reinterpret_cast<const uint4*>(x)[c];
#pragma unroll
      for (int q = 0; q < NV / 4; ++q) *reinterpret_cast<float4*>(bb + 4 * q) = reinterpret_cast<const float4*>(bias)[c * (NV / 4) + q];
      float y[NV];
      float lm = -INFINITY;
      int li = 0;
#pragma unroll
      for (int i = 0; i < NV; ++i) {   // chunk max (first index) ...
        y[i] = (float)e[i] + bb[i];
        if (y[i] > lm) { lm = y[i]; li = i; }
      }
      float ls = 0.0f;
#pragma unroll
      for (int i = 0; i < NV; ++i) ls += __expf(y[i] - lm);   // ... independent exps, then one merge
      if (lm > acc.mx) {
        acc.s = acc.s * __expf(acc.mx - lm) + ls;
        acc.mx = lm;
        acc.arg = c * NV + li;
      } else {
        acc.s += ls * __expf(lm - acc.mx);
      }
    }
  } else {
    for (int v = lane; v < V; v += 64) acc.push((float)x[v] + bias[v], v);
  }
  float mx = acc.mx, s = acc.s;
  int arg = acc.arg;
  for (int m = 32; m >= 1; m >>= 1) {
    const float om = __shfl_xor(mx, m, 64), os = __shfl_xor(s, m, 64);
    const int oa = __shfl_xor(arg, m, 64);
    const float nm = fmaxf(mx, om);
    s = (mx == -INFINITY ? 0.0f : s * __expf(mx - nm)) + (om == -INFINITY ? 0.0f : os * __expf(om - nm));
    if (om > mx || (om == mx && oa < arg)) arg = oa;
    mx = nm;
  }
  if (log_probs) {
    const float lse = mx + logf(s);
    const int64_t orow = tm_B > 0 ? (r % tm_B) * T + r / tm_B : r;
    for (int v = lane; v < V; v += 64) log_probs[orow * V + v] = (float)x[v] + bias[v] - lse;
  }
  if (lane == 0 && best) best[r] = arg;
}

// Argmax only (no log_softmax requested: the greedy decode needs just the
// index -- log_softmax is monotonic per row, ctc.py:455 takes torch.max of
// it).  Persistent: the bias row sits in LDS once per block; each wave walks
// rows r = wave, wave + n_waves, ...; a row's 16-byte chunks are loaded up
// front (kArgChunks per lane), so a row costs one memory round trip, and the
// next row's loads are issued before the current row is reduced.  No exp.
constexpr int kArgChunks = 8;   // 16-byte chunks per lane per row
template <typename LT>
__global__ __launch_bounds__(256) void ctc_argmax_only_kernel(const LT* __restrict__ logits,
                                                              const float* __restrict__ bias, int64_t rows, int V,
                                                              int* __restrict__ best) {
  constexpr int NV = Vec<LT>::N;
  extern __shared__ float sb[];   // [V] bias
  for (int v = threadIdx.x; v < V; v += blockDim.x) sb[v] = bias[v];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int nc = V / NV;   // chunks per row (host checks V % NV == 0 and nc <= 64 * kArgChunks)
  auto load_row = [&](int64_t r, uint4 (&buf)[kArgChunks]) {
    const uint4* x = reinterpret_cast<const uint4*>(logits + r * V);
#pragma unroll
    for (int k = 0; k < kArgChunks; ++k) {
      const int c = lane + 64 * k;
      buf[k] = c < nc ? x[c] : make_uint4(0, 0, 0, 0);
    }
  };
  int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint4 cur[kArgChunks];
  if (r < rows) load_row(r, cur);
  for (; r < rows; r += nw) {
    uint4 nxt[kArgChunks];
    if (r + nw < rows) load_row(r + nw, nxt);
    float mx = -INFINITY;
    int arg = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < kArgChunks; ++k) {
      const int c = lane + 64 * k;
      if (c < nc) {
        LT e[NV];
        *reinterpret_cast<uint4*>(e) = cur[k];
#pragma unroll
        for (int i = 0; i < NV; ++i) {   // ascending index: strict > keeps the first maximum
          const float y = (float)e[i] + sb[c * NV + i];
          if (y > mx) { mx = y; arg = c * NV + i; }
        }
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float om = __shfl_xor(mx, m, 64);
      const int oa = __shfl_xor(arg, m, 64);
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
    if (lane == 0) best[r] = arg;
#pragma unroll
    for (int k = 0; k < kArgChunks; ++k) cur[k] = nxt[k];
  }
}

// decode_predictions (ctc.py:453-471): drop blanks (0) and collapse repeats,
// prev starting at the blank (ctc.py:462).  One wave per utterance, 64 frames
// at a time: a frame is kept when tok != 0 and tok != tok[t-1]; its output slot
// is the count kept so far plus the kept lanes below it (ballot + mbcnt).
// (One thread per utterance walking its T frames serially took 0.17 ms per
// 4096 utterances: strided, dependent loads.)
// tm: best is time-major (frame t of utterance b at t B + b).
// decode_predictions' per-frame argmax (ctc.py:454) in batch-major order:
// pred[b][t] from the output layer's best[] (time-major rows in fp16 mode).
__global__ __launch_bounds__(256) void ctc_pred_kernel(const int* __restrict__ best, int64_t B, int T, int tm,
                                                       int* __restrict__ pred) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= B * (int64_t)T) return;
  const int64_t b = r / T, t = r - b * T;
  pred[r] = best[tm ? t * B + b : r];
}

__global__ __launch_bounds__(256) void ctc_greedy_kernel(const int* __restrict__ best, int64_t B, int T,
                                                         int* __restrict__ tokens, int* __restrict__ lengths,
                                                         int tm = 0) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const int64_t ts = tm ? B : 1;   // frame stride
  const int* p = best + (tm ? b : b * T);
  int* o = tokens + b * T;
  int n = 0;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const int tok = t < T ? p[t * ts] : 0;
    const int prev = t == 0 ? 0 : (t < T ? p[(t - 1) * ts] : 0);
    const bool keep = tok != 0 && tok != prev;
    const uint64_t m = __ballot(keep);
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    if (keep) o[n + below] = tok;
    n += __popcll(m);
  }
  for (int t = n + lane; t < T; t += 64) o[t] = -1;
  if (lane == 0) lengths[b] = n;
}

// ---------------------------------------------------------------------------
// X2 output layer + X3 argmax, fused (fp16 mode): best[r] = first argmax over
// v of (y[r] . W[v] + b[v]) with y [rows][256] and W [V][256] in fp16, fp32
// accumulation on v_mfma_f32_16x16x32_f16 -- the [rows][V] logits never touch
// HBM (they were 2 x 9.9 GB of traffic per 4096 utterances).  A workgroup owns
// kOutRows rows: each of its kOutWaves waves keeps its 16 kOutRF rows' A
// fragments in VGPRs (kOutRF row tiles x 8 K-steps) and walks V in 64-column tiles of W staged through
// a double-buffered LDS image (512-byte rows, 16-byte chunks XOR-swizzled: a
// B-fragment ds_read_b128 is conflict-free), one barrier per tile.  Each lane keeps
// a running (max, index) for its 4 RF rows over its columns, visited in increasing
// order, then 16-lane shuffles pick the first maximum (torch.max semantics).
// LOGITS = true also stores the fp16 logits (bias included) for the log_softmax
// kernel; the argmax is this kernel's in both cases and both variants
// accumulate identically (bias as the first MFMA's C operand, the same K
// order), so tokens do not depend on log-probs being requested.
// ---------------------------------------------------------------------------
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
// Double-buffered W tiles of 64 columns, 3 row tiles per wave, 8 waves (a
// four-buffer ring with the LDS-DMA two tiles ahead, 32- and 128-column tiles,
// 12 waves were measured slower: DESIGN 5.3).
constexpr int kOutNB = 2, kOutAhead = 1;
constexpr int kOutK = 2 * kH, kOutBN = 64, kOutCF = kOutBN / 16, kOutPitch = kOutK, kOutRF = 3, kOutWaves = 8;
// W tile rows are 512 B with their 16-byte chunks XOR-swizzled by the row's
// low 4 bits (chunk c of row n at c ^ (n & 15)): a ds_read_b128 B fragment
// (row 16 cf + li, chunk 4 st + lg) then hits 16 distinct 4-bank windows in
// each of the instruction's four lane groups.  (With the former padded pitch
// of 264 halfs, 42 % of the kernel's LDS cycles were bank conflicts, PMC.)
__device__ __forceinline__ int out_chunk(int n, int c) { return c ^ (n & 15); }
// (RF = 3, 48 rows per wave: each B fragment read from LDS feeds 3 MFMAs -- the
// LDS bytes per MFMA were the limit at RF = 2; 246 VGPRs, still 2 waves per
// SIMD: +3 % utterances/s.)
constexpr int out_rf(bool logits) { return logits ? 2 : kOutRF; }
constexpr int out_rows(bool logits) { return 16 * out_rf(logits) * kOutWaves; }
// KEYED (V <= 4096, so 4 NT <= 256): the running maximum carries its column
// in the value's low 8 mantissa bits, so the epilogue is one VALU per value
// (v_and_or_b32) and one v_max3_f32 per two values instead of compare + two
// selects per value.  The tag is 255 - (4 tile + cf): among values whose
// upper 24 bits agree, an earlier column makes the larger tagged value when
// they are positive, so equal logits keep the first index, as torch.argmax
// does (ctc.py:454).  Between negative values the tag orders the other way
// (round 4 spread the sign into the tag with a v_perm_b32 first: two VALU per
// value); such a tie is within 2^-15 of the row's maximum, which makes the
// row a near-tie that ctc_rescore_kernel decides again in fp32 with the
// first-index rule.  The column is 16 (4 tile + cf) + li.  A tagged value
// moves by < 2^-15 of itself: the first maximum is exact except between
// logits that agree to within that (fp16 operands already put ~1e-3 of noise
// on every logit); the tokens stay a function of the row alone.
// m = max(m, k0, k1) on the tagged values (fmaxf would first canonicalise
// each of them: they come from integer ops).  The tags are applied in C++, so
// the compiler still places the wait states for reading MFMA results.
__device__ __forceinline__ float out_max3(float m, float k0, float k1) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(k0), "v"(k1));
  return r;
}
// mask = 0xffffff00 (in a VGPR: VOP3 takes no literal), tag in an SGPR
__device__ __forceinline__ float out_tag(float x, unsigned mask, unsigned tag) {
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, x) & mask) | tag);
}
// Runner-up tracking (KEYED): the second largest of {m, k0, k1} is their
// median; the row's running second maximum is max(m2, med3(m, k0, k1)), and
// over four values max3(m2, med3(m, k0, k1), med3(max3(m, k0, k1), k2, k3)).
__device__ __forceinline__ float out_med3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// Near-tie re-scoring (decision parity): a row whose top-2 tagged
// logits are closer than this is re-decided between those two columns in fp32
// (ctc_rescore_kernel).  The fp16 operands move a logit by ~3e-4 rms here
// (256 products of fp16-rounded weights); the margin test is generous.
__device__ __forceinline__ bool out_near_tie(float m1, float m2) {
  return m1 - m2 < 4e-3f + 2e-3f * fabsf(m1);
}

// The column block (4 tile + cf) of a tagged value.
__device__ __forceinline__ int out_untag(float m) { return (int)(255u - (__builtin_bit_cast(unsigned, m) & 255u)); }
template <bool LOGITS, bool KEYED>
__global__ __launch_bounds__(kOutWaves * 64) void ctc_out_argmax16_kernel(const __half* __restrict__ y,
                                                                          const __half* __restrict__ w,
                                                                          const float* __restrict__ bias, int64_t rows,
                                                                          int V, __half* __restrict__ logits,
                                                                          int* __restrict__ best,
                                                                          int* __restrict__ best2) {
  constexpr int kOutRF = out_rf(LOGITS), kOutRows = out_rows(LOGITS);
  __shared__ __attribute__((aligned(1024))) _Float16 bt[kOutNB][kOutBN * kOutPitch];   // (EARLYDMA: row addresses XOR the chunk)
  // the tile's bias, staged with its W rows (an L2 load per column in the
  // epilogue stalled it); replicated x4 so one ds_read_b128 is an MFMA C operand
  __shared__ f32x4 bsh[kOutNB][kOutBN];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const bool wave0 = __builtin_amdgcn_readfirstlane(wv) < (kOutBN + 63) / 64;   // the waves that stage the tile's bias
  const int64_t row0 = (int64_t)blockIdx.x * kOutRows + 16 * kOutRF * wv;
  // A fragments: rows row0 + 16 rf + li, k = 32 s + 8 lg .. +7
  h8 a[kOutRF][8];
#pragma unroll
  for (int rf = 0; rf < kOutRF; ++rf) {
    const int64_t r = row0 + 16 * rf + li;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      uint4 v = make_uint4(0, 0, 0, 0);
      // Non-temporal: the once-read y rows do not evict the W tiles every
      // workgroup re-reads from L2 (PMC: 851 -> 681 MB per launch against
      // 638 MB algorithmic, same time; profiles/r05c_*_ctc_hbm_traffic.json).
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      if (r < rows) {
        const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(y + r * kOutK + 32 * st + 8 * lg));
        v = make_uint4(t[0], t[1], t[2], t[3]);
      }
      a[rf][st] = __builtin_bit_cast(h8, v);
    }
  }
  const int NT = (V + kOutBN - 1) / kOutBN;
  // W tile nt -> registers: 64 rows x 32 16-byte chunks, 4 per thread.  Buffer
  // loads: rows past V come back 0 from the range check, no branch per load.
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(w, (uint32_t)V * kOutK * 2);
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(bias, (uint32_t)V * 4);
  float pb = 0.0f;
  // W tile nt -> bt[nt & 1] by LDS-DMA (buffer_load ... lds), issued by waves
  // 0-3 after their MFMA phase: instruction i of wave w fills 1 KB = rows
  // 2 (8 w + i) and +1; lane L writes position L & 31 of its row, so it loads
  // global chunk (L & 31) ^ (row & 15) -- the swizzle is in the global
  // addresses.  The compiler makes every LDS read after an LDS-DMA wait for
  // it, so no wave issues one before its own B-fragment reads of the period;
  // the target buffer was last read in the previous period, and the explicit
  // vmcnt(0) before the closing barrier completes the DMA.
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  constexpr int kDmaWaves = 4, kDmaPer = kOutBN * kOutK * 2 / 1024 / kDmaWaves;   // waves 0-3 (leading) issue the DMA
  // per-lane global offsets within a tile are tile-invariant: computed once,
  // the tile's base goes in the scalar offset
  int dma_off[kDmaPer];
#pragma unroll
  for (int i = 0; i < kDmaPer; ++i) {
    const int q = (wvu < kDmaWaves ? wvu : 0) * kDmaPer + i, rr = 2 * q + (lane >> 5), c = (lane & 31) ^ (rr & 15);
    dma_off[i] = rr * (kOutK * 2) + 16 * c;
  }
  auto dma_piece = [&](int nt, int i) {
    const int q = wvu * kDmaPer + i;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)&bt[nt & (kOutNB - 1)][q * 512], 16,
                                             dma_off[i], nt * (kOutBN * kOutK * 2), 0, 0);
  };
  auto dma_w = [&](int nt) {
    if (wvu >= kDmaWaves) return;
#pragma unroll
    for (int i = 0; i < kDmaPer; ++i) dma_piece(nt, i);
  };
  auto fetch = [&](int nt) {   // the tile's bias (W comes by dma_w)
    if (wave0) pb = buf_load(brs, 4 * (nt * kOutBN + tid), 0);
  };
  auto stash = [&](int buf) {
    if (wave0 && tid < kOutBN) bsh[buf][tid] = f32x4{pb, pb, pb, pb};
  };
  fetch(0);
  stash(0);
  dma_w(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float mx[kOutRF][4], mx2[kOutRF][4];   // (mx2: KEYED runner-up)
  int ix[kOutRF][4];
  unsigned kmask;   // (KEYED) out_tag's mask, in a VGPR (VOP3 takes no literal)
  asm("v_mov_b32 %0, 0xffffff00" : "=v"(kmask));
#pragma unroll
  for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
    for (int i = 0; i < 4; ++i) { mx[rf][i] = -INFINITY; mx2[rf][i] = -INFINITY; ix[rf][i] = 0; }
  // Skew: the second half of the waves (4-7, each the partner of
  // a first-half wave on the same SIMD) runs one tile behind in its epilogue:
  // per tile it finishes tile nt - 1's argmax first, then issues tile nt's
  // MFMAs, while the first half issues tile nt's MFMAs and then its epilogue.
  // The barrier keeps all waves on one tile; the skew puts one wave's epilogue
  // VALU beside its partner's MFMAs instead of both SIMD waves alternating
  // all-MFMA and all-VALU phases in step.
  // lagging: waves 4-7, one of the two waves of each SIMD
  const bool lag = (__builtin_amdgcn_readfirstlane(wv) >> 2) & 1;
  // The bias is the MFMAs' initial C operand (one ds_read_b128 of the
  // replicated bias per column tile), so the epilogue is compare + select.
  f32x4 acc[kOutRF][kOutCF];
  // (FULL: every column of the tile is < V -- all tiles but a ragged last
  // one -- so the per-lane bound check and its exec-mask blocks go)
  auto epilogue_t = [&](int tile, auto full) __attribute__((always_inline)) {
    // column v = 64 tile + 16 cf + li, rows row0 + 16 rf + 4 lg + i
#pragma unroll
    for (int cf = 0; cf < kOutCF; ++cf) {
      const int v = tile * kOutBN + 16 * cf + li;
      if (KEYED) {
        const unsigned tag = 255u - (unsigned)(kOutCF * tile + cf);
        if (LOGITS) {
#pragma unroll
          for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int64_t r = row0 + 16 * rf + 4 * lg + i;
              if ((decltype(full)::value || v < V) && r < rows) logits[r * V + v] = __float2half(acc[rf][cf][i]);
            }
        }
        static_assert(kOutCF == 4, "the epilogue folds the tile's four column blocks at once");
        if (cf == kOutCF - 1) {   // all four column blocks: four tagged values per two v_max3_f32
#pragma unroll
          for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float x[4];
#pragma unroll
              for (int c = 0; c < 4; ++c) {   // (-FLT_MAX past V: tagged -inf would be a NaN)
                x[c] = acc[rf][c][i];
                if (!decltype(full)::value) x[c] = tile * kOutBN + 16 * c + li < V ? x[c] : -FLT_MAX;
              }
              const float t0 = out_tag(x[0], kmask, tag + 3), t1 = out_tag(x[1], kmask, tag + 2);
              const float t2 = out_tag(x[2], kmask, tag + 1), t3 = out_tag(x[3], kmask, tag);
              const float m = mx[rf][i], a = out_med3(m, t0, t1), m1 = out_max3(m, t0, t1);
              const float b = out_med3(m1, t2, t3);
              mx[rf][i] = out_max3(m1, t2, t3);
              mx2[rf][i] = out_max3(mx2[rf][i], a, b);
            }
        }
      } else if (decltype(full)::value || v < V) {
#pragma unroll
        for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float z = acc[rf][cf][i];
            if (z > mx[rf][i]) { mx[rf][i] = z; ix[rf][i] = v; }
            if (LOGITS) {
              const int64_t r = row0 + 16 * rf + 4 * lg + i;
              if (r < rows) logits[r * V + v] = __float2half(acc[rf][cf][i]);
            }
          }
      }
    }
  };
  auto epilogue = [&](int tile) __attribute__((always_inline)) {
    if ((tile + 1) * kOutBN <= V) epilogue_t(tile, std::true_type{});
    else epilogue_t(tile, std::false_type{});
  };
  for (int nt = 0; nt < NT; ++nt) {
    if (nt + kOutAhead < NT) fetch(nt + kOutAhead);
    const _Float16* b = bt[nt & (kOutNB - 1)];
    if (lag && nt > 0) epilogue(nt - 1);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      h8 bf[kOutCF];
#pragma unroll
      for (int cf = 0; cf < kOutCF; ++cf)
        bf[cf] = *reinterpret_cast<const h8*>(b + (16 * cf + li) * kOutPitch + 8 * out_chunk(li, 4 * st + lg));
      if (st == 0) {
#pragma unroll
        for (int cf = 0; cf < kOutCF; ++cf) {
          const f32x4 c0 = bsh[nt & (kOutNB - 1)][16 * cf + li];
#pragma unroll
          for (int rf = 0; rf < kOutRF; ++rf)
            acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rf][0], bf[cf], c0, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
          for (int cf = 0; cf < kOutCF; ++cf)
            acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rf][st], bf[cf], acc[rf][cf], 0, 0, 0);
      }
    }
    if (!lag && nt + kOutAhead < NT) {   // after this wave's last LDS read of the period
      stash((nt + kOutAhead) & (kOutNB - 1));
      dma_w(nt + kOutAhead);
    }
    if (!lag) epilogue(nt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // LDS-DMA done (the barrier's own wait omits it)
    __syncthreads();
  }
  if (lag && NT > 0) epilogue(NT - 1);
  // first maximum across the 16 column lanes of each row
#pragma unroll
  for (int rf = 0; rf < kOutRF; ++rf)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float m = mx[rf][i];
      int k = KEYED ? 16 * out_untag(m) + li : ix[rf][i];
      float m2 = mx2[rf][i];   // (KEYED) runner-up and its column
      int k2 = KEYED ? 16 * out_untag(m2) + li : -1;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float om = __shfl_xor(m, o, 64);
        const int ok = __shfl_xor(k, o, 64);
        if (KEYED) {
          const float om2 = __shfl_xor(m2, o, 64);
          const int ok2 = __shfl_xor(k2, o, 64);
          // the merged runner-up: the loser of the two maxima, or the larger runner-up
          const bool other_wins = om > m || (om == m && ok < k);
          const float lm = other_wins ? m : om;
          const int lk = other_wins ? k : ok;
          const bool r_other = om2 > m2 || (om2 == m2 && ok2 < k2);
          const float rm = r_other ? om2 : m2;
          const int rk = r_other ? ok2 : k2;
          const bool use_loser = lm > rm || (lm == rm && lk < rk);
          m2 = use_loser ? lm : rm;
          k2 = use_loser ? lk : rk;
        }
        if (om > m || (om == m && ok < k)) { m = om; k = ok; }
      }
      const int64_t r = row0 + 16 * rf + 4 * lg + i;
      if (li == 0 && r < rows) {
        best[r] = k;
        best2[r] = KEYED && m2 > -INFINITY && out_near_tie(m, m2) ? k2 : -1;
      }
    }
}

// Decode-only form of the kernel above (KEYED, no logits: wk_ctc_transcribe's
// path), with the epilogue moved in among the MFMAs.  A tile's four
// column blocks are computed in two halves (blocks 0-1, then 2-3); each half's
// 48 MFMAs carry the fold of the OTHER half's finished accumulators (blocks
// 2-3 of the previous tile, then blocks 0-1 of this one), one item per k-step
// with a sched_barrier after each, so the fold's VALU goes into the cycles a
// v_mfma_f32_16x16x32_f16 leaves (8 of its 16) with no second accumulator set.
// Both waves of a SIMD run the same schedule (no skew).  The next tile's W
// goes into the other LDS buffer by DMA at the start of the period (separate
// arrays: the compiler sees they cannot alias, so no read waits for it).
// Columns past V get bias -1e30 and read W rows of 0, so no tile needs a
// bound check; the first tile's dummy fold reads accumulators preset to -1e30.
// Tokens are the same as ctc_out_argmax16_kernel<false, true>'s (same
// accumulation order per logit, same tags; the folds take exact max/median).
__global__ __launch_bounds__(kOutWaves * 64) void ctc_out_decode16_kernel(const __half* __restrict__ y,
                                                                          const __half* __restrict__ w,
                                                                          const float* __restrict__ bias, int64_t rows,
                                                                          int V, int* __restrict__ best,
                                                                          int* __restrict__ best2) {
  constexpr int RF = kOutRF, kRows = 16 * RF * kOutWaves;
  // Two separate W buffers (and bias buffers), selected at compile time: the
  // compiler then knows the LDS-DMA into one cannot alias the B-fragment reads
  // of the other, so a period can start the next tile's DMA and still read its
  // own tile without waiting for it (with one array it waits at the first read).
  __shared__ __attribute__((aligned(1024))) _Float16 bt0[kOutBN * kOutPitch];
  __shared__ __attribute__((aligned(1024))) _Float16 bt1[kOutBN * kOutPitch];
  __shared__ f32x4 bsh0[kOutBN], bsh1[kOutBN];   // the tile's bias x4 (an MFMA C operand)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wvu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * kRows + 16 * RF * wvu;
  h8 a[RF][8];   // A fragments: rows row0 + 16 rf + li, k = 32 st + 8 lg .. +7
#pragma unroll
  for (int rf = 0; rf < RF; ++rf) {
    const int64_t r = row0 + 16 * rf + li;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      uint4 v = make_uint4(0, 0, 0, 0);
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      if (r < rows) {   // non-temporal, as above
        const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(y + r * kOutK + 32 * st + 8 * lg));
        v = make_uint4(t[0], t[1], t[2], t[3]);
      }
      a[rf][st] = __builtin_bit_cast(h8, v);
    }
  }
  const int NT = (V + kOutBN - 1) / kOutBN;
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(w, (uint32_t)V * kOutK * 2);
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(bias, (uint32_t)V * 4);
  // W tiles by LDS-DMA (as above), 4 pieces per wave, all 8 waves
  constexpr int kDmaPer = kOutBN * kOutK * 2 / 1024 / kOutWaves;
  int dma_off[kDmaPer];
#pragma unroll
  for (int i = 0; i < kDmaPer; ++i) {
    const int q = wvu * kDmaPer + i, rr = 2 * q + (lane >> 5), c = (lane & 31) ^ (rr & 15);
    dma_off[i] = rr * (kOutK * 2) + 16 * c;
  }
  auto dma_w = [&](_Float16* dst, int nt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kDmaPer; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)&dst[(wvu * kDmaPer + i) * 512],
                                               16, dma_off[i], nt * (kOutBN * kOutK * 2), 0, 0);
  };
  float pb = 0.0f;
  auto fetch = [&](int nt) {   // wave 0: the tile's bias (used at stash: no wait here)
    if (wvu == 0) pb = buf_load(brs, 4 * (nt * kOutBN + lane), 0);
  };
  auto stash = [&](f32x4* dst, int nt) {   // -1e30 past V
    const float v = nt * kOutBN + lane < V ? pb : -1e30f;
    if (wvu == 0) dst[lane] = f32x4{v, v, v, v};
  };
  fetch(0);
  stash(bsh0, 0);
  dma_w(bt0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float mx[RF][4], mx2[RF][4];
  f32x4 acc[RF][kOutCF];
#pragma unroll
  for (int rf = 0; rf < RF; ++rf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { mx[rf][i] = -INFINITY; mx2[rf][i] = -INFINITY; }
#pragma unroll
    for (int cf = 2; cf < kOutCF; ++cf) acc[rf][cf] = f32x4{-1e30f, -1e30f, -1e30f, -1e30f};   // the first dummy fold
  }
  unsigned kmask;   // out_tag's mask, in a VGPR (VOP3 takes no literal)
  asm("v_mov_b32 %0, 0xffffff00" : "=v"(kmask));
  float carry[RF][4];   // a tile's blocks 0-1 median, folded with its blocks 2-3 (the runner-up, 4 values at once)
#pragma unroll
  for (int rf = 0; rf < RF; ++rf)
#pragma unroll
    for (int i = 0; i < 4; ++i) carry[rf][i] = -INFINITY;
  // One half: blocks 2h and 2h + 1 of the tile in (b, bs) (16 steps of one B
  // fragment x RF MFMAs; fragments read two steps ahead), with the fold of
  // blocks 2eh, 2eh + 1 of tile etile (12 items of 5 VALU) spread one item per
  // step; a sched_barrier after each step keeps that order.
  auto half = [&](const _Float16* b, const f32x4* bs, int h, int etile, int eh) __attribute__((always_inline)) {
    auto frag = [&](int s) -> h8 {
      const int cf = 2 * h + (s >> 3), st = s & 7;
      return *reinterpret_cast<const h8*>(b + (16 * cf + li) * kOutPitch + 8 * out_chunk(li, 4 * st + lg));
    };
    const unsigned tag = 255u - (unsigned)(kOutCF * etile + 2 * eh);   // block 2eh; block 2eh + 1: tag - 1
    constexpr int PD = 4;   // fragment prefetch distance in steps (2: +1.5 % time; profiles/r05p_dec16_variants_ab.txt)
    f32x4 c0 = bs[16 * (2 * h) + li];
    h8 ring[PD + 1];
#pragma unroll
    for (int q = 0; q < PD; ++q) ring[q] = frag(q);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int cf = 2 * h + (s >> 3), st = s & 7;
      if (s + PD < 16) ring[(s + PD) % (PD + 1)] = frag(s + PD);
      if (s == 8) c0 = bs[16 * cf + li];
      const h8 bf = ring[s % (PD + 1)];
#pragma unroll
      for (int rf = 0; rf < RF; ++rf)
        acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rf][st], bf, st == 0 ? c0 : acc[rf][cf], 0, 0, 0);
      if (s < RF * 4) {   // fold item s: row block rf, row i
        const int rf = s >> 2, i = s & 3;
        const float t0 = out_tag(acc[rf][2 * eh][i], kmask, tag), t1 = out_tag(acc[rf][2 * eh + 1][i], kmask, tag - 1);
        const float m = mx[rf][i];
        if (eh == 0) {   // one runner-up update per tile: blocks 0-1's median waits for blocks 2-3's (-1 VALU / 4 logits)
          carry[rf][i] = out_med3(m, t0, t1);
        } else {
          mx2[rf][i] = out_max3(mx2[rf][i], carry[rf][i], out_med3(m, t0, t1));
        }
        mx[rf][i] = out_max3(m, t0, t1);
      }
      __builtin_amdgcn_sched_barrier(0);   // (without: the compiler clusters the fold, +1.5-3 % time)
    }
  };
  // One period: tile nt from (b, bs); the next tile's W and bias go into (nb, nbs)
  // at its start (the other buffers were last read in the previous period).
  auto period = [&](const _Float16* b, const f32x4* bs, _Float16* nb, f32x4* nbs, int nt) __attribute__((always_inline)) {
    const bool more = nt + 1 < NT;
    if (more) {   // (the pieces spread among the MFMAs, one per 4 steps, or s_setprio 1 for waves 4-7: within +-1 %)
      fetch(nt + 1);
      dma_w(nb, nt + 1);
    }
    half(b, bs, 0, nt > 0 ? nt - 1 : 0, 1);   // blocks 0-1 || fold of the previous tile's blocks 2-3
    half(b, bs, 1, nt, 0);                    // blocks 2-3 || fold of this tile's blocks 0-1
    if (more) stash(nbs, nt + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // LDS-DMA done (the barrier's own wait omits it)
    __syncthreads();
  };
  for (int nt = 0; nt < NT; nt += 2) {
    period(bt0, bsh0, bt1, bsh1, nt);
    if (nt + 1 < NT) period(bt1, bsh1, bt0, bsh0, nt + 1);
  }
  {   // the last tile's blocks 2-3
    const unsigned tag = 255u - (unsigned)(kOutCF * (NT - 1) + 2);
#pragma unroll
    for (int rf = 0; rf < RF; ++rf)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float t0 = out_tag(acc[rf][2][i], kmask, tag), t1 = out_tag(acc[rf][3][i], kmask, tag - 1);
        const float m = mx[rf][i];
        mx2[rf][i] = out_max3(mx2[rf][i], carry[rf][i], out_med3(m, t0, t1));
        mx[rf][i] = out_max3(m, t0, t1);
      }
  }
  // first maximum across the 16 column lanes of each row (as above)
#pragma unroll
  for (int rf = 0; rf < RF; ++rf)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float m = mx[rf][i], m2 = mx2[rf][i];
      int k = 16 * out_untag(m) + li, k2 = 16 * out_untag(m2) + li;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float om = __shfl_xor(m, o, 64), om2 = __shfl_xor(m2, o, 64);
        const int ok = __shfl_xor(k, o, 64), ok2 = __shfl_xor(k2, o, 64);
        const bool other_wins = om > m || (om == m && ok < k);
        const float lm = other_wins ? m : om;
        const int lk = other_wins ? k : ok;
        const bool r_other = om2 > m2 || (om2 == m2 && ok2 < k2);
        const float rm = r_other ? om2 : m2;
        const int rk = r_other ? ok2 : k2;
        const bool use_loser = lm > rm || (lm == rm && lk < rk);
        m2 = use_loser ? lm : rm;
        k2 = use_loser ? lk : rk;
        if (other_wins) { m = om; k = ok; }
      }
      const int64_t r = row0 + 16 * rf + 4 * lg + i;
      if (li == 0 && r < rows) {
        best[r] = k;
        best2[r] = m2 > -INFINITY && out_near_tie(m, m2) ? k2 : -1;
      }
    }
}

// Near-tie re-scoring after the fp16 output kernels (V <= 4096): a row whose
// top-2 logits came within out_near_tie of each other is decided between those
// two columns again with fp32 weights (y is the fp16 GRU output, widened
// exactly): bias + sum_k y[k] W[c][k] in fp32, the larger wins, an exact tie
// keeps the smaller column (torch.argmax).  Rows with best2 < 0 keep their fp16
// decision.  A wave takes 64 consecutive rows, finds the flagged ones with a
// ballot and re-scores them one at a time with all 64 lanes (4 k per lane, a
// shuffle-tree sum): the flagged rows are a few percent, and one thread per row
// walking a 256-long dependent FMA chain had cost ~0.11 ms per batch.
__global__ __launch_bounds__(256) void ctc_rescore_kernel(const __half* __restrict__ y, const float* __restrict__ w,
                                                          const float* __restrict__ bias, int64_t rows,
                                                          int* __restrict__ best, const int* __restrict__ best2) {
  const int lane = threadIdx.x & 63;
  const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (base >= rows) return;   // (wave-uniform)
  const int64_t r = base + lane;
  const int c2l = r < rows ? best2[r] : -1;
  uint64_t mask = __ballot(c2l >= 0);
  while (mask) {   // (wave-uniform)
    const int j = __builtin_ctzll(mask);
    mask &= mask - 1;
    const int64_t rj = base + j;
    const int c2 = __shfl(c2l, j, 64), c1 = best[rj];
    const __half2* yr = reinterpret_cast<const __half2*>(y + rj * (2 * kH)) + 2 * lane;
    const float4 w1 = reinterpret_cast<const float4*>(w + (int64_t)c1 * (2 * kH))[lane];
    const float4 w2 = reinterpret_cast<const float4*>(w + (int64_t)c2 * (2 * kH))[lane];
    const float2 ya = __half22float2(yr[0]), yb = __half22float2(yr[1]);
    float s1 = __builtin_fmaf(ya.x, w1.x, __builtin_fmaf(ya.y, w1.y, __builtin_fmaf(yb.x, w1.z, yb.y * w1.w)));
    float s2 = __builtin_fmaf(ya.x, w2.x, __builtin_fmaf(ya.y, w2.y, __builtin_fmaf(yb.x, w2.z, yb.y * w2.w)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    s1 += bias[c1];
    s2 += bias[c2];
    if (lane == 0 && (s2 > s1 || (s2 == s1 && c2 < c1))) best[rj] = c2;
  }
}

// Window starts of ctc_logmel_fft2_kernel's straight-line filterbank.  A tap
// is a ds_read_b64 of the pair-power row at bin ws[lane] + j, served 32 lanes
// at a time: two lanes of a half-wave share banks when their starts differ by
// a nonzero multiple of 32 bins.  A filter shorter than its window can start
// up to (window - length) bins early (the extra taps weigh 0), so the starts
// are chosen with distinct residues mod 32 per half-wave where possible
// (equal starts are free: one address is a broadcast).  Set 1: mel l over
// kMelW1 bins; set 2 (lanes 0-31): mel 64 + l / 2 split at cut[l] between two
// kMelW2-bin windows.  A half-wave without a solution keeps the natural starts.
void pick_mel_windows(const std::vector<int>& st, const std::vector<int>& ln, std::vector<int>& ws, std::vector<int>& cut) {
  auto conflict_free = [](const int* w, int n) {
    for (int a = 0; a < n; ++a)
      for (int b = a + 1; b < n; ++b)
        if (w[a] != w[b] && (w[a] - w[b]) % 32 == 0) return false;
    return true;
  };
  // set 1, per half-wave: bipartite matching of lanes to residues
  for (int h = 0; h < 2; ++h) {
    int* w = &ws[32 * h];
    for (int l = 0; l < 32; ++l) w[l] = std::min(st[32 * h + l], kBins - kMelW1);
    if (conflict_free(w, 32)) continue;
    int owner[32], pick[32];
    std::fill(owner, owner + 32, -1);
    std::function<bool(int, unsigned&)> aug = [&](int l, unsigned& seen) -> bool {
      const int m = 32 * h + l, hi = std::min(st[m], kBins - kMelW1), lo = std::max(0, st[m] + ln[m] - kMelW1);
      for (int s = hi; s >= lo; --s) {
        const int r = s & 31;
        if (seen >> r & 1u) continue;
        seen |= 1u << r;
        if (owner[r] < 0 || aug(owner[r], seen)) { owner[r] = l; pick[l] = s; return true; }
      }
      return false;
    };
    bool ok = true;
    for (int l = 0; l < 32 && ok; ++l) { unsigned seen = 0; ok = aug(l, seen); }
    if (ok)
      for (int l = 0; l < 32; ++l) w[l] = pick[l];
  }
  // set 2: per mel a pair (h0, h1); the cut is h0 + kMelW2.  Depth-first,
  // most constrained mel first, with a node budget (then natural starts)
  int sol[16][2], order[16], nopt[16];
  std::vector<std::pair<int, int>> opts[16];
  for (int p = 0; p < 16; ++p) {
    const int m = 64 + p;
    for (int h0 = std::max(0, st[m] + ln[m] - 2 * kMelW2); h0 <= st[m]; ++h0)
      for (int h1 = std::max(h0, st[m] + ln[m] - kMelW2); h1 <= std::min(h0 + kMelW2, kBins - kMelW2); ++h1)
        if ((h0 & 31) != (h1 & 31)) opts[p].push_back({h0, h1});
    nopt[p] = (int)opts[p].size();
    order[p] = p;
  }
  std::stable_sort(order, order + 16, [&](int a, int b) { return nopt[a] < nopt[b]; });
  unsigned used = 0;
  long budget = 1 << 20;
  std::function<bool(int)> bt = [&](int d) -> bool {
    if (d == 16) return true;
    const int p = order[d];
    for (const auto& o : opts[p]) {
      if (--budget < 0) return false;
      const unsigned bits = (1u << (o.first & 31)) | (1u << (o.second & 31));
      if (used & bits) continue;
      used |= bits;
      sol[p][0] = o.first;
      sol[p][1] = o.second;
      if (bt(d + 1)) return true;
      used &= ~bits;
    }
    return false;
  };
  const bool ok2 = bt(0);
  for (int l = 0; l < 32; ++l) {
    const int m = 64 + l / 2;
    const int h0 = ok2 ? sol[l / 2][0] : std::min(st[m], kBins - kMelW2);
    const int h1 = ok2 ? sol[l / 2][1] : std::min(st[m] + kMelW2, kBins - kMelW2);
    ws[64 + l] = (l & 1) ? h1 : h0;
    cut[64 + l] = (l & 1) ? kBins : std::min(h0 + kMelW2, h1 + kMelW2);
  }
  // (lanes 32-63 of set 2 carry zero weights and all read bin 0: a broadcast)
}

// HTK mel filterbank of torchaudio.functional.melscale_fbanks(201, 0, 8000, 80, 16000), in fp32 like torch.
void mel_fbank(std::vector<float>& fb) {
  fb.assign((size_t)kBins * kMels, 0.0f);
  const double m_min = 0.0, m_max = 2595.0 * log10(1.0 + 8000.0 / 700.0);
  std::vector<float> f_pts(kMels + 2), freqs(kBins);
  for (int i = 0; i < kMels + 2; ++i) {
    const float m = (float)(m_min + (m_max - m_min) * i / (kMels + 1));
    f_pts[i] = 700.0f * (powf(10.0f, m / 2595.0f) - 1.0f);
  }
  for (int k = 0; k < kBins; ++k) freqs[k] = (float)(8000.0 * k / (kBins - 1));
  for (int k = 0; k < kBins; ++k)
    for (int m = 0; m < kMels; ++m) {
      const float down = -(f_pts[m] - freqs[k]) / (f_pts[m + 1] - f_pts[m]);
      const float up = (f_pts[m + 2] - freqs[k]) / (f_pts[m + 2] - f_pts[m + 1]);
      const float v = fminf(down, up);
      fb[(size_t)k * kMels + m] = v > 0.0f ? v : 0.0f;
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
struct wk_ctc {
  wk_ctc_config cfg;
  int n_cu;
  bool f16;             // precision 1: GEMM operands in fp16 (fp32 accumulate); recurrence fp32
  // weights (device)
  float *enc_w, *enc_b, *ln_g, *ln_b;
  float* wih[2];        // per layer: [768][Din] (fwd rows then reverse rows)
  float* bih[2];        // per layer: [768]
  float* bhh[2];        // per layer: [768]
  float* whh_pk[2];     // per layer: [2 dir][24 tiles][32 k-steps][64 lanes]
  float *out_w, *out_b; // [V][256], [V]
  float* zero_b;        // [V] zeros: the log_softmax kernel's bias in fp16 mode (the logits carry theirs)
  __half* wih16[2];     // fp16 copies (precision 1)
  __half* whh16_pk[2];  // per layer: [2 dir][24 tiles][8 k-steps][64 lanes][4]
  __half* whh16x_pk[2]; // per layer: [2 dir][3 gates][8 waves][4 k-steps][64 lanes][8] (W_hh as 16x16x32 fragments, gate-scaled)
  __half* wih16x_pk[2]; // per layer: [2 dir][3 gates][8 waves][din/32 k-steps][64 lanes][8] (fused-projection GRU, gate-scaled)
  bool gru_gemm;        // fp16 mode: input projections as a separate GEMM (WAKEWORD_CTC_GEMM=1; A/B and checks)
  // Decision-parity attribution (WAKEWORD_CTC_MIX): 1 = "out32", the fp16
  // path up to the last GRU layer, then the output layer in fp32 (y1 widened,
  // fp32 W); 2 = "out16", the fp32 path with the fp16 output kernel (y1 and W
  // rounded to fp16).  0 (default) = the precision's own output layer.
  int mix;
  int rescore;          // fp16 output layer: near-tie rows re-decided in fp32 (default; WAKEWORD_CTC_RESCORE=0 off, A/B)
  __half* out_w16;
  float* fft_win;       // [400] periodic Hann
  float* fft_tw;        // [20 k1][20 n2] W400^(n2 k1), complex
  float* melw;          // ctc_logmel_fft2_kernel: per-lane padded mel weights x 1/4, [64][kMelW1] then [64][kMelW2]
  int* melws;           // their window start bins, [64] then [64]
  // workspaces (grown on demand)
  size_t ws_rows;
  float *x0, *gi, *y0, *y1, *logits;
  __half *x0h, *y0h, *y1h, *logits16;
  int* best;
  int* best2;           // fp16 mode: the runner-up column of near-tie rows (else -1), for ctc_rescore_kernel
  float* tr_feats;      // wk_ctc_transcribe: [rows][80] features (raw in fp16 mode), pass partials, per-utterance z-score
  float2* tr_part;       // [tr_slots] per-wave log-mel statistics (ctc_logmel_fft2_kernel<true>)
  float2* tr_zs;
  size_t tr_rows, tr_batch, tr_slots;
  int64_t last_batch;   // geometry of the last wk_ctc_forward (wk_ctc_frame_argmax)
  int32_t last_T;
  // stage timing (wk_ctc_profile): events recorded around each stage on the
  // call's stream, folded into per-stage sums when read or when the ring fills
  int prof;
  struct { int stage; hipEvent_t a, b; } ev[64];
  int n_ev;
  double stage_ms[WK_CTC_N_STAGES];
  int64_t stage_n[WK_CTC_N_STAGES];
};

namespace {

int64_t ctc_num_weights(const wk_ctc_config* c) {
  const int64_t H = c->hidden, V = c->vocab;
  int64_t n = H * kMels + 3 * H;
  for (int l = 0; l < 2; ++l) n += 2 * (3 * H * (l == 0 ? H : 2 * H) + 3 * H * H + 6 * H);
  return n + V * 2 * H + V;
}

void free_ws(wk_ctc* c) {   // (wk_ctc_forward's workspace; the transcribe buffers go in free_all)
  void* ps[] = {c->x0, c->gi, c->y0, c->y1, c->logits, c->best, c->best2, c->x0h, c->y0h, c->y1h, c->logits16};
  for (void* q : ps) (void)hipFree(q);
  c->x0 = c->gi = c->y0 = c->y1 = c->logits = nullptr;
  c->x0h = c->y0h = c->y1h = c->logits16 = nullptr;
  c->best = c->best2 = nullptr;
  c->ws_rows = 0;
}

// Fold the recorded stage events into the per-stage sums (synchronises on them).
hipError_t fold_events(wk_ctc* c) {
  hipError_t err = hipSuccess;
  for (int i = 0; i < c->n_ev; ++i) {
    float ms = 0.0f;
    hipError_t e = hipEventSynchronize(c->ev[i].b);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->ev[i].a, c->ev[i].b);
    if (e == hipSuccess) {
      c->stage_ms[c->ev[i].stage] += ms;
      c->stage_n[c->ev[i].stage] += 1;
    } else if (err == hipSuccess) {
      err = e;
    }
    (void)hipEventDestroy(c->ev[i].a);
    (void)hipEventDestroy(c->ev[i].b);
  }
  c->n_ev = 0;
  return err;
}

// Stage bracket: records an event pair around `launch` when profiling is on.
template <typename F>
wk_status timed(wk_ctc* c, int stage, hipStream_t st, F launch) {
  if (!c->prof) return launch();
  if (c->n_ev == 64 && fold_events(c) != hipSuccess) return fail(WK_ERR_HIP, "wk_ctc stage timing");
  auto& e = c->ev[c->n_ev];
  if (hipEventCreate(&e.a) != hipSuccess) return fail(WK_ERR_HIP, "hipEventCreate");
  if (hipEventCreate(&e.b) != hipSuccess) {
    (void)hipEventDestroy(e.a);
    return fail(WK_ERR_HIP, "hipEventCreate");
  }
  e.stage = stage;
  ++c->n_ev;
  (void)hipEventRecord(e.a, st);
  const wk_status s = launch();
  (void)hipEventRecord(e.b, st);
  return s;
}

void free_all(wk_ctc* c) {
  (void)fold_events(c);
  free_ws(c);
  void* ts[] = {c->tr_feats, c->tr_part, c->tr_zs};
  for (void* q : ts) (void)hipFree(q);
  void* ps[] = {c->enc_w, c->enc_b, c->ln_g, c->ln_b, c->wih[0], c->wih[1], c->bih[0], c->bih[1], c->bhh[0],
                c->bhh[1], c->whh_pk[0], c->whh_pk[1], c->out_w, c->out_b, c->zero_b, c->wih16[0], c->wih16[1],
                c->out_w16, c->fft_win, c->fft_tw, c->whh16_pk[0], c->whh16_pk[1],
                c->wih16x_pk[0], c->wih16x_pk[1], c->whh16x_pk[0], c->whh16x_pk[1], c->melw, c->melws};
  for (void* q : ps) (void)hipFree(q);
}

template <typename T>
hipError_t upload(T** d, const T* h, size_t n) {
  hipError_t e = hipMalloc(d, sizeof(T) * n);
  if (e != hipSuccess) return e;
  return hipMemcpy(*d, h, sizeof(T) * n, hipMemcpyHostToDevice);
}

hipError_t upload_f16(__half** d, const float* h, size_t n) {
  std::vector<__half> t(n);
  for (size_t i = 0; i < n; ++i) t[i] = __float2half(h[i]);
  return upload(d, t.data(), n);
}

}  // namespace

// ---------------------------------------------------------------------------
// Plain GEMM C[M][N] = A[M][K] W[N][K]^T, fp32 accumulate, for the paths that
// materialise a [rows][N] tensor: the fp32 parity mode's input projections (N =
// 768) and output layer (N = V, ctc.py:146), and the fp16 A/B path's
// projections (WAKEWORD_CTC_GEMM=1).  fp32 operands on v_mfma_f32_16x16x4_f32
// (exact fp32 products and sums), fp16 on v_mfma_f32_16x16x16_f16.
// Block tile 128 rows x 128 columns, 4 waves of 64 x 64 (4 x 4 accumulators
// of 16 x 16).  K goes in chunks of 64 bytes per row (16 fp32 / 32 fp16): the
// block stages a chunk of its A rows and W rows in LDS (double-buffered, one
// barrier per chunk; the next chunk's global loads are in flight during this
// chunk's MFMAs), and a lane reads its fragments as 16-byte pieces: lane
// group q = lane >> 4 holds piece q of a row (E = 4 fp32 / 8 fp16 k), and MFMA
// step s takes element s (fp32) or elements 4s .. 4s + 3 (fp16) of it -- the
// same k permutation in A and W, so the chunk is complete after its steps.
// Rows past M and columns past N read a clamped row and are never stored.
// K is a multiple of the chunk.  LDS rows are 64 bytes with their four 16-byte
// pieces swizzled (gemm_piece): the fragment reads are bank-conflict-free.
// ---------------------------------------------------------------------------
namespace {

constexpr int kGemmBM = 128, kGemmBN = 128, kGemmPitch = 4;   // LDS row pitch in 16-byte pieces (swizzled, below)
// piece q of LDS row n sits at q ^ ((n >> 1) & 3): each 16-lane group of a
// fragment ds_read_b128 (rows li, pieces q) then covers all 64 banks (brute-forced).
__device__ __forceinline__ int gemm_piece(int n, int q) { return q ^ ((n >> 1) & 3); }

// Element-wise fp16 <-> fp32 copy (the WAKEWORD_CTC_MIX attribution paths).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void ctc_convert_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if constexpr (std::is_same<TO, __half>::value) out[i] = __float2half((float)in[i]);
    else out[i] = (float)in[i];
  }
}

// ARGMAX (fp32 decode, no log-probs): C is not written; each row's first
// argmax of (A W^T)[row] + bias over the block's columns goes to keys[row] by a
// 64-bit atomicMax on {order-preserving float bits, ~column} (the larger logit
// wins, an equal logit keeps the smaller column, as torch.argmax), so the
// [rows][V] fp32 logits never exist (19.7 GB written and read back at config
// 5 before).  keys must be zeroed first; ctc_keys_to_best_kernel decodes them.
__device__ __forceinline__ unsigned long long argmax_key(float v, int col) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)col);
}

__global__ __launch_bounds__(256) void ctc_keys_to_best_kernel(const unsigned long long* __restrict__ keys,
                                                               int64_t rows, int* __restrict__ best) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < rows) best[r] = (int)(0xFFFFFFFFu - (unsigned)(keys[r] & 0xFFFFFFFFull));
}

template <typename TI, typename TO, bool ARGMAX = false>
__global__ __launch_bounds__(256) void ctc_gemm_nt_kernel(const TI* __restrict__ A, const TI* __restrict__ W,
                                                          TO* __restrict__ C, int64_t M, int N, int K,
                                                          const float* __restrict__ bias = nullptr,
                                                          unsigned long long* __restrict__ keys = nullptr) {
  constexpr bool F16 = std::is_same<TI, __half>::value;
  constexpr int E = 16 / (int)sizeof(TI), KC = 4 * E;
  __shared__ uint4 As[2][kGemmBM * kGemmPitch], Ws[2][kGemmBN * kGemmPitch];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, q = lane >> 4, wm = wave >> 1, wn = wave & 1;
  const int64_t r0 = (int64_t)blockIdx.x * kGemmBM;
  const int c0 = blockIdx.y * kGemmBN;
  // cooperative staging: thread tid moves pieces p = tid and tid + 256 of each
  // operand (row p >> 2, piece p & 3 of the chunk)
  const uint4* ga[2];
  const uint4* gw[2];
  int so[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int p = tid + 256 * h, row = p >> 2, pc = p & 3;
    const int64_t ra = r0 + row < M ? r0 + row : M - 1;
    const int cw = c0 + row < N ? c0 + row : N - 1;
    ga[h] = reinterpret_cast<const uint4*>(A + ra * K) + pc;
    gw[h] = reinterpret_cast<const uint4*>(W + (int64_t)cw * K) + pc;
    so[h] = row * kGemmPitch + gemm_piece(row, pc);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int nch = K / KC;
  uint4 pa[2], pw[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    pa[h] = ga[h][0];
    pw[h] = gw[h][0];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    As[0][so[h]] = pa[h];
    Ws[0][so[h]] = pw[h];
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    {   // next chunk's pieces (the last chunk re-loads itself: unconditional loads keep pa / pw in
        // registers -- under a branch the compiler staged them through scratch and waited at once)
      const int cn = c + 1 < nch ? c + 1 : c;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        pa[h] = ga[h][4 * cn];
        pw[h] = gw[h][4 * cn];
      }
    }
    uint4 a[4], w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = As[buf][(64 * wm + 16 * i + li) * kGemmPitch + gemm_piece(li, q)];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = Ws[buf][(64 * wn + 16 * j + li) * kGemmPitch + gemm_piece(li, q)];
    if constexpr (F16) {
      typedef _Float16 h4v __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint2 au = st ? make_uint2(a[i].z, a[i].w) : make_uint2(a[i].x, a[i].y);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint2 wu = st ? make_uint2(w[j].z, w[j].w) : make_uint2(w[j].x, w[j].y);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4v, au), __builtin_bit_cast(h4v, wu),
                                                              acc[i][j], 0, 0, 0);
          }
        }
    } else {
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float av = __uint_as_float(st == 0 ? a[i].x : st == 1 ? a[i].y : st == 2 ? a[i].z : a[i].w);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float wv = __uint_as_float(st == 0 ? w[j].x : st == 1 ? w[j].y : st == 2 ? w[j].z : w[j].w);
            acc[i][j] = mfma4(av, wv, acc[i][j]);
          }
        }
    }
    if (c + 1 < nch) {   // buffer buf ^ 1 was last read in chunk c - 1, before the barrier below it
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        As[buf ^ 1][so[h]] = pa[h];
        Ws[buf ^ 1][so[h]] = pw[h];
      }
    }
    __syncthreads();
  }
  if constexpr (ARGMAX) {
    float bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + 64 * wn + 16 * j + li;
      bj[j] = col < N ? bias[col] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float bv = -INFINITY;
        int bc = 0x7FFFFFFF;
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // this lane's columns, increasing
          const int col = c0 + 64 * wn + 16 * j + li;
          const float v = acc[i][j][r] + bj[j];
          if (col < N && v > bv) { bv = v; bc = col; }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {   // the 16 column lanes of the row: first maximum
          const float ov = __shfl_xor(bv, o, 64);
          const int oc = __shfl_xor(bc, o, 64);
          if (ov > bv || (ov == bv && oc < bc)) { bv = ov; bc = oc; }
        }
        const int64_t row = r0 + 64 * wm + 16 * i + 4 * q + r;
        if (li == 0 && row < M && bc < N) atomicMax(keys + row, argmax_key(bv, bc));
      }
    return;
  }
  // D of a 16 x 16 tile: lane holds rows 4q .. 4q + 3, column li
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + 64 * wn + 16 * j + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = r0 + 64 * wm + 16 * i + 4 * q + r;
        if (row < M && col < N) {
          if constexpr (std::is_same<TO, __half>::value) C[row * N + col] = __float2half(acc[i][j][r]);
          else C[row * N + col] = acc[i][j][r];
        }
      }
    }
}

// Row-major C[M][N] (fp32, or fp16 with c16) = A[M][K] * W[N][K]^T with A, W
// fp32 or fp16 (fp32 accumulate), on `st`.
wk_status gemm_nt(hipStream_t st, int64_t M, int64_t N, int64_t K, const void* A, const void* W, void* C, bool f16,
                  bool c16 = false) {
  if (M <= 0) return WK_OK;
  if (K % (f16 ? 32 : 16) != 0 || N > INT32_MAX || K > INT32_MAX || (M + kGemmBM - 1) / kGemmBM > INT32_MAX)
    return fail(WK_ERR_UNSUPPORTED, "ctc gemm: K must be a multiple of 16 (fp32) / 32 (fp16)");
  const dim3 g((unsigned)((M + kGemmBM - 1) / kGemmBM), (unsigned)((N + kGemmBN - 1) / kGemmBN));
  if (f16 && c16)
    hipLaunchKernelGGL((ctc_gemm_nt_kernel<__half, __half>), g, dim3(256), 0, st, (const __half*)A, (const __half*)W,
                       (__half*)C, M, (int)N, (int)K);
  else if (f16)
    hipLaunchKernelGGL((ctc_gemm_nt_kernel<__half, float>), g, dim3(256), 0, st, (const __half*)A, (const __half*)W,
                       (float*)C, M, (int)N, (int)K);
  else
    hipLaunchKernelGGL((ctc_gemm_nt_kernel<float, float>), g, dim3(256), 0, st, (const float*)A, (const float*)W,
                       (float*)C, M, (int)N, (int)K);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WK_OK : hip_fail(e, "ctc gemm launch");
}

// fp32 best[row] = first argmax of A[M][K] W[N][K]^T + bias (K % 16 == 0),
// with keys [M] as scratch: zero, GEMM + atomic argmax, decode.
wk_status gemm_argmax(hipStream_t st, int64_t M, int64_t N, int64_t K, const float* A, const float* W, const float* bias,
                      unsigned long long* keys, int* best) {
  if (M <= 0) return WK_OK;
  if (K % 16 != 0 || N > INT32_MAX || K > INT32_MAX || (M + kGemmBM - 1) / kGemmBM > INT32_MAX)
    return fail(WK_ERR_UNSUPPORTED, "ctc gemm: K must be a multiple of 16");
  hipError_t e = hipMemsetAsync(keys, 0, sizeof(unsigned long long) * M, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
  const dim3 g((unsigned)((M + kGemmBM - 1) / kGemmBM), (unsigned)((N + kGemmBN - 1) / kGemmBN));
  hipLaunchKernelGGL((ctc_gemm_nt_kernel<float, float, true>), g, dim3(256), 0, st, A, W, (float*)nullptr, M, (int)N,
                     (int)K, bias, keys);
  hipLaunchKernelGGL(ctc_keys_to_best_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, keys, M, best);
  e = hipGetLastError();
  return e == hipSuccess ? WK_OK : hip_fail(e, "ctc gemm-argmax launch");
}

}  // namespace

extern "C" {

int64_t wk_ctc_num_weights(const wk_ctc_config* cfg) { return cfg ? ctc_num_weights(cfg) : -1; }

wk_status wk_ctc_create(const wk_ctc_config* cfg, const float* w, wk_ctc** out) {
  if (!cfg || !w || !out) return invalid("wk_ctc_create: null argument");
  if (cfg->hidden != kH || cfg->layers != 2 || cfg->n_mels != kMels || cfg->vocab < 2)
    return fail(WK_ERR_UNSUPPORTED, "wk_ctc_create: this build implements hidden=128, layers=2, n_mels=80, vocab>=2");
  if (cfg->precision != 0 && cfg->precision != 1) return invalid("wk_ctc_create: precision must be 0 (fp32) or 1 (fp16)");
  *out = nullptr;
  return on_device(cfg->device, [&]() -> wk_status {
    wk_ctc* c = (wk_ctc*)calloc(1, sizeof(wk_ctc));
    if (!c) return WK_ERR_NO_MEMORY;
    c->cfg = *cfg;
    c->f16 = cfg->precision == 1;
    const char* gg = getenv("WAKEWORD_CTC_GEMM");
    c->gru_gemm = gg && gg[0] == '1';
    const char* mx = getenv("WAKEWORD_CTC_MIX");
    c->mix = mx ? (strcmp(mx, "out32") == 0 ? 1 : strcmp(mx, "out16") == 0 ? 2 : 0) : 0;
    const char* rs = getenv("WAKEWORD_CTC_RESCORE");
    c->rescore = !(rs && rs[0] == '0');
    hipDeviceProp_t prop;
    c->n_cu = hipGetDeviceProperties(&prop, cfg->device) == hipSuccess ? prop.multiProcessorCount : 256;
    const int H = kH, V = cfg->vocab;
    const float* p = w;
    auto take = [&](size_t n) { const float* q = p; p += n; return q; };
    const float* enc_w = take((size_t)H * kMels);
    const float* enc_b = take(H);
    const float* ln_g = take(H);
    const float* ln_b = take(H);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = upload(&c->enc_w, enc_w, (size_t)H * kMels);
    if (e == hipSuccess) e = upload(&c->enc_b, enc_b, H);
    if (e == hipSuccess) e = upload(&c->ln_g, ln_g, H);
    if (e == hipSuccess) e = upload(&c->ln_b, ln_b, H);
    for (int l = 0; l < 2 && e == hipSuccess; ++l) {
      const int din = l == 0 ? H : 2 * H;
      std::vector<float> wih(6 * (size_t)H * din), whh_all(6 * (size_t)H * H), bih(6 * H), bhh(6 * H), pk(2 * 24 * 32 * 64), pk16(2 * 24 * 8 * 64 * 4);
      for (int d = 0; d < 2; ++d) {
        const float* wi = take(3 * (size_t)H * din);
        const float* wh = take(3 * (size_t)H * H);
        memcpy(&whh_all[(size_t)d * 3 * H * H], wh, sizeof(float) * 3 * H * H);
        const float* bi = take(3 * H);
        const float* bh = take(3 * H);
        memcpy(&wih[(size_t)d * 3 * H * din], wi, sizeof(float) * 3 * H * din);
        memcpy(&bih[d * 3 * H], bi, sizeof(float) * 3 * H);
        memcpy(&bhh[d * 3 * H], bh, sizeof(float) * 3 * H);
        for (int tl = 0; tl < 24; ++tl)
          for (int s = 0; s < 32; ++s)
            for (int ln = 0; ln < 64; ++ln)
              pk[(((size_t)d * 24 + tl) * 32 + s) * 64 + ln] = wh[(size_t)(16 * tl + (ln & 15)) * H + 4 * s + (ln >> 4)];
        for (int tl = 0; tl < 24; ++tl)
          for (int s = 0; s < 8; ++s)
            for (int ln = 0; ln < 64; ++ln)
              for (int j = 0; j < 4; ++j)
                pk16[((((size_t)d * 24 + tl) * 8 + s) * 64 + ln) * 4 + j] =
                    wh[(size_t)(16 * tl + (ln & 15)) * H + 16 * s + 4 * (ln >> 4) + j];
      }
      e = upload(&c->wih[l], wih.data(), wih.size());
      if (e == hipSuccess && c->f16) e = upload_f16(&c->wih16[l], wih.data(), wih.size());
      if (e == hipSuccess && c->f16) {   // W_ih as 16x16x32 A fragments: [dir][gate][wave][ks][lane][8]
        // scaled for the fused kernel's exp2 gates: r, z rows by -log2(e), n rows by 2 log2(e)
        const double gsc[3] = {-1.4426950408889634, -1.4426950408889634, 2.8853900817779268};
        const int kx = din / 32;
        std::vector<float> px((size_t)2 * 3 * 8 * kx * 64 * 8);
        size_t o = 0;
        for (int d = 0; d < 2; ++d)
          for (int g = 0; g < 3; ++g)
            for (int w = 0; w < 8; ++w)
              for (int ks = 0; ks < kx; ++ks)
                for (int ln = 0; ln < 64; ++ln)
                  for (int j = 0; j < 8; ++j)
                    px[o++] = gsc[g] * wih[((size_t)d * 3 * H + g * H + 16 * w + (ln & 15)) * din + 32 * ks + 8 * (ln >> 4) + j];
        e = upload_f16(&c->wih16x_pk[l], px.data(), px.size());
        std::vector<float> ph((size_t)2 * 3 * 8 * 4 * 64 * 8);   // W_hh the same way (k = H): [dir][gate][wave][ks][lane][8]
        o = 0;
        for (int d = 0; d < 2; ++d)
          for (int g = 0; g < 3; ++g)
            for (int w = 0; w < 8; ++w)
              for (int ks = 0; ks < 4; ++ks)
                for (int ln = 0; ln < 64; ++ln)
                  for (int j = 0; j < 8; ++j)
                    ph[o++] = gsc[g] * whh_all[((size_t)d * 3 * H + g * H + 16 * w + (ln & 15)) * H + 32 * ks + 8 * (ln >> 4) + j];
        if (e == hipSuccess) e = upload_f16(&c->whh16x_pk[l], ph.data(), ph.size());
      }
      if (e == hipSuccess) e = upload(&c->bih[l], bih.data(), bih.size());
      if (e == hipSuccess) e = upload(&c->bhh[l], bhh.data(), bhh.size());
      if (e == hipSuccess) e = upload(&c->whh_pk[l], pk.data(), pk.size());
      if (e == hipSuccess && c->f16) e = upload_f16(&c->whh16_pk[l], pk16.data(), pk16.size());
    }
    const float* ow = take((size_t)V * 2 * H);
    if (e == hipSuccess) e = upload(&c->out_w, ow, (size_t)V * 2 * H);
    if (e == hipSuccess && (c->f16 || c->mix == 2)) e = upload_f16(&c->out_w16, ow, (size_t)V * 2 * H);
    if (e == hipSuccess) e = upload(&c->out_b, take(V), V);
    if (e == hipSuccess) {
      const std::vector<float> z((size_t)V, 0.0f);
      e = upload(&c->zero_b, z.data(), (size_t)V);
    }
    // FFT tables: periodic Hann(400) and the four-step twiddles W400^(n2 k1), in double -> fp32
    {
      std::vector<float> wnd(kNfft), tw(2 * 400);
      for (int n = 0; n < kNfft; ++n) wnd[n] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * n / kNfft));
      for (int k1 = 0; k1 < 20; ++k1)
        for (int n2 = 0; n2 < 20; ++n2) {
          const double ang = -2.0 * M_PI * (double)(n2 * k1) / kNfft;
          tw[2 * (k1 * 20 + n2)] = (float)cos(ang);
          tw[2 * (k1 * 20 + n2) + 1] = (float)sin(ang);
        }
      if (e == hipSuccess) e = upload(&c->fft_win, wnd.data(), wnd.size());
      if (e == hipSuccess) e = upload(&c->fft_tw, tw.data(), tw.size());
    }
    // mel filterbank as CSR (per filter: first bin, count, weights)
    std::vector<float> fb;
    mel_fbank(fb);
    std::vector<int> st(kMels), ln(kMels), off(kMels);
    std::vector<float> wv;
    for (int m = 0; m < kMels; ++m) {
      int a0 = -1, z = -1;
      for (int k = 0; k < kBins; ++k)
        if (fb[(size_t)k * kMels + m] != 0.0f) { if (a0 < 0) a0 = k; z = k; }
      if (a0 < 0) a0 = z = 0;
      st[m] = a0;
      ln[m] = z - a0 + 1;
      off[m] = (int)wv.size();
      for (int k = a0; k <= z; ++k) wv.push_back(fb[(size_t)k * kMels + m]);
    }
    {   // straight-line windows of ctc_logmel_fft2_kernel (see there)
      std::vector<float> mw((size_t)64 * (kMelW1 + kMelW2), 0.0f);
      std::vector<int> ws(128, 0);
      std::vector<int> cut(128, kBins);   // (second set) a lane takes filter bins in [ws, cut)
      bool fits = kMels == 80;
      for (int m = 0; m < 64 && fits; ++m) fits = ln[m] <= kMelW1;
      for (int m = 64; m < kMels && fits; ++m) fits = ln[m] <= 2 * kMelW2;
      if (fits) {
        pick_mel_windows(st, ln, ws, cut);
        for (int m = 0; m < 64; ++m)
          for (int j = 0; j < kMelW1; ++j) {
            const int k = ws[m] + j;
            const bool mine = k >= st[m] && k < st[m] + ln[m];
            mw[(size_t)m * kMelW1 + j] = mine ? 0.25f * fb[(size_t)k * kMels + m] : 0.0f;
          }
        for (int l = 0; l < 32; ++l) {
          const int m = 64 + l / 2;
          for (int j = 0; j < kMelW2; ++j) {
            const int k = ws[64 + l] + j;
            const bool mine = k >= st[m] && k < st[m] + ln[m] && k < cut[64 + l] && ((l & 1) == 0 || k >= cut[64 + l - 1]);
            mw[(size_t)64 * kMelW1 + (size_t)l * kMelW2 + j] = mine ? 0.25f * fb[(size_t)k * kMels + m] : 0.0f;
          }
        }
        // every filter tap lands in exactly one window
        for (int m = 0; m < kMels && fits; ++m) {
          int taps = 0;
          if (m < 64) {
            for (int j = 0; j < kMelW1; ++j) taps += mw[(size_t)m * kMelW1 + j] != 0.0f;
          } else {
            for (int h = 0; h < 2; ++h)
              for (int j = 0; j < kMelW2; ++j) taps += mw[(size_t)64 * kMelW1 + (size_t)(2 * (m - 64) + h) * kMelW2 + j] != 0.0f;
          }
          int nz = 0;
          for (int k = st[m]; k < st[m] + ln[m]; ++k) nz += fb[(size_t)k * kMels + m] != 0.0f;
          fits = taps == nz;
        }
      }
      if (e == hipSuccess && !fits) e = hipErrorInvalidValue;
      if (e == hipSuccess) e = upload(&c->melw, mw.data(), mw.size());
      if (e == hipSuccess) e = upload(&c->melws, ws.data(), ws.size());
    }
    if (e != hipSuccess) {
      free_all(c);
      free(c);
      return e == hipErrorOutOfMemory ? WK_ERR_NO_MEMORY : hip_fail(e, "wk_ctc_create");
    }
    *out = c;
    return WK_OK;
  });
}

wk_status wk_ctc_destroy(wk_ctc* c) {
  if (!c) return WK_OK;
  return on_device(c->cfg.device, [&]() -> wk_status {
    (void)hipDeviceSynchronize();
    free_all(c);
    free(c);
    return WK_OK;
  });
}

namespace {
// The log-mel kernel's launch: at most one 12-wave workgroup per CU, each wave
// a contiguous range of R passes; MS statistics slots per wave (the most
// utterances 6 R rows can touch), slots = waves x MS.
struct LogmelLayout {
  unsigned grid;
  int64_t R;
  int MS;
  int64_t slots;
};
LogmelLayout logmel_layout(const wk_ctc* c, int64_t rows, int T) {
  LogmelLayout L;
  const int64_t passes = (rows + 2 * kF2Pairs - 1) / (2 * kF2Pairs);
  const int64_t blocks = (passes + kF2Waves - 1) / kF2Waves;
  L.grid = (unsigned)(blocks < c->n_cu ? blocks : c->n_cu);
  const int64_t nw = (int64_t)L.grid * kF2Waves;
  L.R = (passes + nw - 1) / nw;
  L.MS = (int)((2 * kF2Pairs * L.R - 1) / T + 2);
  L.slots = nw * L.MS;
  return L;
}

// wk_ctc_features; with `part` (wk_ctc_transcribe, T >= 6) the features stay
// raw and the z-score's statistics go to zs instead of being applied in place.
wk_status ctc_features(wk_ctc* c, const float* d_audio, int64_t batch, int32_t n_valid, int32_t n_samples,
                       int64_t stride, float* d_feats, void* stream, float2* part, float2* zs) {
  if (!c || batch < 0 || (batch > 0 && (!d_audio || !d_feats)) || n_samples < kNfft / 2 + 1 || n_valid < 0 ||
      (batch > 1 && stride < (n_valid < n_samples ? n_valid : n_samples)))
    return invalid("wk_ctc_features: bad arguments (n_samples must exceed 200 for the reflect pad)");
  if (batch == 0) return WK_OK;
  const int T = 1 + n_samples / kHop;
  const int64_t rows = batch * (int64_t)T;
  if (rows > INT32_MAX) return invalid("wk_ctc_features: batch x frames exceeds 2^31 rows");
  return on_device(c->cfg.device, [&]() -> wk_status {
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    const int nv = n_valid < n_samples ? n_valid : n_samples;
    // n_valid == 0: every sample is padding; the kernel's (masked) loads then
    // read a device table instead of a possibly empty audio buffer
    const float* au = nv > 0 ? d_audio : c->fft_win;
    const LogmelLayout lay = logmel_layout(c, rows, T);
    if (part && (size_t)lay.slots > c->tr_slots) return invalid("wk_ctc_transcribe: statistics workspace too small");
    wk_status s = timed(c, WK_CTC_STAGE_LOGMEL, st, [&]() -> wk_status {
      const dim3 lg2(lay.grid);
      if (part)
        hipLaunchKernelGGL(ctc_logmel_fft2_kernel<true>, lg2, dim3(kF2Waves * 64), 0, st, au, nv > 0 ? stride : (int64_t)0,
                           nv, n_samples, T, rows, c->fft_win, c->fft_tw, c->melw, c->melws, d_feats, lay.R, lay.MS, part);
      else
        hipLaunchKernelGGL(ctc_logmel_fft2_kernel<false>, lg2, dim3(kF2Waves * 64), 0, st, au, nv > 0 ? stride : (int64_t)0,
                           nv, n_samples, T, rows, c->fft_win, c->fft_tw, c->melw, c->melws, d_feats, lay.R, lay.MS,
                           (float2*)nullptr);
      return WK_OK;
    });
    if (s == WK_OK)
      s = timed(c, WK_CTC_STAGE_ZSCORE, st, [&]() -> wk_status {
        if (part)
          hipLaunchKernelGGL(ctc_zstats_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, part, d_feats, batch, T,
                             lay.R, lay.MS, zs);
        else
          hipLaunchKernelGGL(ctc_zscore_kernel, dim3((unsigned)batch), dim3(1024), 0, st, d_feats, (int64_t)T * kMels);
        return WK_OK;
      });
    if (s != WK_OK) return s;
    e = hipGetLastError();
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_features launch");
  });
}

// wk_ctc_forward; with zs (wk_ctc_transcribe, fp16 mode) the encoder z-scores
// the raw feature rows as it loads them.
wk_status ctc_forward(wk_ctc* c, const float* d_feats, int64_t batch, int32_t T, float* d_log_probs, int32_t* d_tokens,
                      int32_t* d_lengths, void* stream, const float2* zs) {
  if (!c || batch < 0 || T < 1 || (batch > 0 && (!d_feats || !d_tokens || !d_lengths)))
    return invalid("wk_ctc_forward: bad arguments");
  if (batch == 0) return WK_OK;
  const int V = c->cfg.vocab, H = kH;
  const int64_t rows = batch * (int64_t)T;
  if (rows > INT32_MAX) return invalid("wk_ctc_forward: batch x frames exceeds 2^31 rows");
  const bool f16 = c->f16;
  // fp16 encoder: 32-bit buffer offsets over the [rows][80] fp32 features
  if (f16 && rows * kMels * 4 >= (int64_t)0x7FFFFF00) return invalid("wk_ctc_forward: fp16 mode takes < 6.7 M rows per call");
  return on_device(c->cfg.device, [&]() -> wk_status {
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if ((size_t)rows > c->ws_rows) {   // workspace grows on first use of a larger batch (then reused)
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
      free_ws(c);
      if ((!f16 && (e = hipMalloc(&c->x0, sizeof(float) * rows * H)) != hipSuccess) ||
          ((!f16 || c->gru_gemm) && (e = hipMalloc(&c->gi, sizeof(float) * rows * 6 * H)) != hipSuccess) ||
          (!f16 && (e = hipMalloc(&c->y0, sizeof(float) * rows * 2 * H)) != hipSuccess) ||
          ((!f16 || c->mix == 1) && (e = hipMalloc(&c->y1, sizeof(float) * rows * 2 * H)) != hipSuccess) ||
          ((!f16 || c->mix == 1) && (e = hipMalloc(&c->logits, sizeof(float) * rows * V)) != hipSuccess) ||
          (!f16 && c->mix == 2 && (e = hipMalloc(&c->y1h, sizeof(__half) * rows * 2 * H)) != hipSuccess) ||
          (e = hipMalloc(&c->best, sizeof(int) * rows)) != hipSuccess ||
          (e = hipMalloc(&c->best2, sizeof(int) * rows)) != hipSuccess ||
          (f16 && (e = hipMalloc(&c->x0h, sizeof(__half) * rows * H)) != hipSuccess) ||
          (f16 && (e = hipMalloc(&c->y0h, sizeof(__half) * rows * 2 * H)) != hipSuccess) ||
          (f16 && (e = hipMalloc(&c->y1h, sizeof(__half) * rows * 2 * H)) != hipSuccess) ||
          (f16 && (e = hipMalloc(&c->logits16, sizeof(__half) * rows * V)) != hipSuccess)) {
        free_ws(c);
        return e == hipErrorOutOfMemory ? WK_ERR_NO_MEMORY : hip_fail(e, "wk_ctc_forward workspace");
      }
      c->ws_rows = rows;
    }
    c->last_batch = batch;
    c->last_T = T;
    // two 4-wave workgroups per CU: 3 or more measured slower (0.187 -> 0.21-0.22 ms, profiles/r05g_ctc_ab.txt)
    const int enc_grid = (int)((rows + 63) / 64 < 2 * c->n_cu ? (rows + 63) / 64 : 2 * c->n_cu);
    wk_status s = timed(c, WK_CTC_STAGE_ENCODER, st, [&]() -> wk_status {
      if (f16 && zs)
        hipLaunchKernelGGL(ctc_encoder16_kernel<true>, dim3(enc_grid), dim3(256), 0, st, d_feats, rows, c->enc_w,
                           c->enc_b, c->ln_g, c->ln_b, (int)batch, T, zs, c->x0h);
      else if (f16)
        hipLaunchKernelGGL(ctc_encoder16_kernel<false>, dim3(enc_grid), dim3(256), 0, st, d_feats, rows, c->enc_w,
                           c->enc_b, c->ln_g, c->ln_b, (int)batch, T, (const float2*)nullptr,
                           c->x0h);   // fp16 path: time-major rows from here on
      else
        hipLaunchKernelGGL(ctc_encoder_kernel<float>, dim3(enc_grid), dim3(256), 0, st, d_feats, rows, c->enc_w,
                           c->enc_b, c->ln_g, c->ln_b, c->x0);
      return WK_OK;
    });
    if (s != WK_OK) return s;
    const float* in = c->x0;
    const __half* in16 = c->x0h;
    float* ys[2] = {c->y0, c->y1};
    __half* ys16[2] = {c->y0h, c->y1h};
    for (int l = 0; l < 2; ++l) {
      const int din = l == 0 ? H : 2 * H;
      if (f16 && !c->gru_gemm) {   // projection fused into the recurrence: no GEMM, no gate-input tensor
        const dim3 gx((unsigned)((batch + kGxRows - 1) / kGxRows), 2);
        s = timed(c, WK_CTC_STAGE_GRU0 + 2 * l, st, [&]() -> wk_status {
          if (l == 0)
            hipLaunchKernelGGL(ctc_gru16x_kernel<128>, gx, dim3(kGxThreads), 0, st, in16, (const h8x*)c->wih16x_pk[0],
                               (const h8x*)c->whh16x_pk[0], c->bih[0], c->bhh[0], batch, T, ys16[0]);
          else
            hipLaunchKernelGGL(ctc_gru16x_kernel<256>, gx, dim3(kGxThreads), 0, st, in16, (const h8x*)c->wih16x_pk[1],
                               (const h8x*)c->whh16x_pk[1], c->bih[1], c->bhh[1], batch, T, ys16[1]);
          return WK_OK;
        });
        if (s != WK_OK) return s;
        in16 = ys16[l];
        continue;
      }
      s = timed(c, WK_CTC_STAGE_PROJ0 + 2 * l, st, [&]() -> wk_status {
        return f16 ? gemm_nt(st, rows, 6 * H, din, in16, c->wih16[l], c->gi, true, true)   // fp16 gates
                   : gemm_nt(st, rows, 6 * H, din, in, c->wih[l], c->gi, false);
      });
      if (s != WK_OK) return s;
      const dim3 gg((unsigned)((batch + kGruBatch - 1) / kGruBatch), 2);
      s = timed(c, WK_CTC_STAGE_GRU0 + 2 * l, st, [&]() -> wk_status {
        if (f16)
          hipLaunchKernelGGL(ctc_gru16_kernel, gg, dim3(kGru16Threads), 0, st, (const __half*)c->gi,
                             (const h4*)c->whh16_pk[l], c->bih[l], c->bhh[l], batch, T, ys16[l]);
        else
          hipLaunchKernelGGL(ctc_gru_kernel, gg, dim3(kGruThreads), 0, st, c->gi, c->whh_pk[l], c->bih[l], c->bhh[l],
                             batch, T, ys[l]);
        return WK_OK;
      });
      if (s != WK_OK) return s;
      in = ys[l];
      in16 = ys16[l];
    }
    if (f16 && c->mix == 1) {   // attribution: the fp16 path's y1, widened, through the fp32 output layer
      if (d_log_probs) return fail(WK_ERR_UNSUPPORTED, "WAKEWORD_CTC_MIX=out32 decodes only (no log-probs)");
      hipLaunchKernelGGL((ctc_convert_kernel<__half, float>), dim3(2 * c->n_cu), dim3(256), 0, st, c->y1h, c->y1,
                         rows * 2 * H);
      in = c->y1;
    } else if (!f16 && c->mix == 2) {   // attribution: the fp32 path's y1, rounded, through the fp16 output kernel
      hipLaunchKernelGGL((ctc_convert_kernel<float, __half>), dim3(2 * c->n_cu), dim3(256), 0, st, c->y1, c->y1h,
                         rows * 2 * H);
      const dim3 og((unsigned)((rows + out_rows(false) - 1) / out_rows(false)));
      const bool keyed = V <= 16 * 256;
      hipLaunchKernelGGL((keyed ? ctc_out_argmax16_kernel<false, true> : ctc_out_argmax16_kernel<false, false>), og,
                         dim3(kOutWaves * 64), 0, st, c->y1h, c->out_w16, c->out_b, rows, V, (__half*)nullptr, c->best,
                         c->best2);
      if (keyed && c->rescore)
        hipLaunchKernelGGL(ctc_rescore_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, c->y1h, c->out_w,
                           c->out_b, rows, c->best, c->best2);
      hipLaunchKernelGGL(ctc_greedy_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, c->best, batch, T,
                         d_tokens, d_lengths, 0);
      e = hipGetLastError();
      return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_forward launch");
    }
    if (f16 && c->mix != 1) {
      // fused output layer + argmax; fp16 logits are written only for log_softmax
      const dim3 og((unsigned)((rows + out_rows(d_log_probs != nullptr) - 1) / out_rows(d_log_probs != nullptr)));
      s = timed(c, WK_CTC_STAGE_OUTPUT, st, [&]() -> wk_status {
        const bool keyed = V <= 16 * 256;   // the tag holds kOutCF tile + cf in 8 bits
        if (d_log_probs) {
          hipLaunchKernelGGL((keyed ? ctc_out_argmax16_kernel<true, true> : ctc_out_argmax16_kernel<true, false>), og,
                             dim3(kOutWaves * 64), 0, st, c->y1h, c->out_w16, c->out_b, rows, V, c->logits16, c->best,
                             c->best2);
          hipLaunchKernelGGL(ctc_argmax_kernel<__half>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st,
                             c->logits16, c->zero_b, rows, V, d_log_probs, (int*)nullptr, (int)batch, T);   // bias already in
        } else {
          if (keyed)   // the decode-only kernel, the fold among the MFMAs
            hipLaunchKernelGGL(ctc_out_decode16_kernel, og, dim3(kOutWaves * 64), 0, st, c->y1h, c->out_w16, c->out_b,
                               rows, V, c->best, c->best2);
          else
            hipLaunchKernelGGL((ctc_out_argmax16_kernel<false, false>), og, dim3(kOutWaves * 64), 0, st, c->y1h,
                               c->out_w16, c->out_b, rows, V, (__half*)nullptr, c->best, c->best2);
        }
        if (keyed && c->rescore)   // near-tie rows decided again in fp32 (tokens independent of log-probs: both variants)
          hipLaunchKernelGGL(ctc_rescore_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, c->y1h,
                             c->out_w, c->out_b, rows, c->best, c->best2);
        return WK_OK;
      });
      if (s == WK_OK)
        s = timed(c, WK_CTC_STAGE_DECODE, st, [&]() -> wk_status {
          hipLaunchKernelGGL(ctc_greedy_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, c->best, batch, T,
                             d_tokens, d_lengths, 1);
          return WK_OK;
        });
      if (s != WK_OK) return s;
      e = hipGetLastError();
      return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_forward launch");
    }
    const bool arg_only = !d_log_probs && V % Vec<float>::N == 0 && V / Vec<float>::N <= 64 * kArgChunks && V <= 16384;
    const unsigned ag = (unsigned)((rows + 3) / 4 < 8 * c->n_cu ? (rows + 3) / 4 : 8 * c->n_cu);
    s = timed(c, WK_CTC_STAGE_OUTPUT, st, [&]() -> wk_status {
      if (!d_log_probs)   // decode only: the argmax inside the GEMM, no [rows][V] logits (c->logits: the keys)
        return gemm_argmax(st, rows, V, 2 * H, in, c->out_w, c->out_b, reinterpret_cast<unsigned long long*>(c->logits),
                           c->best);
      wk_status g = gemm_nt(st, rows, V, 2 * H, in, c->out_w, c->logits, false);
      if (g != WK_OK) return g;
      if (arg_only)
        hipLaunchKernelGGL(ctc_argmax_only_kernel<float>, dim3(ag), dim3(256), V * sizeof(float), st, c->logits,
                           c->out_b, rows, V, c->best);
      else
        hipLaunchKernelGGL(ctc_argmax_kernel<float>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, c->logits,
                           c->out_b, rows, V, d_log_probs, c->best);
      return WK_OK;
    });
    if (s == WK_OK)
      s = timed(c, WK_CTC_STAGE_DECODE, st, [&]() -> wk_status {
        hipLaunchKernelGGL(ctc_greedy_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, c->best, batch, T,
                           d_tokens, d_lengths, f16 ? 1 : 0);   // (fp16 rows are time-major)
        return WK_OK;
      });
    if (s != WK_OK) return s;
    e = hipGetLastError();
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_forward launch");
  });
}
}  // namespace

wk_status wk_ctc_features(wk_ctc* c, const float* d_audio, int64_t batch, int32_t n_valid, int32_t n_samples,
                          int64_t stride, float* d_feats, void* stream) {
  return ctc_features(c, d_audio, batch, n_valid, n_samples, stride, d_feats, stream, nullptr, nullptr);
}

wk_status wk_ctc_forward(wk_ctc* c, const float* d_feats, int64_t batch, int32_t T, float* d_log_probs,
                         int32_t* d_tokens, int32_t* d_lengths, void* stream) {
  return ctc_forward(c, d_feats, batch, T, d_log_probs, d_tokens, d_lengths, stream, nullptr);
}

wk_status wk_ctc_transcribe(wk_ctc* c, const float* d_audio, int64_t batch, int32_t n_valid, int32_t n_samples,
                            int64_t stride, int32_t* d_tokens, int32_t* d_lengths, void* stream) {
  if (!c || batch < 0 || n_samples < kNfft / 2 + 1 || (batch > 0 && (!d_tokens || !d_lengths)))
    return invalid("wk_ctc_transcribe: bad arguments");
  if (batch == 0) return WK_OK;
  const int T = 1 + n_samples / kHop;
  const int64_t rows = batch * (int64_t)T;
  if (rows > INT32_MAX) return invalid("wk_ctc_transcribe: batch x frames exceeds 2^31 rows");
  const bool fused = c->f16 && T >= 6;   // (a log-mel pass of 6 rows then spans at most two utterances)
  return on_device(c->cfg.device, [&]() -> wk_status {
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    const int64_t slots = logmel_layout(c, rows, T).slots;
    if ((size_t)rows > c->tr_rows || (size_t)batch > c->tr_batch || (size_t)slots > c->tr_slots) {   // grows, then reused
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
      (void)hipFree(c->tr_feats);
      (void)hipFree(c->tr_part);
      (void)hipFree(c->tr_zs);
      c->tr_feats = nullptr;
      c->tr_part = nullptr;
      c->tr_zs = nullptr;
      c->tr_rows = c->tr_batch = c->tr_slots = 0;
      if ((e = hipMalloc(&c->tr_feats, sizeof(float) * rows * kMels)) != hipSuccess ||
          (e = hipMalloc(&c->tr_part, sizeof(float2) * slots)) != hipSuccess ||
          (e = hipMalloc(&c->tr_zs, sizeof(float2) * batch)) != hipSuccess)
        return e == hipErrorOutOfMemory ? WK_ERR_NO_MEMORY : hip_fail(e, "wk_ctc_transcribe workspace");
      c->tr_rows = (size_t)rows;
      c->tr_batch = (size_t)batch;
      c->tr_slots = (size_t)slots;
    }
    wk_status s = ctc_features(c, d_audio, batch, n_valid, n_samples, stride, c->tr_feats, stream,
                               fused ? c->tr_part : nullptr, fused ? c->tr_zs : nullptr);
    if (s != WK_OK) return s;
    return ctc_forward(c, c->tr_feats, batch, T, nullptr, d_tokens, d_lengths, stream, fused ? c->tr_zs : nullptr);
  });
}

wk_status wk_ctc_profile(wk_ctc* c, int32_t enable) {
  if (!c) return invalid("wk_ctc_profile: null handle");
  return on_device(c->cfg.device, [&]() -> wk_status {
    const hipError_t e = fold_events(c);
    for (int i = 0; i < WK_CTC_N_STAGES; ++i) {
      c->stage_ms[i] = 0.0;
      c->stage_n[i] = 0;
    }
    c->prof = enable ? 1 : 0;
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_profile");
  });
}

wk_status wk_ctc_stage_times(wk_ctc* c, double* ms_sum, int64_t* counts) {
  if (!c || !ms_sum || !counts) return invalid("wk_ctc_stage_times: null argument");
  return on_device(c->cfg.device, [&]() -> wk_status {
    const hipError_t e = fold_events(c);
    for (int i = 0; i < WK_CTC_N_STAGES; ++i) {
      ms_sum[i] = c->stage_ms[i];
      counts[i] = c->stage_n[i];
    }
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_stage_times");
  });
}

wk_status wk_ctc_frame_argmax(wk_ctc* c, int64_t batch, int32_t T, int32_t* d_pred, void* stream) {
  if (!c || batch < 0 || T < 1 || (batch > 0 && !d_pred)) return invalid("wk_ctc_frame_argmax: bad arguments");
  if (batch == 0) return WK_OK;
  if (batch != c->last_batch || T != c->last_T || !c->best)
    return invalid("wk_ctc_frame_argmax: batch and T must be those of the handle's last wk_ctc_forward");
  return on_device(c->cfg.device, [&]() -> wk_status {
    const int64_t rows = batch * (int64_t)T;
    hipLaunchKernelGGL(ctc_pred_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream, c->best,
                       batch, T, c->f16 ? 1 : 0, d_pred);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WK_OK : hip_fail(e, "wk_ctc_frame_argmax launch");
  });
}

}  // extern "C"


