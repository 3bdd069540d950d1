// wk_fused.hip -- the whole hot path in one persistent, warp-specialised kernel.
//
//   audio (HBM) -> MFCC front-end (VALU/LDS) -> features (LDS) -> xiaoa CNN
//   (fp32 MFMA) -> logit (HBM)
//
// One 16-wave workgroup per CU.  Waves 0-7 (front-end role) run the FFT and
// the lane-per-frame mel filterbank of wk_fe_dev.h clip after clip and write
// each clip's log-mel image [40][63] into one of two LDS buffers.  Waves 8-15
// (CNN role) take the DCT-II + CMVN from that buffer into the conv1 input
// image (one wave per clip, on the matrix cores: dct_cmvn_clip), then run the
// CNN of wk_cnn_dev.h on batches of NBF = 4 clips.  The
// roles share no s_barrier: each synchronises its own 8 waves through an LDS
// counter barrier, and the hand-off is two LDS counters (log-mel ready /
// log-mel buffer free).  Moving the DCT + CMVN to the CNN waves (which wait
// on the front-end about half the time) shortened the front-end's per-clip
// critical path by ~15 %.  The front-end is VALU + LDS bound and the CNN is
// MFMA bound; on CDNA4 the matrix and vector pipes issue concurrently from
// different waves, so the roles overlap on every SIMD (2 front-end + 2 CNN
// waves per SIMD), and features never touch HBM: per clip the kernel reads
// its 64,000 audio bytes and writes one 4-byte logit.
//
// Product builds compile this file twice.  Here: the fp32 convolutions, with
// the front-end's complex arithmetic as packed fp32 (v_pk_*_f32).  Through
// wk_fused_xdl.hip (WK_FUSED_XDL_TU): the bf16 / bf16x3 convolutions, with the
// same front-end as scalar fp32 pairs (WK_FE_SCALAR, wk_common.h).  Beside the
// bf16 MFMAs, which run on the matrix pipe, packed fp32 issues slower than
// scalar: +4.8 % bf16.  Beside the fp32 MFMAs, which share the fp32
// datapath, scalar is 2.8 % slower (profiles/r05au_*).
// Diagnostic builds (WK_FUSED_ONE_TU) keep every precision here.
#define WK_FUSED_TU   // (wk_common.h: WK_FE_SCALAR applies to the fused translation units only)
#include "wk_cnn_dev.h"
#include "wk_fe_dev.h"
#include "wk_kernels.h"

using namespace wk;

#if !(defined(WK_FUSED_XDL_TU) && WK_FUSED_ONE_TU)   // (the XDL unit is empty in diagnostic builds)
namespace {

#ifdef WK_DIAG
// Diagnostic builds only (-DWK_DIAG, tools/debug): per-wave cycle sums per phase.
__device__ unsigned long long g_wk_stamps[16][16];
#define WK_STAMP_INIT WkStamps _stamps; _stamps.init();
#define WK_STAMP(k) _stamps.hit(k)
#define WK_STAMP_FLUSH(w) do { if (lane == 0) for (int _k = 0; _k < 16; ++_k) atomicAdd(&g_wk_stamps[w][_k], _stamps.st[_k]); } while (0)
#define WK_SP_ARG , &_stamps
#else
#define WK_STAMP_INIT
#define WK_STAMP(k) do {} while (0)
#define WK_STAMP_FLUSH(w) do {} while (0)
#define WK_SP_ARG
#endif



constexpr int NBF = 4;               // clips per CNN batch
#ifndef WK_FE_WAVES
#define WK_FE_WAVES 8
#endif
#if WK_FE_WAVES != 8 && !defined(WK_DIAG)
#error "WK_FE_WAVES != 8 is a diagnostic build (front-end role alone, WAKEWORD_FUSED_EXP=1)"
#endif
constexpr int kFeWaves = WK_FE_WAVES;
constexpr int kFusedBlock = 1024;    // 8 front-end + 8 CNN waves
// LDS carve after the front-end's (wk_fe_dev.h): fixed tail, then the CNN
// images [clip][t][ci] -- fp32, or bf16 for bf16 convolutions -- overlaying
// one region.  ci pitch = 8 mod 16 elements: the 16 t-lanes of each lane
// group of a B-fragment read (ds_read_b128 fp32 / ds_read_b64 bf16) and of the
// pooled stores land on distinct banks.
constexpr int kGOff = (kFeLds + 3) & ~3;            // pooled features [128][4] (16-byte aligned carve below)
constexpr int kFcpOff = kGOff + 128 * NBF;          // classifier.0 partials [8 k-slices][4 clips][64 o]
constexpr int kFcpSize = 8 * NBF * 64;
constexpr int kL1Off = kFcpOff + kFcpSize;          // second log-mel buffer [40][64] (first: kLOff)
static_assert(kLOff % 4 == 0 && kL1Off % 4 == 0, "log-mel buffers are read with ds_read_b128");
constexpr int kCtrlOff = kL1Off + kLSize;           // control words
constexpr int kImgOff = (kCtrlOff + 16 + 3) & ~3;   // 16-byte aligned
constexpr int I0_CIP = 24, I1_CIP = 40, I2_CIP = 72;                 // elements (= 8 mod 16)
// t rows: row 0 is the left zero guard, rows 1..L hold the L frames.  No right
// guard: every layer's length L is odd, so maxpool(2) drops the one output
// that would read it; the dropped outputs' reads of rows L+1, L+2 land in the
// next clip's (or the next image's) rows, which only affects their own MFMA
// columns.  conv3 keeps 2 spare rows so its last clip stays inside the carve.
constexpr int I0_TP = 64, I1_TP = 32, I2_TP = 18;
// fp32 images (float units), read by the Winograd convolutions in row pairs:
// pitch = 4 mod 8 floats keeps the stride-2 row reads conflict-free.
constexpr int F0_CIP = 20, F1_CIP = 36, F2_CIP = 68;
constexpr int kF0Off = kImgOff;
constexpr int kF1Off = kF0Off + NBF * I0_TP * F0_CIP;
constexpr int kF2Off = kF1Off + NBF * I1_TP * F1_CIP;
constexpr int kF2End = kF2Off + NBF * I2_TP * F2_CIP;
// bf16 images (the largest user of the carve is the split-bf16 set below)
constexpr int kImgEnd = kImgOff + NBF * (I0_TP * 40 + I1_TP * 72 + I2_TP * 136) / 2 > kF2End
                            ? kImgOff + NBF * (I0_TP * 40 + I1_TP * 72 + I2_TP * 136) / 2
                            : kF2End;
// bf16 images (offsets in float units)
constexpr int kB0Off = kImgOff;
constexpr int kB1Off = kB0Off + NBF * I0_TP * I0_CIP / 2;
constexpr int kB2Off = kB1Off + NBF * I1_TP * I1_CIP / 2;
// split-bf16 images (WK_PREC_BF16X3): xh at ci, xl at ci + 16 CB of the same row
constexpr int X0_CIP = 40, X1_CIP = 72, X2_CIP = 136;                // halfs (= 8 mod 16)
constexpr int kX0Off = kImgOff;
constexpr int kX1Off = kX0Off + NBF * I0_TP * X0_CIP / 2;
constexpr int kX2Off = kX1Off + NBF * I1_TP * X1_CIP / 2;
static_assert(kX2Off + NBF * I2_TP * X2_CIP / 2 <= kImgEnd, "split images fit the fp32 carve");
static_assert(kF1Off % 4 == 0 && kF2Off % 4 == 0 && kB1Off % 2 == 0 && kB2Off % 2 == 0 && kX1Off % 2 == 0 &&
                  kX2Off % 2 == 0, "vector-aligned images");
enum { kConvF32 = 0, kConvBf16 = 1, kConvBf16x3 = 2 };
// Scratch power row for the one frame slot past the clip (frame 63): its lanes
// still run the FFT so that the prefetch loads issued inside fe_rest execute.
constexpr int kDummyRowOff = (kImgEnd + 1) & ~1;          // even: its scratch is row + (63 & 1)
constexpr int kFusedLds = kDummyRowOff + kPRow + 1;
static_assert(kFusedLds * 4 <= 163840, "fused LDS budget");
// The CNN role writes only inside [kGOff, kImgEnd) (pooled features,
// classifier partials, the second log-mel buffer it reads, control words,
// conv images); the front-end writes its power rows, the first log-mel
// buffer and (frame 63) the dummy row: the two write sets are disjoint.
static_assert(kPOff + kPSize <= kGOff && kLOff + kLSize <= kPOff && kImgEnd <= kDummyRowOff,
              "CNN carve disjoint from the front-end's power rows, log-mel buffer and dummy row");
// Inside the window, the front-end writes the second log-mel buffer and the
// control words; the CNN role's writes (pooled features, classifier partials,
// every precision's image set) sit in ranges that miss it.
static_assert(kGOff + 128 * NBF <= kFcpOff && kFcpOff + kFcpSize <= kL1Off && kL1Off + kLSize <= kCtrlOff &&
                  kCtrlOff + 16 <= kImgOff,
              "pooled features | partials | log-mel buffer 1 | control words, in that order, disjoint");
static_assert(kF2End <= kImgEnd && kB2Off + NBF * I2_TP * I2_CIP / 2 <= kImgEnd &&
                  kX2Off + NBF * I2_TP * X2_CIP / 2 <= kImgEnd,
              "every precision's conv images end inside [kImgOff, kImgEnd)");

// kCtrlLFree + w (w = CNN wave 0..7): clips whose log-mel buffer CNN wave w
// has finished reading.  Per wave, not one shared count: the CNN waves are not
// lock-stepped inside a batch's DCT loop (and the classifier.2 wave starts the
// next batch late), so a summed count can reach 8 (i - 1) while one wave is
// still reading clip i - 2's buffer -- 7 waves ahead by a clip or more paid
// for the laggard.  That race corrupted the laggard's DCT coefficients in ~1
// clip per 65k (seen with split-bf16 timing).  The other counters are sound as
// sums: their producers pass a barrier between consecutive signals.
enum { kCtrlFeBar = 0, kCtrlCnnBar = 1, kCtrlLReady = 2, kCtrlLFree = 4, kCtrlAbort = 15 };
static_assert(kCtrlOff % 4 == 0 && kCtrlLFree % 4 == 0, "spin_until_all8 reads the eight LFree words as two uint4");
// Every spin is bounded (~4M sleeps, well under a second): a protocol bug
// yields wrong logits and a drained grid, never a hung GPU.
constexpr unsigned kSpinLimit = 1u << 22;

__device__ __forceinline__ unsigned lds_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The same word as a wave-uniform (SGPR) value: every lane reads the same
// address, and a spin's exit tests on an SGPR compile to a scalar compare and
// branch instead of the exec-mask bookkeeping of a divergent loop exit.
__device__ __forceinline__ unsigned lds_load_u(const unsigned* p) {
  return __builtin_amdgcn_readfirstlane(lds_load(p));
}

constexpr int kPrioFe = 3;     // issue priority of the front-end waves (the critical path; see the kernel)
constexpr int kSpinSleep = 2;  // s_sleep argument (x 64 cycles) between polls (2 measured >= 1; 4, 8 equal)

// Spin until ready() (a wave-uniform test of an LDS word).  On a timeout the
// workgroup's abort word is set and every later spin returns at once.  Every
// poll is issue time taken from the other waves of the SIMD, so a waiting wave
// drops to issue priority 0 (PRIO = the role's priority, restored on exit),
// polls four times per loop trip and checks the bound and the abort word only
// every 32nd poll: per poll a sleep, the read, its wait, one readfirstlane, a
// scalar compare and branch (the former one-poll loop with its two exits
// compiled to ~19 instructions of exec-mask bookkeeping per poll).
template <int PRIO, typename F>
__device__ __forceinline__ void spin_on(unsigned* ctrl, const F& ready) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (!ready()) {
    if (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    for (unsigned n = 4;; n += 4) {
      __builtin_amdgcn_s_sleep(kSpinSleep);
      if (ready()) break;
      __builtin_amdgcn_s_sleep(kSpinSleep);
      if (ready()) break;
      __builtin_amdgcn_s_sleep(kSpinSleep);
      if (ready()) break;
      __builtin_amdgcn_s_sleep(kSpinSleep);
      if (ready()) break;
      if ((n & 31) == 0 && (n >= kSpinLimit || lds_load_u(ctrl + kCtrlAbort))) {
        __hip_atomic_store(ctrl + kCtrlAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
    }
    if (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
  }
  asm volatile("" ::: "memory");
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Spin until ctrl[idx] >= v.
template <int PRIO>
__device__ __forceinline__ void spin_until(unsigned* ctrl, int idx, unsigned v) {
  spin_on<PRIO>(ctrl, [=] { return lds_load_u(ctrl + idx) >= v; });
}

// Barrier among the 8 waves of one role (LDS counter; s_barrier would also
// stop the other role's waves).  LDS operations of a wave complete in order,
// so a wave's data writes are visible before its arrival is.
template <int PRIO, int N = 8>
__device__ __forceinline__ void role_sync(unsigned* ctrl, int idx, unsigned& gen, int lane) {
  gen += N;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctrl + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until<PRIO>(ctrl, idx, gen);
}

// Spin until ctrl[idx + w] >= v for all w < 8 (same rules as spin_until).
// The eight words are 16-byte aligned (idx = kCtrlLFree = 4): two 16-byte LDS
// reads per poll instead of eight.
__device__ __forceinline__ unsigned min8(const unsigned* ctrl, int idx) {
  asm volatile("" ::: "memory");
  const uint4* q = reinterpret_cast<const uint4*>(ctrl + idx);
  const uint4 a = q[0], b = q[1];
  return min(min(min(a.x, a.y), min(a.z, a.w)), min(min(b.x, b.y), min(b.z, b.w)));
}
template <int PRIO>
__device__ __forceinline__ void spin_until_all8(unsigned* ctrl, int idx, unsigned v) {
  spin_on<PRIO>(ctrl, [=] { return __builtin_amdgcn_readfirstlane(min8(ctrl, idx)) >= v; });
}

// Publish a per-wave progress value once this wave's LDS ops are complete.
__device__ __forceinline__ void signal_set(unsigned* ctrl, int idx, unsigned v, int lane) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(ctrl + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ void signal_add(unsigned* ctrl, int idx, int lane) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctrl + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ---------------------------------------------------------------------------
// Front-end role (waves 0-7): mode B (torchaudio + CMVN), one clip at a time.
// FEW = 12 (diagnostic builds only, WK_FE_WAVES): 12 front-end waves, 3 per
// SIMD -- waves 0-3 run rounds 0 and 1 of frame slot w, waves 4-7 round 0 of
// slot w, waves 8-11 round 1 of slot w - 4; the mel stays 8-way, on waves 4-11.
// ---------------------------------------------------------------------------
template <typename T, int FEW = 8>
__device__ __forceinline__ void fe_role(float* smem, const T* __restrict__ audio, int64_t n_mine,
                                        int64_t clip_stride, float* __restrict__ feats_out, int wave, int lane,
                                        int diag) {
  static_assert(FEW == 8 || FEW == 12, "8 or 12 front-end waves");
  float* P = smem + kPOff;
  float* L = smem + kLOff;
  float* L1 = smem + kL1Off;
  unsigned* ctrl = reinterpret_cast<unsigned*>(smem + kCtrlOff);
  const int g = lane >> 4, j = lane & 15;
  const FeTables tb = {smem + kWinOff, smem + kTwOff};
  const TwsLds tws = {smem + kTwsOff};
  const f2 w0 = fe_split_tw(j, 0);
  const int slot_base = 16 * (g & 1) + 32 * (g >> 1);
  // frame slot of this wave (moving the edge frames to other waves measured neutral), its rounds r0..r1
  const int fw = FEW == 8 || wave < 8 ? wave : wave - 4;
  const int r0 = FEW == 8 || wave < 8 ? 0 : 1, r1 = FEW == 8 || wave < 4 ? 1 : r0;
  const bool mel_wave = FEW == 8 || wave >= 4;
  const int melw = FEW == 8 ? wave : wave - 4;
  const int64_t G = gridDim.x;
  unsigned gen = 0, p_wait = 0;

  // Static frame assignment: wave w, round r, lane group g takes frame
  // w + 8r + 16(g&1) + 32(g>>1) (groups 0/1 16 frames apart: disjoint LDS
  // banks).  A dynamic hand-out through an LDS counter was measured slower:
  // the atomic's return latency lands on the prefetch path.  Both edge
  // frames in wave 0's round 0 (one reflected-index round per clip instead
  // of two) measured -1 %: that wave then finishes last at the clip barrier.
  //
  // Prefetch context of a round, built once per round: the clip's buffer
  // resource and whether the round holds a reflected edge frame (frame 0 in
  // wave 0 round 0, frame 62 in wave 6 round 1; wave-uniform).  Past the
  // workgroup's last clip the resource has num_records 0, so those loads
  // return 0 without a branch; the padding slot (frame 63) needs no lane mask
  // either, since its samples past the clip's end come back 0 from the same
  // bounds check.  (Rebuilt inside each of the four prefetch parts, the 64-bit
  // clip address, the `i < n_mine` test and the per-lane `frame < 63` exec mask
  // cost ~28 scalar/branch instructions per part, ~13 % of a round's issue.)
  const int64_t step = G * clip_stride;
  const T* cptr = audio + (int64_t)blockIdx.x * clip_stride;   // clip i of this workgroup
  constexpr uint32_t kClipBytes = kWinSamples * sizeof(T);
  struct PfCtx {
    __amdgpu_buffer_rsrc_t rs;
    int base;       // first sample of the lane group's frame (before reflection)
    bool general;   // edge frame: per-lane reflected indices, issued whole with part 0
  };
  // Frame slot of round r.  The bf16-family unit (scalar front-end) swaps
  // round 1's slots between waves w and w ^ 4, so its second edge frame (62)
  // runs on wave 2 rather than wave 6: waves 4-7 issue after 0-3 on each SIMD
  // and reach the power-row barrier last, wave 6 with the edge frame latest.
  // bf16 +0.8 %; the packed fp32 unit measured -0.8 % with it
  // (profiles/r06ae_round1_swap_ab.txt).  Bit-identical either way.
  auto fwr = [&](int r) { return FEW == 8 && WK_FE_STAGED && r == 1 ? fw ^ 4 : fw; };
  auto pf_ctx = [&](const T* p, bool ok, int r) -> PfCtx {
    const int fl = fwr(r) + 8 * r + slot_base;
    return {make_rsrc(p, ok ? kClipBytes : 0u), 256 * fl - 160, (r == 0 && fwr(r) == 0) || (r == 1 && fwr(r) == 6)};
  };

  Raw<T> pf;
  {
    const PfCtx c0 = pf_ctx(cptr, n_mine > 0, r0);
    load_raw<true>(c0.rs, c0.base, j, kWinSamples, true, c0.general, pf);
  }
  WK_STAMP_INIT
  for (int64_t i = 0; i < n_mine; ++i) {
#pragma unroll 1
    for (int r = r0; r <= r1; ++r) {
      const int fl = fwr(r) + 8 * r + slot_base;   // == frame index t (one chunk per clip)
      const bool general = (r == 0 && fwr(r) == 0) || (r == 1 && fwr(r) == 6);
      f2 a[16];
#ifdef WK_DIAG
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // diagnostic: time the wait for the prefetched audio apart
      WK_STAMP(11);
#endif
      // Every lane runs the round (the frame-63 slot into a scratch row) so
      // the prefetch parts issued from inside fe_rest load for all lanes.
      fe_stage0<true>(pf, 256 * fl - 160, kWinSamples, j, general, tb, a);
      WK_STAMP(0);
      // next round: (i, 1) after round 0, (i + 1, 0) after round 1 (one-round waves: (i + 1, r0))
      const PfCtx nx = r < r1 ? pf_ctx(cptr, true, r + 1) : pf_ctx(cptr + step, i + 1 < n_mine, r0);
      // k = -1: the round is about to write its first power-row element.  In
      // round 0 that needs every wave done reading clip i-1's rows (its mel);
      // waiting there rather than before the round lets stage 0, the loads and
      // the first DFT16 overlap the slower waves' mel.
      auto pf_part = [&](int k) {
        if (k >= 0) {
          load_raw_part<true>(nx.rs, nx.base, j, kWinSamples, true, nx.general, pf, k);
        } else if (r == r0) {
          spin_until<kPrioFe>(ctrl, kCtrlFeBar, p_wait);
          WK_STAMP(9);
        }
      };
      WK_STAMP(1);
      float* row = fl < kNFramesB ? P + fl * kPRow : smem + kDummyRowOff;
      fe_rest<true>(a, j, row, row + (fl & 1), tb, w0, tws, 0, pf_part WK_SP_ARG);
    }
    role_sync<kPrioFe, FEW>(ctrl, kCtrlFeBar, gen, lane);               // all power rows of clip i written
    WK_STAMP(7);
    if (mel_wave && i >= 2 && !(diag & 1)) spin_until_all8<kPrioFe>(ctrl, kCtrlLFree, (unsigned)(i - 1));   // clip i-2's DCT done
    WK_STAMP(10);
    if (mel_wave) {
      // The row base stays opaque (one VGPR with kPOff in it), so the mel's
      // power reads take bin offsets as read2 immediates; folded into the
      // immediates, kPOff pushed them past read2's 255-dword reach and every
      // pair of reads cost a v_add_u32 for its address.
      int prow = kPOff + min(lane, kNFramesB - 1) * kPRow;
      asm volatile("" : "+v"(prow));
      mel_dispatch<true>(melw, smem + prow, (i & 1 ? L1 : L) + lane);
      WK_STAMP(8);
      signal_add(ctrl, kCtrlLReady, lane);
    }
    // Split barrier: arrive now, wait before this wave next writes a power
    // row (its first round of clip i+1), after its stage 0 and prefetch.
    gen += FEW;
    signal_add(ctrl, kCtrlFeBar, lane);
    p_wait = gen;
    cptr += step;
  }
  WK_STAMP_FLUSH(wave);
}

// ---------------------------------------------------------------------------
// DCT-II + CMVN of one clip on the matrix cores (extract_mfcc.py:70-80; the
// DCT of torchaudio.transforms.MFCC, ortho, 13 of 40): the 13x40 DCT (rows
// 13-15 zero) times the [40 mel][64 frame] log-mel image is a 16x40x64 fp32
// GEMM = 10 K-steps x 4 column tiles of v_mfma_f32_16x16x4f32, run by ONE wave.
// Column li of tile nt is frame 4 li + nt, so a lane's B values of one K-step
// are 4 consecutive frames: one ds_read_b128 feeds the 4 tiles.  The lane then
// holds coefficients 4 lk .. 4 lk + 3 of frames 4 li .. 4 li + 3: CMVN's
// per-coefficient sums are 3 in-register adds + a 16-lane DPP row reduction,
// and the 4 normalised coefficients of a frame leave as one 16-byte (fp32) or
// 8-byte (bf16) store into the conv1 image [clip][t][ci].  Frame 63 (column
// 15 of tile 3) is a padding column: excluded from the statistics, not stored.
// (Replaces 13 x 40 lane-per-frame FMAs + 13 separate wave reductions spread
// over the 8 CNN waves: ~1,300 VALU instructions per clip -> 40 MFMA + ~150.)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float row_sum16(float v) {   // sum over the lane's 16-lane row, in every lane
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

template <int CM>
__device__ __forceinline__ void dct_cmvn_clip(const float* __restrict__ lbuf, int slot, float* __restrict__ F0,
                                              uint16_t* __restrict__ B0, uint16_t* __restrict__ X0,
                                              float* __restrict__ fo, int lane) {
  const int li = lane & 15, lk = lane >> 4;
  // A fragments kDctB16[li][4 s + lk], re-read (L1/L2-resident, 2.5 KB) per
  // clip: kept live across the batch they pushed the fp32 CNN into spills.
  int aoff = 4 * (li * 40 + lk);
  asm volatile("" : "+v"(aoff));   // not loop-invariant: keep the loads here
  const auto ra = make_rsrc(kDctB16, sizeof(kDctB16));
  float dA[10];
#pragma unroll
  for (int s = 0; s < 10; ++s) dA[s] = buf_load(ra, aoff, 16 * s);
  f32x4 d[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
  for (int s = 0; s < 10; ++s) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(lbuf + (4 * s + lk) * WK_LSTRIDE + 4 * li);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) d[nt] = mfma4(dA[s], b[nt], d[nt]);
  }
  const bool v3 = li != 15;   // tile 3 column 15 = frame 63 (padding)
  float mean[4], inv[4];
  // Reciprocal constants, v_sqrt_f32 and v_rcp_f32 (each <= 1 ulp) instead of
  // IEEE divisions and the libm square root: 12 divisions per clip had
  // compiled to ~10-instruction div_scale/div_fmas/div_fixup sequences.
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x3 = v3 ? d[3][r] : 0.0f;
    mean[r] = row_sum16((d[0][r] + d[1][r]) + (d[2][r] + x3)) * (1.0f / kNFramesB);
    float dv[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dv[nt] = d[nt][r] - mean[r];
    dv[3] = v3 ? dv[3] : 0.0f;
    const float q = row_sum16((dv[0] * dv[0] + dv[1] * dv[1]) + (dv[2] * dv[2] + dv[3] * dv[3]));
    float sd = __builtin_amdgcn_sqrtf(q * (1.0f / (kNFramesB - 1)));
    sd = sd == 0.0f ? 1.0f : sd;   // rows 13-15 (all zero) land here and stay 0
    inv[r] = __builtin_amdgcn_rcpf(sd + 1e-8f);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int t = 4 * li + nt;
    if (nt == 3 && !v3) continue;
    const int row = slot * I0_TP + 1 + t;
    float y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = (d[nt][r] - mean[r]) * inv[r];
    if constexpr (CM == kConvBf16) {
      uint2 pk;
      pk.x = bf16_bits(y[0]) | (bf16_bits(y[1]) << 16);
      pk.y = bf16_bits(y[2]) | (bf16_bits(y[3]) << 16);
      *reinterpret_cast<uint2*>(B0 + row * I0_CIP + 4 * lk) = pk;
    } else if constexpr (CM == kConvBf16x3) {
      uint32_t h[4], l[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = bf16_bits(y[r]);
        l[r] = bf16_bits(y[r] - __uint_as_float(h[r] << 16));
      }
      *reinterpret_cast<uint2*>(X0 + row * X0_CIP + 4 * lk) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
      *reinterpret_cast<uint2*>(X0 + row * X0_CIP + 16 + 4 * lk) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
    } else {
      *reinterpret_cast<f32x4*>(F0 + row * F0_CIP + 4 * lk) = f32x4{y[0], y[1], y[2], y[3]};
    }
    if (fo) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * lk + r < 13) fo[(4 * lk + r) * kNFramesB + t] = y[r];
    }
  }
}

// ---------------------------------------------------------------------------
// CNN role (waves 8-15): batches of NBF clips from the conv1 image.
// ---------------------------------------------------------------------------
// Where the CNN role's LDS lives: the fused kernel's carve window
// [kGOff, kImgEnd) -- pooled features, classifier partials, control words, the
// conv images -- at `base + offset` (base = smem in the fused kernel; the
// standalone CNN kernel below places two such windows per workgroup).
// SRC supplies the conv1 input image of each clip (interface below):
//   init(cw, lane)   once per wave;
//   ready(i)         whether clip i's image can be made without waiting;
//   wait(i)          block until it can;
//   load(i, slot)    write clip i's normalised [63][13] MFCC into conv1 slot `slot`.
// The fused kernel's source is the DCT + CMVN of the front-end's log-mel
// (LogmelSrc); the standalone CNN's is the caller's features in HBM (FeatSrc).
template <int CM, class SRC>   // kConvF32 / kConvBf16 / kConvBf16x3
__device__ __forceinline__ void cnn_role(float* base, const float* __restrict__ pk, const uint16_t* __restrict__ pkb,
                                         int64_t n_mine, int64_t clip_base, int64_t clip_step,
                                         float* __restrict__ logits, int cw, int lane, SRC& src) {
  float* F0 = base + kF0Off;
  float* F1 = base + kF1Off;
  float* F2 = base + kF2Off;
  uint16_t* B0 = reinterpret_cast<uint16_t*>(base + kB0Off);
  uint16_t* B1 = reinterpret_cast<uint16_t*>(base + kB1Off);
  uint16_t* B2 = reinterpret_cast<uint16_t*>(base + kB2Off);
  uint16_t* X0 = reinterpret_cast<uint16_t*>(base + kX0Off);
  uint16_t* X1 = reinterpret_cast<uint16_t*>(base + kX1Off);
  uint16_t* X2 = reinterpret_cast<uint16_t*>(base + kX2Off);
  constexpr bool BF = CM == kConvBf16, X3 = CM == kConvBf16x3;
  constexpr int kLoW = kNumPackedBf16;   // the xl fragments follow the xh ones (pack_fragments_bf16x3)
  const auto rsb = make_rsrc(pkb, 2 * kNumPackedBf16 * (X3 ? 2 : 1));
  auto frag_bf = [&](int elem_off) -> s8 {   // one lane's 8 bf16 of the fragment at elem_off (x 64 lanes x 8)
    return __builtin_bit_cast(s8, __builtin_amdgcn_raw_buffer_load_b128(rsb, 16 * lane, 2 * elem_off, 0));
  };
  float* Gp = base + kGOff;
  float* FCP = base + kFcpOff;
  unsigned* ctrl = reinterpret_cast<unsigned*>(base + kCtrlOff);
  const int li = lane & 15, lk = lane >> 4;
  unsigned gen = 0;
  const auto rs = make_rsrc(pk, 4 * kNumPacked);
  const int lv = 4 * lane;

  // Weights come fragment-major (wk_kernels.h pack_fragments): one coalesced
  // 256-byte load per A fragment.  conv3's (48 fragments) stay in VGPRs; the
  // other layers' are re-read from L2 per batch.
  float w3[48];
  s8 w3b[6];
  if constexpr (BF || X3) {
#pragma unroll
    for (int s = 0; s < 6; ++s) w3b[s] = frag_bf(kPbW3 + (cw * 6 + s) * kBfFrag);
  }
  if constexpr (CM == kConvF32) {
#pragma unroll
    for (int s = 0; s < 48; ++s) w3[s] = buf_load(rs, lv, 4 * (kPkW3 + (cw * 48 + s) * 64));
  }
  const int64_t n_batches = (n_mine + NBF - 1) / NBF;
  src.init(cw, lane);
  bool eager_done = false;
  // Between the conv phases of batch b (after its conv1 has consumed the conv1
  // image): if clip 4(b+1) + cw's input is already available, make its image
  // now (fused: its buffer goes back to the front-end a whole batch earlier;
  // the double buffer otherwise stalled the front-end ~13 % of the time in fp32).
  auto try_eager = [&](int64_t b) {
    if (cw >= NBF || eager_done) return;
    const int64_t i = (b + 1) * NBF + cw;
    if (i >= n_mine) return;
    if (src.ready(i)) {
      src.load(i, cw);
      eager_done = true;
    }
  };
  // ReLU -> classifier.2 (64 -> 1) of batch bb from the classifier.0 partials
  // (one per CNN wave's k-slice): lane = (o group q = lane>>2, clip = lane&3),
  // one 16-byte read per slice.  Run by one wave, deferred to just after the
  // next batch's first barrier (one barrier per batch fewer).
  auto fc2 = [&](int64_t bb) {
    if (cw != 0) return;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int cl = ln & (NBF - 1), q = ln >> 2;
    // In the bf16 family the slice sums are scalar fp32 adds, never f32x4
    // arithmetic (which is v_pk_add_f32): this wave runs beside the K = 32
    // convolutions of the other CNN waves on its SIMD (the K = 32 rule,
    // DESIGN 5.1; tests/test_isa_rules.py).  The fp32 build keeps the packed
    // adds (its MFMAs are K = 4; scalar measured -1 %, profiles/r06b_ab.txt).
    float h[4];
    if constexpr (CM == kConvF32) {
      f32x4 v = *reinterpret_cast<const f32x4*>(FCP + cl * 64 + 4 * q);
#pragma unroll
      for (int w = 1; w < 8; ++w) v += *reinterpret_cast<const f32x4*>(FCP + (w * NBF + cl) * 64 + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = v[r];
    } else {
      const f32x4 v = *reinterpret_cast<const f32x4*>(FCP + cl * 64 + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = v[r];
#pragma unroll
      for (int w = 1; w < 8; ++w) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(FCP + (w * NBF + cl) * 64 + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] += u[r];
      }
    }
    float acc = 0.0f;
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) acc = __builtin_fmaf(buf_load(rs, 16 * q, 4 * (kPkF2 + i2)), fmaxf(h[i2], 0.0f), acc);
    acc += __shfl_xor(acc, 4, 64);
    acc += __shfl_xor(acc, 8, 64);
    acc += __shfl_xor(acc, 16, 64);
    acc += __shfl_xor(acc, 32, 64);
    const int64_t i = bb * NBF + cl;
    if (q == 0 && i < n_mine) logits[clip_base + clip_step * i] = acc;
  };
  WK_STAMP_INIT
  for (int64_t b = 0; b < n_batches; ++b) {
    // DCT-II + CMVN (extract_mfcc.py:70-80): CNN wave s < NBF takes clip
    // 4b + s whole on the matrix cores (dct_cmvn_clip), unless it already did
    // so eagerly during the previous batch (try_eager below).
    if (cw < NBF && !eager_done) {
      const int64_t i = b * NBF + cw;
      if (i < n_mine) {
        src.wait(i);
        src.load(i, cw);
      }
    }
    eager_done = false;
    // conv1's A fragments: loaded after the DCT (register pressure), landing during the sync.
    float w1[12];
    s8 w1b[2], w1l[2];
    if constexpr (BF || X3) {
#pragma unroll
      for (int s = 0; s < 2; ++s) w1b[s] = frag_bf(kPbW1 + ((cw & 1) * 2 + s) * kBfFrag);
    }
    if constexpr (X3) {
#pragma unroll
      for (int s = 0; s < 2; ++s) w1l[s] = frag_bf(kLoW + kPbW1 + ((cw & 1) * 2 + s) * kBfFrag);
    }
    if constexpr (CM == kConvF32) {
#pragma unroll
      for (int s = 0; s < 12; ++s) w1[s] = buf_load(rs, lv, 4 * (kPkW1 + ((cw & 1) * 12 + s) * 64));
    }
    WK_STAMP(0);
    role_sync<0>(ctrl, kCtrlCnnBar, gen, lane);   // conv1 image complete (and the previous batch's partials)
    if (b > 0) fc2(b - 1);

    // Clips of this batch that exist (wave-uniform): a short last batch -- and
    // the one-window launches of the streaming path -- skip the conv passes
    // that cover only absent clips, which shortens each wave's MFMA chain
    // (single-window latency).  Full batches run every pass.
    const int nv = n_mine - b * NBF < NBF ? (int)(n_mine - b * NBF) : NBF;

    // conv1: co tile (cw&1), clip (cw>>1), 4 t-tiles.
    if ((cw >> 1) < nv) {
      const int co0 = 16 * (cw & 1), cl = cw >> 1;
      const int bo = (cl * I0_TP + li) * I0_CIP;   // this lane's t row in the bf16 [clip][t][ci] image
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int ta = 32 * p, tb = ta + 16;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        if constexpr (BF) {
          conv_pair_bf<2, 16, I0_CIP>(B0, w1b, bo + ta * I0_CIP, bo + tb * I0_CIP, lk, acc_a, acc_b);
          epi_pool_bf<I1_CIP, I1_TP, 31>(acc_a, B1, co0, cl, ta, lane);
          epi_pool_bf<I1_CIP, I1_TP, 31>(acc_b, B1, co0, cl, tb, lane);
        } else if constexpr (X3) {
          const int bx = (cl * I0_TP + li) * X0_CIP;
          conv_pair_bf3<2, 16, X0_CIP>(X0, w1b, w1l, bx + ta * X0_CIP, bx + tb * X0_CIP, lk, acc_a, acc_b);
          epi_pool_bf3<X1_CIP, I1_TP, 31, 32>(acc_a, X1, co0, cl, ta, lane);
          epi_pool_bf3<X1_CIP, I1_TP, 31, 32>(acc_b, X1, co0, cl, tb, lane);
        } else {
          // Winograd pairs 16 p .. 16 p + 15 (outputs 32 p .. 32 p + 31)
          f32x4 m[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
          conv_wino_v<1, F0_CIP>(F0, w1, (cl * I0_TP + 2 * (16 * p + li)) * F0_CIP + 4 * lk, m);
          epi_wino_pool<F1_CIP, I1_TP, 31>(m, F1, co0, cl, 16 * p, lane);
        }
      }
    }
    WK_STAMP(1);
    role_sync<0>(ctrl, kCtrlCnnBar, gen, lane);
    try_eager(b);
    WK_STAMP(2);

    // conv2: co tile (cw&3), clips 2*(cw>>2) + {0,1}, 2 t-tiles each.
    if constexpr (BF) {
      s8 w2b[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) w2b[s] = frag_bf(kPbW2 + ((cw & 3) * 3 + s) * kBfFrag);
      const int co0 = 16 * (cw & 3);
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int cl = 2 * (cw >> 2) + p;
        if (cl >= nv) break;
        const int bb = (cl * I1_TP + li) * I1_CIP;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair_bf<3, 32, I1_CIP>(B1, w2b, bb, bb + 16 * I1_CIP, lk, acc_a, acc_b);
        epi_pool_bf<I2_CIP, I2_TP, 15>(acc_a, B2, co0, cl, 0, lane);
        epi_pool_bf<I2_CIP, I2_TP, 15>(acc_b, B2, co0, cl, 16, lane);
      }
    } else if constexpr (X3) {
      s8 w2b[3], w2l[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) w2b[s] = frag_bf(kPbW2 + ((cw & 3) * 3 + s) * kBfFrag);
#pragma unroll
      for (int s = 0; s < 3; ++s) w2l[s] = frag_bf(kLoW + kPbW2 + ((cw & 3) * 3 + s) * kBfFrag);
      const int co0 = 16 * (cw & 3);
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int cl = 2 * (cw >> 2) + p;
        if (cl >= nv) break;
        const int bb = (cl * I1_TP + li) * X1_CIP;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair_bf3<3, 32, X1_CIP>(X1, w2b, w2l, bb, bb + 16 * X1_CIP, lk, acc_a, acc_b);
        epi_pool_bf3<X2_CIP, I2_TP, 15, 64>(acc_a, X2, co0, cl, 0, lane);
        epi_pool_bf3<X2_CIP, I2_TP, 15, 64>(acc_b, X2, co0, cl, 16, lane);
      }
    } else {
      float w2[24];
#pragma unroll
      for (int s = 0; s < 24; ++s) w2[s] = buf_load(rs, lv, 4 * (kPkW2 + ((cw & 3) * 24 + s) * 64));
      const int co0 = 16 * (cw & 3);
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int cl = 2 * (cw >> 2) + p;
        if (cl >= nv) break;
        f32x4 m[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        conv_wino_v<2, F1_CIP, 1>(F1, w2, (cl * I1_TP + 2 * li) * F1_CIP + 4 * lk, m);
        epi_wino_pool<F2_CIP, I2_TP, 15>(m, F2, co0, cl, 0, lane);
      }
    }
    WK_STAMP(3);
    role_sync<0>(ctrl, kCtrlCnnBar, gen, lane);
    try_eager(b);
    WK_STAMP(4);

    // conv3: co tile cw, the 4 clips; GAP -> G[128][4].
    {
      const int co0 = 16 * cw;
      const int bo = li * I2_CIP;
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        // between conv3's two passes too: the longest phase, during which the
        // front-end otherwise waited on the log-mel buffer (fp32 +1.1 %, bf16
        // +0.6 %, profiles/r06ac_eager_ab.txt; inside conv2 as well spilled, -0.6 %)
        if (p > 0) try_eager(b);
        const int ca = 2 * p, cb = 2 * p + 1;
        if (ca >= nv) break;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        if constexpr (BF) {
          conv_pair_bf<6, 64, I2_CIP, 3>(B2, w3b, bo + ca * I2_TP * I2_CIP, bo + cb * I2_TP * I2_CIP, lk, acc_a,
                                         acc_b);
        } else if constexpr (X3) {
          s8 w3l[6];   // the lo parts are re-read from L2 per pass (VGPR budget)
#pragma unroll
          for (int s = 0; s < 6; ++s) w3l[s] = frag_bf(kLoW + kPbW3 + (cw * 6 + s) * kBfFrag);
          const int bx = li * X2_CIP;
          conv_pair_bf3<6, 64, X2_CIP, 2>(X2, w3b, w3l, bx + ca * I2_TP * X2_CIP, bx + cb * I2_TP * X2_CIP, lk,
                                          acc_a, acc_b);
        } else {
          // Winograd: one tile of 16 pair columns = 8 pairs of clip ca, 8 of clip cb
          f32x4 m[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
          conv_wino_v<4, F2_CIP, 1>(F2, w3, ((ca + (li >> 3)) * I2_TP + 2 * (li & 7)) * F2_CIP + 4 * lk, m);
          epi_wino_gap<NBF>(m, Gp, co0, ca, lane);
          continue;
        }
        epi_gap<NBF>(acc_a, Gp, co0, ca, lane);
        epi_gap<NBF>(acc_b, Gp, co0, cb, lane);
      }
    }
    float wf1[16];
    {
#pragma unroll
      for (int s = 0; s < 16; ++s) wf1[s] = buf_load(rs, lv, 4 * (kPkF1 + (cw * 16 + s) * 64));
    }
    WK_STAMP(5);
    role_sync<0>(ctrl, kCtrlCnnBar, gen, lane);
    try_eager(b);
    WK_STAMP(6);

    // classifier.0 (128 -> 64) on v_mfma_f32_4x4x1_16b_f32: 16 blocks of 4 o x
    // 4 clips, block b = lane>>2 taking o = 4b .. 4b + 3 (A: lane = o, B: lane
    // & 3 = clip), so every column is a real clip (the 16x16x4 form used 4 of its
    // 16); wave cw takes k = 16 cw .. 16 cw + 15, and its partial
    // [o = 4(lane>>2) + r][clip lane&3] leaves as one 16-byte store.
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));   // addresses recomputed here rather than kept live (and spilled)
      f32x4 acc = {0, 0, 0, 0};
      const float* g = Gp + 16 * cw * NBF + (ln & (NBF - 1));
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma4x4(wf1[s], g[s * NBF], acc);
      *reinterpret_cast<f32x4*>(FCP + (cw * NBF + (ln & (NBF - 1))) * 64 + 4 * (ln >> 2)) = acc;
    }
    // No barrier here: classifier.2 of this batch reads the partials after the
    // next batch's first barrier (below), which already orders them; the
    // partials are next overwritten three barriers later.
    try_eager(b);
    WK_STAMP(8);
  }
  if (n_batches > 0) {
    role_sync<0>(ctrl, kCtrlCnnBar, gen, lane);
    fc2(n_batches - 1);
  }
  WK_STAMP_FLUSH(8 + cw);
}

// The fused kernel's clip source: DCT-II + CMVN of the front-end's log-mel
// image (dct_cmvn_clip), with the front-end hand-off protocol.
// FEATS: the launch also writes the CMVN'd features (parity dumps).  A
// template flag rather than a null test, so the product kernel carries no
// feature-store code (its address registers pushed the fp32 build to spill).
template <int CM, bool FEATS>
struct LogmelSrc {
  float* smem;
  unsigned* ctrl;
  float* feats_out;
  int64_t clip_base, clip_step;
  int cw, lane, diag;
  // Log-mel buffer release (kCtrlLFree + w): wave w < NBF reads only clips
  // w, w + NBF, w + 2 NBF, ...; its word holds the next clip it will read, so
  // every clip below it is released.  Waves >= NBF read none.
  __device__ __forceinline__ void init(int cw_, int lane_) {
    cw = cw_;
    lane = lane_;
    signal_set(ctrl, kCtrlLFree + cw, cw < NBF ? (unsigned)cw : 0xFFFFFFFFu, lane);
  }
  // A true answer is an acquire, like spin_until's exit: the compiler may not
  // move the caller's reads of the log-mel buffer (load() below) above the
  // ready-count read (LDS operations of a wave then complete in order).
  __device__ __forceinline__ bool ready(int64_t i) const {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const bool r = (diag & 2) ||
                   __builtin_amdgcn_readfirstlane(lds_load(ctrl + kCtrlLReady)) >= 8u * (unsigned)(i + 1);
    asm volatile("" ::: "memory");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return r;
  }
  __device__ __forceinline__ void wait(int64_t i) const {
    if (!(diag & 2)) spin_until<0>(ctrl, kCtrlLReady, 8u * (unsigned)(i + 1));
  }
  __device__ __forceinline__ void load(int64_t i, int slot) const {
    float* fo = FEATS ? feats_out + (clip_base + clip_step * i) * (13 * kNFramesB) : nullptr;
    dct_cmvn_clip<CM>(smem + (i & 1 ? kL1Off : kLOff), slot, smem + kF0Off,
                      reinterpret_cast<uint16_t*>(smem + kB0Off), reinterpret_cast<uint16_t*>(smem + kX0Off), fo,
                      lane);
    signal_set(ctrl, kCtrlLFree + cw, (unsigned)(i + NBF), lane);
  }
};

// Protocol health: a spin that timed out set its role's abort word, and every
// logit of the launch is then suspect.  Each wave reports what it sees on exit
// to the handle's error word (host-visible; read by wk_check_device_errors /
// wk_stream_push): bit 0 = a spin timed out, bit 1 = the abort word holds a
// value no spin writes (LDS corruption).
__device__ __forceinline__ void report_abort(const unsigned* ctrl, unsigned* err, int lane) {
  if (lane == 0 && err) {
    const unsigned ab = lds_load(ctrl + kCtrlAbort);
    if (ab) __hip_atomic_store(err, ab == 1u ? 1u : 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T, int CM, bool FEATS>
__global__ __launch_bounds__(kFusedBlock, 4) void wk_fused_kernel(const T* __restrict__ audio, int64_t batch,
                                                                 int64_t clip_stride, const float* __restrict__ wts,
                                                                 const uint16_t* __restrict__ wbf,
                                                                 float* __restrict__ logits,
                                                                 float* __restrict__ feats_out, unsigned* err,
                                                                 int diag) {
  __shared__ __attribute__((aligned(16))) float smem[kFusedLds];
#ifndef WK_DIAG
  diag = 0;   // role isolation (1 = front-end role only, 2 = CNN role only) in -DWK_DIAG builds; folded away here
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  fe_init_tables<true, true>(smem, tid, kFusedBlock);
  for (int i = tid; i < kFusedLds - kGOff; i += kFusedBlock) smem[kGOff + i] = 0.0f;  // ctrl, guards, pads
  __syncthreads();
  const int64_t n_mine = batch > (int64_t)blockIdx.x ? (batch - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  // The front-end role is the critical path: static issue priority over the
  // CNN role measured +0.5-0.9 % (priority 1-3); the reverse (CNN over
  // front-end) measured -13 %.
  if (wave < kFeWaves) __builtin_amdgcn_s_setprio(kPrioFe);
  if (wave < kFeWaves) {
    if (!(diag & 2)) fe_role<T, kFeWaves>(smem, audio, n_mine, clip_stride, feats_out, wave, lane, diag);
  } else {
    if (!(diag & 1)) {
      LogmelSrc<CM, FEATS> src = {smem, reinterpret_cast<unsigned*>(smem + kCtrlOff), feats_out, (int64_t)blockIdx.x,
                                  (int64_t)gridDim.x, 0, 0, diag};
      cnn_role<CM>(smem, wts, wbf, n_mine, (int64_t)blockIdx.x, (int64_t)gridDim.x, logits, wave - 8, lane, src);
    }
  }
  report_abort(reinterpret_cast<unsigned*>(smem + kCtrlOff), err, lane);
}

// ---------------------------------------------------------------------------
// Standalone CNN (wk_cnn: LightweightKWS.forward on caller features, the ONNX
// `run` surface).  The same CNN role as the fused kernel, fed from HBM: each
// 1024-thread workgroup runs TWO independent CNN roles of 8 waves, each with its
// own carve of images / pooled features / control words, on interleaved clips.
// FeatSrc copies clip i's CMVN'd features [13][63] (wakeModel.py input layout)
// into the conv1 image as [t][ci] rows: lane t reads its frame's 13
// coefficients (63 lanes of one coefficient are one coalesced 252-byte read).
// ---------------------------------------------------------------------------
template <int CM>
struct FeatSrc {
  const float* feats;
  float* base;   // the role's carve base (cnn_role's `base`)
  int64_t clip_base, clip_step;
  int lane;
  __device__ __forceinline__ void init(int, int lane_) { lane = lane_; }
  __device__ __forceinline__ bool ready(int64_t) const { return true; }
  __device__ __forceinline__ void wait(int64_t) const {}
  __device__ __forceinline__ void load(int64_t i, int slot) const {
    const float* f = feats + (clip_base + clip_step * i) * (13 * kNFramesB);
    if (lane >= kNFramesB) return;
    float y[13];
#pragma unroll
    for (int c = 0; c < 13; ++c) y[c] = __builtin_nontemporal_load(f + c * kNFramesB + lane);
    const int row = slot * I0_TP + 1 + lane;
    if constexpr (CM == kConvBf16) {
      uint16_t* B0 = reinterpret_cast<uint16_t*>(base + kB0Off) + row * I0_CIP;
#pragma unroll
      for (int c = 0; c < 12; c += 4)
        *reinterpret_cast<uint2*>(B0 + c) = make_uint2(bf16_bits(y[c]) | (bf16_bits(y[c + 1]) << 16),
                                                       bf16_bits(y[c + 2]) | (bf16_bits(y[c + 3]) << 16));
      B0[12] = (uint16_t)bf16_bits(y[12]);
    } else if constexpr (CM == kConvBf16x3) {
      uint16_t* X0 = reinterpret_cast<uint16_t*>(base + kX0Off) + row * X0_CIP;
#pragma unroll
      for (int c = 0; c < 13; ++c) {
        const uint32_t h = bf16_bits(y[c]);
        X0[c] = (uint16_t)h;
        X0[16 + c] = (uint16_t)bf16_bits(y[c] - __uint_as_float(h << 16));
      }
    } else {
      float* F0 = base + kF0Off + row * F0_CIP;
#pragma unroll
      for (int c = 0; c < 12; c += 4) *reinterpret_cast<f32x4*>(F0 + c) = f32x4{y[c], y[c + 1], y[c + 2], y[c + 3]};
      F0[12] = y[12];
    }
  }
};

constexpr int kCnnCarve = kImgEnd - kGOff;   // floats per CNN role: the fused carve window [kGOff, kImgEnd)
constexpr int kCnnLds = 2 * kCnnCarve;
static_assert(kCnnLds * 4 <= 163840, "standalone CNN LDS budget");
static_assert(kCnnCarve % 4 == 0 && kGOff % 4 == 0, "16-byte aligned carves");

template <int CM>
__global__ __launch_bounds__(kFusedBlock, 4) void wk_cnn_fused_kernel(const float* __restrict__ feats, int64_t batch,
                                                                     const float* __restrict__ wts,
                                                                     const uint16_t* __restrict__ wbf,
                                                                     float* __restrict__ logits, unsigned* err) {
  __shared__ __attribute__((aligned(16))) float smem[kCnnLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kCnnLds; i += kFusedBlock) smem[i] = 0.0f;   // guards, padding ci, control words
  __syncthreads();
  const int role = wave >> 3;
  float* base = smem + role * kCnnCarve - kGOff;   // base + kGOff = this role's window
  const int64_t cb = 2 * (int64_t)blockIdx.x + role, cs = 2 * (int64_t)gridDim.x;
  const int64_t n_mine = batch > cb ? (batch - 1 - cb) / cs + 1 : 0;
  FeatSrc<CM> src = {feats, base, cb, cs, 0};
  cnn_role<CM>(base, wts, wbf, n_mine, cb, cs, logits, wave & 7, lane, src);
  report_abort(reinterpret_cast<const unsigned*>(base + kCtrlOff), err, lane);   // this wave's role
}

}  // namespace

#ifndef WK_FUSED_XDL_TU
#ifdef WK_DIAG
extern "C" int wk_debug_stamps(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wk_stamps), sizeof(g_wk_stamps)) != hipSuccess) return 1;
  if (reset) {
    static unsigned long long zero[16][16];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wk_stamps), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

#endif   // !WK_FUSED_XDL_TU

namespace wk {

#ifdef WK_FUSED_XDL_TU
hipError_t launch_fused_xdl(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                            const uint16_t* wbf, int conv_mode, float* logits, float* feats_or_null, int grid_cap,
                            hipStream_t stream, unsigned* err, int diag) {
#else
hipError_t launch_fused(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                        const uint16_t* wbf, int conv_mode, float* logits, float* feats_or_null, int grid_cap,
                        hipStream_t stream, unsigned* err, int diag) {
#endif
  if (batch == 0) return hipSuccess;
  const int grid = (int)(batch < grid_cap ? batch : grid_cap);
  const dim3 g(grid), blk(kFusedBlock);
  if (conv_mode != kConvF32 && !wbf) return hipErrorInvalidValue;
#if !WK_FUSED_ONE_TU && !defined(WK_FUSED_XDL_TU)
  if (conv_mode != kConvF32)   // the bf16 family: wk_fused_xdl.hip (scalar-fp32 front-end)
    return launch_fused_xdl(i16, audio, batch, clip_stride, w, wbf, conv_mode, logits, feats_or_null, grid_cap, stream,
                            err, diag);
#endif
#define WK_FUSED_LAUNCH(T, CM)                                                                              \
  do {                                                                                                         \
    if (feats_or_null)                                                                                         \
      hipLaunchKernelGGL((wk_fused_kernel<T, CM, true>), g, blk, 0, stream, (const T*)audio, batch, clip_stride, \
                         w, wbf, logits, feats_or_null, err, diag);                                               \
    else                                                                                                       \
      hipLaunchKernelGGL((wk_fused_kernel<T, CM, false>), g, blk, 0, stream, (const T*)audio, batch,            \
                         clip_stride, w, wbf, logits, nullptr, err, diag);                                        \
  } while (0)
#if defined(WK_FUSED_XDL_TU)   // bf16 / bf16x3 only
  if (i16) {
    if (conv_mode == kConvBf16x3) WK_FUSED_LAUNCH(int16_t, kConvBf16x3);
    else WK_FUSED_LAUNCH(int16_t, kConvBf16);
  } else {
    if (conv_mode == kConvBf16x3) WK_FUSED_LAUNCH(float, kConvBf16x3);
    else WK_FUSED_LAUNCH(float, kConvBf16);
  }
#elif !WK_FUSED_ONE_TU   // fp32 only (the bf16 family returned above)
  if (i16) WK_FUSED_LAUNCH(int16_t, kConvF32);
  else WK_FUSED_LAUNCH(float, kConvF32);
#else
  if (i16) {
    if (conv_mode == kConvBf16) WK_FUSED_LAUNCH(int16_t, kConvBf16);
    else if (conv_mode == kConvBf16x3) WK_FUSED_LAUNCH(int16_t, kConvBf16x3);
    else WK_FUSED_LAUNCH(int16_t, kConvF32);
  } else {
    if (conv_mode == kConvBf16) WK_FUSED_LAUNCH(float, kConvBf16);
    else if (conv_mode == kConvBf16x3) WK_FUSED_LAUNCH(float, kConvBf16x3);
    else WK_FUSED_LAUNCH(float, kConvF32);
  }
#endif
#undef WK_FUSED_LAUNCH
  return hipGetLastError();
}

#ifndef WK_FUSED_XDL_TU

hipError_t launch_cnn_fused(const float* feats, int64_t batch, const float* w, const uint16_t* wbf, int conv_mode,
                            float* logits, int grid_cap, hipStream_t stream, unsigned* err) {
  if (batch == 0) return hipSuccess;
  if (conv_mode != kConvF32 && !wbf) return hipErrorInvalidValue;
  const int64_t roles = (batch + NBF - 1) / NBF;   // at least one batch of clips per CNN role
  const int grid = (int)((roles + 1) / 2 < grid_cap ? (roles + 1) / 2 : grid_cap);
  if (conv_mode == kConvBf16)
    hipLaunchKernelGGL(wk_cnn_fused_kernel<kConvBf16>, dim3(grid), dim3(kFusedBlock), 0, stream, feats, batch, w, wbf,
                       logits, err);
  else if (conv_mode == kConvBf16x3)
    hipLaunchKernelGGL(wk_cnn_fused_kernel<kConvBf16x3>, dim3(grid), dim3(kFusedBlock), 0, stream, feats, batch, w,
                       wbf, logits, err);
  else
    hipLaunchKernelGGL(wk_cnn_fused_kernel<kConvF32>, dim3(grid), dim3(kFusedBlock), 0, stream, feats, batch, w, wbf,
                       logits, err);
  return hipGetLastError();
}
#endif   // !WK_FUSED_XDL_TU

}  // namespace wk
#endif   // !(WK_FUSED_XDL_TU && WK_FUSED_ONE_TU)
