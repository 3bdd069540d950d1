// wk_fused.hip -- the whole hot path in one persistent, warp-specialised kernel.
//
//   audio (HBM) -> MFCC front-end (VALU/LDS) -> features (LDS) -> xiaoa CNN
//   (fp32 MFMA) -> logit (HBM)
//
// One 16-wave workgroup per CU.  Waves 0-7 run the front-end of wk_frontend.hip
// clip after clip (FFT / lane-per-frame mel / DCT + CMVN, see wk_fe_dev.h) and
// write each clip's CMVN'd [13][63] features straight into the CNN's conv1
// input image in LDS.  Waves 8-15 run the CNN of wk_cnn.hip on batches of
// NBF = 4 clips from that image.  The two roles share no s_barrier: each role
// synchronises its own 8 waves through an LDS counter barrier, and the
// hand-off is two LDS counters (features ready / conv1 input free).  The
// front-end is VALU + LDS bound and the CNN is MFMA bound; on CDNA4 the
// matrix and vector pipes issue concurrently from different waves, so the
// two roles overlap on every SIMD (2 front-end + 2 CNN waves per SIMD), and
// features never touch HBM: per clip the kernel reads its 64,000 audio bytes
// and writes one 4-byte logit.
#include "wk_cnn_dev.h"
#include "wk_fe_dev.h"
#include "wk_kernels.h"

using namespace wk;

namespace {

constexpr int NBF = 4;               // clips per CNN batch
constexpr int kFusedBlock = 1024;    // 8 front-end + 8 CNN waves
// CNN images (floats); ci pitches are 16 mod 32 (conflict-free B fragments).
constexpr int F0_CLIP = 66, F0_CI = NBF * 66 + 8;   // conv1 input [16 ci][4][66], pitch 272
constexpr int F1_CLIP = 34, F1_CI = NBF * 34 + 8;   // conv2 input [32 ci][4][34], pitch 144
constexpr int F2_CLIP = 18, F2_CI = NBF * 18 + 8;   // conv3 input [64 ci][4][18], pitch 80
static_assert(F0_CI % 32 == 16 && F1_CI % 32 == 16 && F2_CI % 32 == 16, "bank-conflict-free pitches");
constexpr int kF0Off = kFeLds;
constexpr int kF1Off = kF0Off + 16 * F0_CI;
constexpr int kF2Off = kF1Off + 32 * F1_CI;
constexpr int kGOff = kF2Off + 64 * F2_CI;          // pooled features [128][4]
constexpr int kFcpOff = kGOff + 128 * NBF;          // classifier.0 partials [2][64][4]
constexpr int kCtrlOff = kFcpOff + 2 * 64 * NBF;    // control words
constexpr int kFusedLds = kCtrlOff + 16;
static_assert(kFusedLds * 4 <= 163840, "fused LDS budget");

enum { kCtrlFeBar = 0, kCtrlCnnBar = 1, kCtrlFeatReady = 2, kCtrlAct0Free = 3, kCtrlAbort = 15 };
// Every spin is bounded (~4M sleeps, well under a second): a protocol bug
// yields wrong logits and a drained grid, never a hung GPU.
constexpr unsigned kSpinLimit = 1u << 22;

__device__ __forceinline__ unsigned lds_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Spin until ctrl[idx] >= v.  On a timeout the workgroup's abort word is set
// and every later spin returns at once.
__device__ __forceinline__ void spin_until(unsigned* ctrl, int idx, unsigned v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  for (unsigned n = 0; lds_load(ctrl + idx) < v; ++n) {
    if (n >= kSpinLimit || lds_load(ctrl + kCtrlAbort)) {
      __hip_atomic_store(ctrl + kCtrlAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Barrier among the 8 waves of one role (LDS counter; s_barrier would also
// stop the other role's waves).  LDS operations of a wave complete in order,
// so a wave's data writes are visible before its arrival is.
__device__ __forceinline__ void role_sync(unsigned* ctrl, int idx, unsigned& gen, int lane) {
  gen += 8;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctrl + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until(ctrl, idx, gen);
}

__device__ __forceinline__ void signal_add(unsigned* ctrl, int idx, int lane) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctrl + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ---------------------------------------------------------------------------
// Front-end role (waves 0-7): mode B (torchaudio + CMVN), one clip at a time.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void fe_role(float* smem, const T* __restrict__ audio, int64_t n_mine,
                                        int64_t clip_stride, float* __restrict__ feats_out, int wave, int lane) {
  float* P = smem + kPOff;
  float* L = smem + kLOff;
  float* F0 = smem + kF0Off;
  unsigned* ctrl = reinterpret_cast<unsigned*>(smem + kCtrlOff);
  const int g = lane >> 4, j = lane & 15;
  const FeTables tb = {smem + kWinOff, smem + kTwOff};
  const cf w512 = fe_w512(j);
  const int slot_base = 16 * (g & 1) + 32 * (g >> 1);
  const int64_t G = gridDim.x;
  unsigned gen = 0;

  auto clip_of = [&](int64_t i) { return (int64_t)blockIdx.x + G * i; };
  auto prefetch = [&](int64_t i, int r, Raw<T>& dst) {
    if (i < n_mine) {
      const int fl = wave + 8 * r + slot_base;
      const bool slow = (r == 0 && wave == 0) || (r == 1 && wave == 6);
      load_raw<true>(make_rsrc(audio + clip_of(i) * clip_stride, kWinSamples * sizeof(T)), 256 * fl - 160, j,
                     kWinSamples, fl < kNFramesB, slow, dst);
    }
  };

  Raw<T> pf;
  prefetch(0, 0, pf);
  for (int64_t i = 0; i < n_mine; ++i) {
    const int64_t clip = clip_of(i);
#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
      const int fl = wave + 8 * r + slot_base;   // == frame index t (one chunk per clip)
      const bool slow = (r == 0 && wave == 0) || (r == 1 && wave == 6);
      cf a[16];
      if (fl < kNFramesB) {
        fe_stage0<true>(pf, 256 * fl - 160, kWinSamples, j, slow, tb, a);
      }
      prefetch(r == 0 ? i : i + 1, r ^ 1, pf);
      if (fl < kNFramesB) fe_rest<true>(a, j, lane, P + fl * kPRow, tb, w512, 0);
    }
    role_sync(ctrl, kCtrlFeBar, gen, lane);

    mel_dispatch<true>(wave, P + min(lane, kNFramesB - 1) * kPRow, L + lane);
    role_sync(ctrl, kCtrlFeBar, gen, lane);

    const int64_t b = i / NBF;
    const int s = (int)(i - b * NBF);
    if (s == 0 && b > 0) spin_until(ctrl, kCtrlAct0Free, (unsigned)b);   // CNN done reading batch b-1
    const float* lrow = L + lane;
    const bool valid = lane < kNFramesB;
    const int c0 = wave < 5 ? 2 * wave : wave + 5;
    const int nc = wave < 5 ? 2 : 1;
    for (int ci = 0; ci < nc; ++ci) {
      const int cc = c0 + ci;
      const float y = cmvn_lane(dct_coef<true>(cc, lrow), valid, kNFramesB);
      if (valid) {
        F0[cc * F0_CI + s * F0_CLIP + 1 + lane] = y;
        if (feats_out) feats_out[clip * (13 * kNFramesB) + cc * kNFramesB + lane] = y;
      }
    }
    if (s == NBF - 1 || i == n_mine - 1) signal_add(ctrl, kCtrlFeatReady, lane);
  }
}

// ---------------------------------------------------------------------------
// CNN role (waves 8-15): batches of NBF clips from the conv1 image.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cnn_role(float* smem, const float* __restrict__ pk, int64_t n_mine,
                                         float* __restrict__ logits, int cw, int lane) {
  float* F0 = smem + kF0Off;
  float* F1 = smem + kF1Off;
  float* F2 = smem + kF2Off;
  float* Gp = smem + kGOff;
  float* FCP = smem + kFcpOff;
  unsigned* ctrl = reinterpret_cast<unsigned*>(smem + kCtrlOff);
  const int li = lane & 15, lk = lane >> 4;
  const int64_t G = gridDim.x;
  unsigned gen = 0;
  const auto rs = make_rsrc(pk, 4 * kNumPacked);
  const int lv = 4 * lane;

  // Weights come fragment-major (wk_kernels.h pack_fragments): one coalesced
  // 256-byte load per A fragment.  conv3's (48 fragments) stay in VGPRs; the
  // other layers' are re-read from L2 per batch.
  float w3[48];
  {
#pragma unroll
    for (int s = 0; s < 48; ++s) w3[s] = buf_load(rs, lv, 4 * (kPkW3 + (cw * 48 + s) * 64));
  }
  const int64_t n_batches = (n_mine + NBF - 1) / NBF;
  for (int64_t b = 0; b < n_batches; ++b) {
    float w1[12];
    {
#pragma unroll
      for (int s = 0; s < 12; ++s) w1[s] = buf_load(rs, lv, 4 * (kPkW1 + ((cw & 1) * 12 + s) * 64));
    }
    spin_until(ctrl, kCtrlFeatReady, 8u * (unsigned)(b + 1));

    // conv1: co tile (cw&1), clip (cw>>1), 4 t-tiles.
    {
      const int co0 = 16 * (cw & 1), cl = cw >> 1;
      const int bo = lk * F0_CI + li + cl * F0_CLIP;
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int ta = 32 * p, tb = ta + 16;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<12, F0_CI, 4, 6>(F0, w1, bo + ta, bo + tb, acc_a, acc_b);
        epi_pool<F1_CI, F1_CLIP, 31>(acc_a, F1, co0, cl, ta, lane);
        epi_pool<F1_CI, F1_CLIP, 31>(acc_b, F1, co0, cl, tb, lane);
      }
    }
    role_sync(ctrl, kCtrlCnnBar, gen, lane);
    if (cw == 0) signal_add(ctrl, kCtrlAct0Free, lane);   // front-end may overwrite the conv1 image

    // conv2: co tile (cw&3), clips 2*(cw>>2) + {0,1}, 2 t-tiles each.
    {
      float w2[24];
#pragma unroll
      for (int s = 0; s < 24; ++s) w2[s] = buf_load(rs, lv, 4 * (kPkW2 + ((cw & 3) * 24 + s) * 64));
      const int co0 = 16 * (cw & 3);
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int cl = 2 * (cw >> 2) + p;
        const int bo = lk * F1_CI + li + cl * F1_CLIP;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<24, F1_CI, 8, 8>(F1, w2, bo, bo + 16, acc_a, acc_b);
        epi_pool<F2_CI, F2_CLIP, 15>(acc_a, F2, co0, cl, 0, lane);
        epi_pool<F2_CI, F2_CLIP, 15>(acc_b, F2, co0, cl, 16, lane);
      }
    }
    role_sync(ctrl, kCtrlCnnBar, gen, lane);

    // conv3: co tile cw, the 4 clips; GAP -> G[128][4].
    {
      const int co0 = 16 * cw;
      const int bo = lk * F2_CI + li;
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int ca = 2 * p, cb = 2 * p + 1;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<48, F2_CI, 16, 8>(F2, w3, bo + ca * F2_CLIP, bo + cb * F2_CLIP, acc_a, acc_b);
        epi_gap<NBF>(acc_a, Gp, co0, ca, lane);
        epi_gap<NBF>(acc_b, Gp, co0, cb, lane);
      }
    }
    float wf1[16];
    {
#pragma unroll
      for (int s = 0; s < 16; ++s) wf1[s] = buf_load(rs, lv, 4 * (kPkF1 + ((cw & 3) * 32 + 16 * (cw >> 2) + s) * 64));
    }
    role_sync(ctrl, kCtrlCnnBar, gen, lane);

    // classifier.0 (128 -> 64): o tile (cw&3), k half (cw>>2); columns >= NBF are don't-care.
    {
      f32x4 acc = {0, 0, 0, 0};
      const int kh = cw >> 2;
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma4(wf1[s], Gp[(64 * kh + 4 * s + lk) * NBF + (li & (NBF - 1))], acc);
      if (li < NBF) {
#pragma unroll
        for (int r = 0; r < 4; ++r) FCP[kh * 64 * NBF + (16 * (cw & 3) + 4 * lk + r) * NBF + li] = acc[r];
      }
    }
    role_sync(ctrl, kCtrlCnnBar, gen, lane);

    // ReLU -> classifier.2 (64 -> 1): lane = (o group q = lane>>2, clip = lane&3).
    if (cw == 0) {
      const int cl = lane & (NBF - 1), q = lane >> 2;
      float acc = 0.0f;
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) {
        const int o = 4 * q + i2;
        const float h = fmaxf(FCP[o * NBF + cl] + FCP[64 * NBF + o * NBF + cl], 0.0f);
        acc = __builtin_fmaf(buf_load(rs, 16 * q, 4 * (kPkF2 + i2)), h, acc);
      }
      acc += __shfl_xor(acc, 4, 64);
      acc += __shfl_xor(acc, 8, 64);
      acc += __shfl_xor(acc, 16, 64);
      acc += __shfl_xor(acc, 32, 64);
      const int64_t i = b * NBF + cl;
      if (q == 0 && i < n_mine) logits[(int64_t)blockIdx.x + G * i] = acc;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kFusedBlock, 4) void wk_fused_kernel(const T* __restrict__ audio, int64_t batch,
                                                                 int64_t clip_stride, const float* __restrict__ wts,
                                                                 float* __restrict__ logits,
                                                                 float* __restrict__ feats_out) {
  __shared__ __attribute__((aligned(16))) float smem[kFusedLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  fe_init_tables<true>(smem, tid, kFusedBlock);
  for (int i = tid; i < kFusedLds - kF0Off; i += kFusedBlock) smem[kF0Off + i] = 0.0f;  // guards, pads, ctrl
  __syncthreads();
  const int64_t n_mine = batch > (int64_t)blockIdx.x ? (batch - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (wave < 8) {
#ifndef WK_EXPERIMENT_NO_FE
    fe_role<T>(smem, audio, n_mine, clip_stride, feats_out, wave, lane);
#endif
  } else {
#ifndef WK_EXPERIMENT_NO_CNN
    cnn_role(smem, wts, n_mine, logits, wave - 8, lane);
#endif
  }
}

}  // namespace

namespace wk {

hipError_t launch_fused(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                        float* logits, float* feats_or_null, int grid_cap, hipStream_t stream) {
  if (batch == 0) return hipSuccess;
  const int grid = (int)(batch < grid_cap ? batch : grid_cap);
  if (i16)
    hipLaunchKernelGGL(wk_fused_kernel<int16_t>, dim3(grid), dim3(kFusedBlock), 0, stream, (const int16_t*)audio,
                       batch, clip_stride, w, logits, feats_or_null);
  else
    hipLaunchKernelGGL(wk_fused_kernel<float>, dim3(grid), dim3(kFusedBlock), 0, stream, (const float*)audio, batch,
                       clip_stride, w, logits, feats_or_null);
  return hipGetLastError();
}

}  // namespace wk
