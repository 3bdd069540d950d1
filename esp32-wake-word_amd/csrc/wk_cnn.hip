// wk_cnn.hip -- the xiaoa CNN (LightweightKWS, ml_models/src/wakeModel.py:4-34)
// on gfx950 fp32 matrix cores.
//
//   conv(13->32,k3,p1) ReLU maxpool2 -> conv(32->64) ReLU pool -> conv(64->128)
//   ReLU pool -> mean over time -> Linear(128,64) ReLU -> Linear(64,1)
//
// Every conv is a GEMM D[co][t] = sum_k W[co][k] X[k][t], k = (tap, ci), run
// with v_mfma_f32_16x16x4_f32 (exact fp32 fma chains, 16 co x 16 t per
// instruction).  The weights (157 KB fp32) are too big for LDS next to the
// activations, so they live in VGPRs: each of the 8 waves of a workgroup holds
// the A fragments of the output-channel tile(s) it owns (100 VGPRs / lane),
// loaded once per persistent workgroup.  Activations of a batch of 16 clips
// stay in LDS as [ci][clip][t + guards] images (guard columns = the conv
// zero padding; ci pitch = 16 mod 32 banks so the two 16-lane halves of a
// B-fragment read hit disjoint banks).  ReLU + maxpool run on the
// accumulators (pool partner = adjacent lane, DPP quad_perm), GAP is a
// 16-lane row reduction, and the two Linear layers are one more MFMA pass
// plus a wave reduction.
#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_cnn_dev.h"

using namespace wk;

namespace {

constexpr int NB = 16;           // clips per workgroup iteration
constexpr int kCnnBlock = 512;   // 8 waves
// LDS images (floats).
constexpr int A0_CLIP = 66, A0_CI = 16 * 66 + 16;   // conv1 input  [16 ci][16][66]
constexpr int A1_CLIP = 34, A1_CI = 16 * 34 + 16;   // conv2 input  [32 ci][16][34]
constexpr int A2_CLIP = 18, A2_CI = 16 * 18 + 16;   // conv3 input  [64 ci][16][18]
constexpr int A0_SIZE = 16 * A0_CI;                 // 17152
constexpr int A1_SIZE = 32 * A1_CI;                 // 17920
constexpr int A2_SIZE = 64 * A2_CI;                 // 19456
constexpr int R0_SIZE = A2_SIZE > A0_SIZE ? A2_SIZE : A0_SIZE;  // act0 / act2 / fc partials
constexpr int FCP_OFF = A0_SIZE;                    // fc1 partials [2][64][16] behind act0
constexpr int G_SIZE = 128 * NB;
constexpr int LDS_FLOATS = R0_SIZE + A1_SIZE + G_SIZE;
static_assert(FCP_OFF + 2 * 64 * NB <= R0_SIZE, "fc partials must fit in region 0");
static_assert(LDS_FLOATS * 4 <= 163840, "LDS budget");

__global__ __launch_bounds__(kCnnBlock, 2) void wk_cnn_kernel(const float* __restrict__ feats, int64_t batch,
                                                             const float* __restrict__ wts,
                                                             float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];
  float* R0 = smem;                 // act0 (conv1 in) / act2 (conv3 in) / fc partials
  float* A1 = smem + R0_SIZE;       // act1 (conv2 in)
  float* G = A1 + A1_SIZE;          // pooled features [128][16]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;

  // ---- weights -> VGPRs (A fragments: row co = co0 + li, k = 4s + lk) ----
  float w1[12], w2[24], w3[48], wf1[16];
  {
    const int co = 16 * (wave & 1) + li;
#pragma unroll
    for (int s = 0; s < 12; ++s) {
      const int tap = s >> 2, ci = 4 * (s & 3) + lk;
      w1[s] = ci < 13 ? wts[kOffW1 + (co * 13 + ci) * 3 + tap] : 0.0f;
    }
  }
  {
    const int co = 16 * (wave & 3) + li;
#pragma unroll
    for (int s = 0; s < 24; ++s) w2[s] = wts[kOffW2 + (co * 32 + 4 * (s & 7) + lk) * 3 + (s >> 3)];
  }
  {
    const int co = 16 * wave + li;
#pragma unroll
    for (int s = 0; s < 48; ++s) w3[s] = wts[kOffW3 + (co * 64 + 4 * (s & 15) + lk) * 3 + (s >> 4)];
  }
  {
    const int o = 16 * (wave & 3) + li, kh = wave >> 2;
#pragma unroll
    for (int s = 0; s < 16; ++s) wf1[s] = wts[kOffF1 + o * 128 + 64 * kh + 4 * s + lk];
  }

  const int64_t n_iter = (batch + NB - 1) / NB;
  for (int64_t it = blockIdx.x; it < n_iter; it += gridDim.x) {
    const int64_t clip0 = it * NB;
    // ---- 1. features -> act0 image (zeros in guards / padded ci); act1 guards ----
    for (int idx = tid; idx < A0_SIZE; idx += kCnnBlock) {
      const int ci = idx / A0_CI, rem = idx - ci * A0_CI;
      const int cl = rem / A0_CLIP, col = rem - cl * A0_CLIP;
      float v = 0.0f;
      if (ci < 13 && cl < NB && col >= 1 && col <= 63 && clip0 + cl < batch)
        v = feats[(clip0 + cl) * (13 * 63) + ci * 63 + col - 1];
      R0[idx] = v;
    }
    for (int idx = tid; idx < 32 * NB * 3; idx += kCnnBlock) {
      const int row = idx / 3, e = idx - row * 3;
      const int ci = row / NB, cl = row - ci * NB;
      A1[ci * A1_CI + cl * A1_CLIP + (e == 0 ? 0 : 31 + e)] = 0.0f;
    }
    __syncthreads();

    // ---- 2. conv1: co tile (wave&1), clips 4*(wave>>1).., 4 t-tiles each ----
    {
      const int co0 = 16 * (wave & 1);
      const int lp = lk * A0_CI + li;
#pragma unroll 1
      for (int p = 0; p < 8; ++p) {
        const int cl = 4 * (wave >> 1) + (p >> 1);
        const int ta = 32 * (p & 1), tb = ta + 16;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<12, A0_CI, 4>(R0, w1, lp + cl * A0_CLIP + ta, lp + cl * A0_CLIP + tb, acc_a, acc_b);
        epi_pool<A1_CI, A1_CLIP, 31>(acc_a, A1, co0, cl, ta, lane);
        epi_pool<A1_CI, A1_CLIP, 31>(acc_b, A1, co0, cl, tb, lane);
      }
    }
    __syncthreads();

    // ---- 3. act2 guards (region 0 is free now); conv2 ----
    for (int idx = tid; idx < 64 * NB * 3; idx += kCnnBlock) {
      const int row = idx / 3, e = idx - row * 3;
      const int ci = row / NB, cl = row - ci * NB;
      R0[ci * A2_CI + cl * A2_CLIP + (e == 0 ? 0 : 15 + e)] = 0.0f;
    }
    {
      const int co0 = 16 * (wave & 3);
      const int lp = lk * A1_CI + li;
#pragma unroll 1
      for (int p = 0; p < 8; ++p) {
        const int cl = 8 * (wave >> 2) + p;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<24, A1_CI, 8>(A1, w2, lp + cl * A1_CLIP, lp + cl * A1_CLIP + 16, acc_a, acc_b);
        epi_pool<A2_CI, A2_CLIP, 15>(acc_a, R0, co0, cl, 0, lane);
        epi_pool<A2_CI, A2_CLIP, 15>(acc_b, R0, co0, cl, 16, lane);
      }
    }
    __syncthreads();

    // ---- 4. conv3: co tile = wave, one t-tile per clip; GAP -> G ----
    {
      const int co0 = 16 * wave;
      const int lp = lk * A2_CI + li;
#pragma unroll 1
      for (int p = 0; p < NB / 2; ++p) {
        const int ca = 2 * p, cb = 2 * p + 1;
        f32x4 acc_a = {0, 0, 0, 0}, acc_b = {0, 0, 0, 0};
        conv_pair<48, A2_CI, 16>(R0, w3, lp + ca * A2_CLIP, lp + cb * A2_CLIP, acc_a, acc_b);
        epi_gap<NB>(acc_a, G, co0, ca, lane);
        epi_gap<NB>(acc_b, G, co0, cb, lane);
      }
    }
    __syncthreads();

    // ---- 5. classifier.0 (128 -> 64): o tile (wave&3), k half (wave>>2) ----
    {
      f32x4 acc = {0, 0, 0, 0};
      const int kh = wave >> 2;
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma4(wf1[s], G[(64 * kh + 4 * s + lk) * NB + li], acc);
      float* fcp = R0 + FCP_OFF + kh * 64 * NB;
#pragma unroll
      for (int r = 0; r < 4; ++r) fcp[(16 * (wave & 3) + 4 * lk + r) * NB + li] = acc[r];
    }
    __syncthreads();

    // ---- 6. ReLU -> classifier.2 (64 -> 1) ----
    if (wave == 0) {
      const float* fcp = R0 + FCP_OFF;
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 16 * lk + i;
        const float h = fmaxf(fcp[o * NB + li] + fcp[64 * NB + o * NB + li], 0.0f);
        s = __builtin_fmaf(wts[kOffF2 + o], h, s);
      }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lk == 0 && clip0 + li < batch) logits[clip0 + li] = s;
    }
  }
}

}  // namespace

namespace wk {

hipError_t launch_cnn(const float* feats, int64_t batch, const float* w, float* logits, bool bf16, int grid_cap,
                      hipStream_t stream) {
  if (bf16) return hipErrorNotSupported;
  const int64_t n_iter = (batch + NB - 1) / NB;
  if (n_iter == 0) return hipSuccess;
  const int grid = (int)(n_iter < grid_cap ? n_iter : grid_cap);
  hipLaunchKernelGGL(wk_cnn_kernel, dim3(grid), dim3(kCnnBlock), 0, stream, feats, batch, w, logits);
  return hipGetLastError();
}

}  // namespace wk
