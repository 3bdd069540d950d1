// wk_int8.hip -- the xiaoa CNN in the device's int8 arithmetic (SURVEY 8(f)
// item 3): esp-dl / esp-ppq power-of-2, symmetric, per-tensor int8
// (ml_models/xiaoa.json:1-40), exponents from ml_models/xiaoa.info:3139-3150.
//
//   input    q = clamp(lroundf(x * 2^4))                      exp -4  (TensorBase::assign)
//   conv k3  acc = sum q_x q_w (int32); q = clamp(rne(acc / 2^s)) s = e_x + e_w - e_out
//            ReLU fused, MaxPool(2) on int8
//            conv1: -4 -8 -> -5 (s = 7); conv2: -5 -9 -> -5 (s = 9); conv3: -5 -9 -> -4 (s = 10)
//   GAP      mean of 7, exp -4 -> -5: q = clamp(rne(2 s / 7))  (2s/7 never ties)
//   MatMul   128 -> 64, -5 -9 -> -4 (s = 10), ReLU; 64 -> 1, -4 -9 -> -3 (s = 10)
//   output   logit = q * 2^-3
//
// rne = round half to even (esp-ppq's default rounding policy): with it the
// network reproduces the reference's int8 known-answer test exactly
// (xiaoa.info test input -> -40, tests/golden/kat.npz), as it does for the
// int8 weights, which are rne(w * 2^-e) of xiaoa.onnx.  (Half-away requant
// with a truncating GAP would also give -40; floor or truncating requant
// would not.)  Parity: pinned by that single KAT; bit-exact against
// oracle.kws_forward_int8.
//
// One 256-thread block per clip (grid-stride), int8 weights (40 KB) staged in
// LDS, int32 dot products on the VALU -- a device-faithful checking mode, not
// the throughput path.
#include <math.h>
#include <stdlib.h>

#include "wk_common.h"
#include "wk_kernels.h"

namespace {

constexpr int kW0 = 3 * 13 * 32, kW3 = 3 * 32 * 64, kW6 = 3 * 64 * 128, kM23 = 128 * 64, kM24 = 64;

__device__ __forceinline__ int sat8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }

// acc / 2^s rounded half to even (s >= 1), then saturated.
__device__ __forceinline__ int rq(int acc, int s) {
  int q = acc >> s;                       // floor
  const int rem = acc - (q << s), half = 1 << (s - 1);
  q += (rem > half || (rem == half && (q & 1))) ? 1 : 0;
  return sat8(q);
}

// weights: int8 in logical layouts conv [k][ci][co], matmul [in][out] (quantize_int8_weights;
// the esp-dl export stores the same values in its (N/16)WC16 order)
__global__ __launch_bounds__(256) void wk_int8_cnn_kernel(const float* __restrict__ feats, int64_t batch,
                                                          const int8_t* __restrict__ wq, float* __restrict__ logits) {
  __shared__ int8_t w[kW0 + kW3 + kW6 + kM23 + kM24];
  __shared__ int x0[65][13];    // input, time-major, zero guard rows 0 and 64
  __shared__ int a1[33][32];    // pooled conv1, guards 0 and 32
  __shared__ int a2[17][64];    // pooled conv2, guards 0 and 16
  __shared__ int a3[7][128];    // pooled conv3
  __shared__ int g[128], hid[64];
  const int tid = threadIdx.x;
  for (int i = tid; i < (int)sizeof(w); i += 256) w[i] = wq[i];
  const int8_t* W0 = w;
  const int8_t* W3 = W0 + kW0;
  const int8_t* W6 = W3 + kW3;
  const int8_t* M23 = W6 + kW6;
  const int8_t* M24 = M23 + kM23;
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    __syncthreads();
    for (int i = tid; i < 65 * 13; i += 256) {
      const int t = i / 13, c = i - t * 13;
      x0[t][c] = (t == 0 || t == 64) ? 0 : sat8((int)lroundf(feats[b * (13 * 63) + c * 63 + (t - 1)] * 16.0f));
    }
    for (int i = tid; i < 32; i += 256) a1[0][i] = a1[32][i] = 0;
    for (int i = tid; i < 64; i += 256) a2[0][i] = a2[16][i] = 0;
    __syncthreads();
    for (int i = tid; i < 31 * 32; i += 256) {   // conv1 + ReLU + pool
      const int tp = i / 32, co = i - tp * 32;
      int m = 0;
      for (int d = 0; d < 2; ++d) {
        const int t = 2 * tp + d;
        int acc = 0;
        for (int k = 0; k < 3; ++k)
          for (int ci = 0; ci < 13; ++ci) acc += x0[t + k][ci] * (int)W0[(k * 13 + ci) * 32 + co];
        m = max(m, rq(acc, 7));
      }
      a1[tp + 1][co] = m;
    }
    __syncthreads();
    for (int i = tid; i < 15 * 64; i += 256) {   // conv2 + ReLU + pool
      const int tp = i / 64, co = i - tp * 64;
      int m = 0;
      for (int d = 0; d < 2; ++d) {
        const int t = 2 * tp + d;
        int acc = 0;
        for (int k = 0; k < 3; ++k)
          for (int ci = 0; ci < 32; ++ci) acc += a1[t + k][ci] * (int)W3[(k * 32 + ci) * 64 + co];
        m = max(m, rq(acc, 9));
      }
      a2[tp + 1][co] = m;
    }
    __syncthreads();
    for (int i = tid; i < 7 * 128; i += 256) {   // conv3 + ReLU + pool
      const int tp = i / 128, co = i - tp * 128;
      int m = 0;
      for (int d = 0; d < 2; ++d) {
        const int t = 2 * tp + d;
        int acc = 0;
        for (int k = 0; k < 3; ++k)
          for (int ci = 0; ci < 64; ++ci) acc += a2[t + k][ci] * (int)W6[(k * 64 + ci) * 128 + co];
        m = max(m, rq(acc, 10));
      }
      a3[tp][co] = m;
    }
    __syncthreads();
    if (tid < 128) {   // GAP: exp -4 -> -5, q = rne(2 s / 7) = floor(2 s / 7 + 1/2) (no ties; s >= 0)
      int s = 0;
      for (int t = 0; t < 7; ++t) s += a3[t][tid];
      g[tid] = sat8((4 * s + 7) / 14);
    }
    __syncthreads();
    if (tid < 64) {
      int acc = 0;
      for (int c = 0; c < 128; ++c) acc += g[c] * (int)M23[c * 64 + tid];
      hid[tid] = max(0, rq(acc, 10));
    }
    __syncthreads();
    if (tid < 64) {
      int v = hid[tid] * (int)M24[tid];
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (tid == 0) logits[b] = (float)rq(v, 10) * 0.125f;
    }
  }
}

// ---------------------------------------------------------------------------
// The same network on the int8 matrix cores (v_mfma_i32_16x16x64_i8): one
// wave per clip (grid-stride), 4 waves per block.  Each conv layer is a GEMM
// D[co][t] = W[co][K] X[K][t] with K = (k, ci), ci padded to 16 / 32 / 64 so
// that a lane group's 16 K-bytes are one 16-byte read of an activation row
// [t + k][ci0 .. ci0 + 15]; the weights of all three convs stay in VGPRs as A
// fragments (built once per wave from the staged [k][ci][co] bytes).  int32
// accumulation is exact, and the requantisation, ReLU, pool, GAP and FC steps
// are the checking kernel's integer code on the MFMA results, so the two
// kernels agree bit for bit (tests/test_gpu_int8.py).
// Fragment layout (16x16x64 i8): lane (li = l & 15, lg = l >> 4) holds A row
// li / B column li at K bytes 16 lg .. 16 lg + 15, and D column li, rows
// 4 lg .. 4 lg + 3.  (Any K order the hardware uses applies to A and B alike.)
// ---------------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kQW = 8;                        // waves per block (2 per SIMD)
constexpr int kX0 = 66 * 16, kA1 = 34 * 32, kA2 = 18 * 64;   // per-wave images: [t][ci] int8, zero guards

__device__ __forceinline__ int q_even(int v) {   // pool partner: the other lane of the pair (li ^ 1)
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ int row16_sum_i(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
  return v;
}
__device__ __forceinline__ unsigned pack4(int a, int b, int c, int d) {
  return (unsigned)(a & 255) | ((unsigned)(b & 255) << 8) | ((unsigned)(c & 255) << 16) | ((unsigned)(d & 255) << 24);
}

__global__ __launch_bounds__(64 * kQW) void wk_int8_mfma_kernel(const float* __restrict__ feats, int64_t batch,
                                                                 const int8_t* __restrict__ wq,
                                                                 float* __restrict__ logits) {
  __shared__ int8_t w[kW0 + kW3 + kW6 + kM23 + kM24];
  __shared__ __attribute__((aligned(16))) int8_t img[kQW][kX0 + kA1 + kA2 + 128];
  __shared__ i32x4 fimg[10][64];
  __shared__ int m23t[32][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  for (int i = tid; i < (int)sizeof(w); i += 64 * kQW) w[i] = wq[i];
  for (int i = tid; i < kQW * (kX0 + kA1 + kA2 + 128); i += 64 * kQW) (&img[0][0])[i] = 0;   // guards and pads stay 0
  __syncthreads();
  const int8_t* W0 = w;
  const int8_t* W3 = W0 + kW0;
  const int8_t* W6 = W3 + kW3;
  const int8_t* M23 = W6 + kW6;
  const int8_t* M24 = M23 + kM23;
  int8_t* x0 = img[wv];
  int8_t* a1 = x0 + kX0;
  int8_t* a2 = a1 + kA1;
  int8_t* gq = a2 + kA2;
  // A fragments: co = 16 ct + li, K bytes kk = 64 s + 16 lg + j -> (k, ci) = (kk / CIP, kk % CIP)
  auto frag = [&](const int8_t* W, int CI, int CIP, int CO, int ct, int st) {
    int b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int kk = 64 * st + 16 * lg + j, k = kk / CIP, ci = kk % CIP, co = 16 * ct + li;
      b[j] = (k < 3 && ci < CI) ? (int)W[(k * CI + ci) * CO + co] : 0;
    }
    return i32x4{(int)pack4(b[0], b[1], b[2], b[3]), (int)pack4(b[4], b[5], b[6], b[7]),
                 (int)pack4(b[8], b[9], b[10], b[11]), (int)pack4(b[12], b[13], b[14], b[15])};
  };
  // conv3's 24 fragments stay in VGPRs; conv1's 2 and conv2's 8 live in a
  // block-shared LDS image [fragment][lane] (each wave builds some of them)
  i32x4 f3[8][3];
#pragma unroll
  for (int ct = 0; ct < 8; ++ct)
#pragma unroll
    for (int st = 0; st < 3; ++st) f3[ct][st] = frag(W6, 64, 64, 128, ct, st);
  for (int fi = wv; fi < 10; fi += kQW)
    fimg[fi][lane] = fi < 2 ? frag(W0, 13, 16, 32, fi, 0) : frag(W3, 32, 32, 64, (fi - 2) >> 1, (fi - 2) & 1);
  __syncthreads();
  // classifier.0: lane o's column of M23 as 4-byte groups over c, [group][lane] in LDS
  for (int j = wv; j < 32; j += kQW)
    m23t[j][lane] = (int)pack4(M23[(4 * j) * 64 + lane], M23[(4 * j + 1) * 64 + lane], M23[(4 * j + 2) * 64 + lane],
                               M23[(4 * j + 3) * 64 + lane]);
  __syncthreads();
  const int m24 = M24[lane];
  const int64_t wstride = (int64_t)gridDim.x * kQW;
  for (int64_t b = (int64_t)blockIdx.x * kQW + wv; b < batch; b += wstride) {
    // input: x0[t + 1][c] = sat8(lround(16 x[c][t])), t < 63, c < 13
    const float* f = feats + b * (13 * 63);
#pragma unroll
    for (int m = 0; m < 13; ++m) {
      const int e = lane + 64 * m;   // < 832; 819 values
      if (e < 13 * 63) {
        const int c = e / 63, t = e - 63 * c;
        x0[(t + 1) * 16 + c] = (int8_t)sat8((int)lroundf(f[e] * 16.0f));
      }
    }
    wk::wave_lds_sync();
    // conv1 (s = 7): 4 column tiles of t, K = 3 x 16 (lane group 3: zeros)
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int t = 16 * tt + li;
      i32x4 bx = i32x4{0, 0, 0, 0};
      if (lg < 3) bx = *reinterpret_cast<const i32x4*>(x0 + (t + lg) * 16);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const i32x4 acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fimg[ct][lane], bx, i32x4{0, 0, 0, 0}, 0, 0, 0);
        int q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int v = rq(acc[i], 7);
          q[i] = max(0, max(v, q_even(v)));
        }
        const int tp = t >> 1;
        if (!(li & 1) && tp < 31) *reinterpret_cast<unsigned*>(a1 + (tp + 1) * 32 + 16 * ct + 4 * lg) = pack4(q[0], q[1], q[2], q[3]);
      }
    }
    wk::wave_lds_sync();
    // conv2 (s = 9): 2 column tiles, K = 2 steps over (k, ci < 32)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 16 * tt + li;
      i32x4 acc[4] = {};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int kk = 64 * st + 16 * lg, k = kk >> 5, ci0 = kk & 31;
        i32x4 bx = i32x4{0, 0, 0, 0};
        if (k < 3) bx = *reinterpret_cast<const i32x4*>(a1 + (t + k) * 32 + ci0);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          acc[ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fimg[2 + 2 * ct + st][lane], bx, acc[ct], 0, 0, 0);
      }
      const int tp = t >> 1;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        int q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int v = rq(acc[ct][i], 9);
          q[i] = max(0, max(v, q_even(v)));
        }
        if (!(li & 1) && tp < 15) *reinterpret_cast<unsigned*>(a2 + (tp + 1) * 64 + 16 * ct + 4 * lg) = pack4(q[0], q[1], q[2], q[3]);
      }
    }
    wk::wave_lds_sync();
    // conv3 (s = 10): one column tile (t < 14 used), K = 3 steps, one per tap;
    // pool, then GAP over the 7 pooled steps: a 16-lane row sum of the even lanes
    {
      i32x4 acc[8] = {};
#pragma unroll
      for (int st = 0; st < 3; ++st) {
        const i32x4 bx = *reinterpret_cast<const i32x4*>(a2 + (li + st) * 64 + 16 * lg);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) acc[ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f3[ct][st], bx, acc[ct], 0, 0, 0);
      }
      const bool live = !(li & 1) && li < 14;   // pooled step li / 2 < 7
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        int gs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int v = rq(acc[ct][i], 10);
          const int p = max(0, max(v, q_even(v)));
          const int sum = row16_sum_i(live ? p : 0);
          gs[i] = sat8((4 * sum + 7) / 14);   // GAP: exp -4 -> -5, rne(2 s / 7)
        }
        if (li == 0) *reinterpret_cast<unsigned*>(gq + 16 * ct + 4 * lg) = pack4(gs[0], gs[1], gs[2], gs[3]);
      }
    }
    wk::wave_lds_sync();
    // MatMul 128 -> 64 (s = 10) + ReLU: lane o, 32 dot4 over the broadcast g bytes
    int acc = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) acc = __builtin_amdgcn_sdot4(*reinterpret_cast<const int*>(gq + 4 * j), m23t[j][lane], acc, false);
    const int hid = max(0, rq(acc, 10));
    int v = hid * m24;   // MatMul 64 -> 1 (s = 10)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    if (lane == 0) logits[b] = (float)rq(v, 10) * 0.125f;
    wk::wave_lds_sync();   // this clip's images are read before the next clip's input overwrites x0
  }
}

}  // namespace

namespace wk {

hipError_t launch_int8_cnn(const float* feats, int64_t batch, const int8_t* wq, float* logits, int grid_cap,
                           hipStream_t stream) {
  if (batch == 0) return hipSuccess;
  static const bool checking = getenv("WAKEWORD_INT8_VALU") != nullptr;   // the one-block-per-clip VALU kernel (A/B, checks)
  if (checking) {
    const int grid = (int)(batch < grid_cap ? batch : grid_cap);
    hipLaunchKernelGGL(wk_int8_cnn_kernel, dim3(grid), dim3(256), 0, stream, feats, batch, wq, logits);
  } else {
    const int64_t blocks = (batch + kQW - 1) / kQW;
    const int grid = (int)(blocks < grid_cap ? blocks : grid_cap);
    hipLaunchKernelGGL(wk_int8_mfma_kernel, dim3(grid), dim3(64 * kQW), 0, stream, feats, batch, wq, logits);
  }
  return hipGetLastError();
}

// Quantise the fp32 state dict blob (WK_NUM_WEIGHTS layout) to the int8 export:
// rne(w * 2^-e) with the per-tensor weight exponents of xiaoa.info
// (conv -8, -9, -9; matmul -9, -9), re-laid out conv [k][ci][co], matmul [in][out].
void quantize_int8_weights(const float* w, int8_t* q) {
  auto qz = [](float v, int e) {
    const float s = ldexpf(v, -e);
    const long r = lrintf(s);   // round half to even (default rounding mode)
    return (int8_t)(r < -128 ? -128 : (r > 127 ? 127 : r));
  };
  int8_t* o = q;
  for (int k = 0; k < 3; ++k)
    for (int ci = 0; ci < 13; ++ci)
      for (int co = 0; co < 32; ++co) *o++ = qz(w[kOffW1 + (co * 13 + ci) * 3 + k], -8);
  for (int k = 0; k < 3; ++k)
    for (int ci = 0; ci < 32; ++ci)
      for (int co = 0; co < 64; ++co) *o++ = qz(w[kOffW2 + (co * 32 + ci) * 3 + k], -9);
  for (int k = 0; k < 3; ++k)
    for (int ci = 0; ci < 64; ++ci)
      for (int co = 0; co < 128; ++co) *o++ = qz(w[kOffW3 + (co * 64 + ci) * 3 + k], -9);
  for (int c = 0; c < 128; ++c)
    for (int oo = 0; oo < 64; ++oo) *o++ = qz(w[kOffF1 + oo * 128 + c], -9);
  for (int c = 0; c < 64; ++c) *o++ = qz(w[kOffF2 + c], -9);
}

}  // namespace wk
