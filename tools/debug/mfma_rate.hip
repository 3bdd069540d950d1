// MFMA issue-rate and MFMA/VALU co-issue microbenchmark (dev tool).
//   hipcc -O3 --offload-arch=gfx950 mfma_rate.hip -o mfma_rate && ./mfma_rate
// Per MFMA kind: (1) cycles per MFMA, one wave per SIMD, 4 independent
// accumulators; (2) the same MFMA stream beside VW VALU waves per SIMD that
// run independent v_fma_f32 chains -- how many VALU cycles an MFMA takes from
// the other waves of its SIMD (the fused kernel runs 2 front-end VALU waves
// beside 2 CNN MFMA waves on every SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

enum { K_F32 = 0, K_BF16_K16 = 1, K_BF16_K32 = 2, K_F16_K32 = 3, K_NONE = 4 };
static const char* kName[] = {"f32_16x16x4", "bf16_16x16x16_1k", "bf16_16x16x32", "f16_16x16x32", "none"};

template <int KIND>
__device__ __forceinline__ void mfma_loop(int iters, float seed, float* out) {
  f32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  const float a = seed, b = seed + 1.0f;
  s4 a4, b4;
  bf8 a8, b8;
  h8 ha, hb;
  for (int i = 0; i < 4; ++i) { a4[i] = (short)(0x3f80 + i); b4[i] = (short)(0x3f00 + i); }
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(seed + i); b8[i] = (__bf16)(seed - i); ha[i] = (_Float16)(seed + i); hb[i] = (_Float16)(seed * i); }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (KIND == K_F32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
        else if constexpr (KIND == K_BF16_K16) acc[q] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[q], 0, 0, 0);
        else if constexpr (KIND == K_BF16_K32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[q], 0, 0, 0);
        else if constexpr (KIND == K_F16_K32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[q], 0, 0, 0);
      }
    }
  }
  float s = 0;
  for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  *out = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
// 64 v_fma_f32 per iteration, or (PK) the same 128 flop-lanes as 32 v_pk_fma_f32.
template <bool PK>
__device__ __forceinline__ void valu_loop(int iters, float seed, float* out) {
  float a[8];
  f2 p[4];
  for (int i = 0; i < 8; ++i) a[i] = seed + i;
  for (int i = 0; i < 4; ++i) p[i] = f2{seed + i, seed - i};
  const float m = 0.999f, c = 1e-4f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if constexpr (PK) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = __builtin_elementwise_fma(p[i], f2{m - i * 1e-6f, m}, f2{c, c});
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_fmaf(a[i], m - i * 1e-6f, c);
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  for (int i = 0; i < 4; ++i) s += p[i].x + p[i].y;
  *out = s;
}

// Waves 0..4*MW-1: MFMA loop (16 MFMAs per iteration); the rest: VALU loop
// (64 v_fma_f32 per iteration).  cyc[0] = mean MFMA-wave cycles, cyc[1] = mean VALU-wave cycles (block 0).
template <int KIND, bool PK>
__global__ void k(float* out, int m_iters, int v_iters, int mfma_waves, unsigned long long* cyc) {
  const int wave = threadIdx.x >> 6;
  const float seed = threadIdx.x * 1e-3f;
  float* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < mfma_waves) {
    if constexpr (KIND != K_NONE) mfma_loop<KIND>(m_iters, seed, o);
  } else {
    valu_loop<PK>(v_iters, seed, o);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) atomicAdd(&cyc[wave < mfma_waves ? 0 : 1], t1 - t0);
}

template <int KIND, bool PK = false>
void run(float* out, unsigned long long* cyc, int mw, int vw, int m_iters, int v_iters) {
  const int ncu = 256;
  const int threads = 64 * 4 * (mw + vw);
  unsigned long long h[2] = {0, 0};
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(cyc, 0, 16);
    hipLaunchKernelGGL((k<KIND, PK>), dim3(ncu), dim3(threads), 0, 0, out, m_iters, v_iters, 4 * mw, cyc);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
  const double mc = mw ? (double)h[0] / (4 * mw) : 0, vc = vw ? (double)h[1] / (4 * vw) : 0;
  const double n_mfma = (double)m_iters * 16, n_valu = (double)v_iters * 64;
  printf("%s %-18s mfma_waves/SIMD=%d valu_waves/SIMD=%d | mfma wave: %9.0f cyc, %6.2f cyc/MFMA/SIMD | valu wave: %9.0f cyc, "
         "%5.2f cyc/v_fma/SIMD\n",
         PK ? "pk " : "fma", kName[KIND], mw, vw, mc, mw ? mc / (n_mfma * mw) : 0.0, vc, vw ? vc / (n_valu * vw) : 0.0);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 16);
  const int m_iters = 2000, v_iters = 2000;
  // VALU waves alone (2/SIMD), then beside one MFMA wave per SIMD: plain vs packed FMA.
  run<K_NONE, false>(out, cyc, 0, 2, 0, v_iters);
  run<K_NONE, true>(out, cyc, 0, 2, 0, v_iters);
  run<K_F32, false>(out, cyc, 1, 2, m_iters / 4, v_iters);
  run<K_F32, true>(out, cyc, 1, 2, m_iters / 4, v_iters);
  run<K_BF16_K16, false>(out, cyc, 1, 2, m_iters, v_iters);
  run<K_BF16_K16, true>(out, cyc, 1, 2, m_iters, v_iters);
  run<K_NONE, false>(out, cyc, 0, 1, 0, v_iters);
  run<K_NONE, true>(out, cyc, 0, 1, 0, v_iters);
  run<K_F32, false>(out, cyc, 1, 1, m_iters / 4, v_iters);
  run<K_F32, true>(out, cyc, 1, 1, m_iters / 4, v_iters);
  return 0;
}
