// Minimal co-residence probe for the K = 32 question.
//
// The fused kernel's front-end values change run to run when its CNN waves
// use the K = 32 MFMA forms (v_mfma_f32_16x16x32_{bf16,f16}) on the same SIMDs,
// and not with the K = 16 pair.  This program asks whether that needs the
// fused kernel at all: one 1,024-thread workgroup per CU, waves 0-7 run a
// deterministic packed-fp32 VALU chain (v_pk_fma_f32 / v_pk_mul_f32 rotations,
// a DPP row_mirror exchange and an LDS round trip per iteration, the front-end's
// instruction mix), waves 8-15 run an MFMA stream for as long as any VALU wave
// is running.  Every wave index maps to SIMDs as in the fused kernel (two of
// each role per SIMD).  The VALU results must not depend on the MFMA form.
//
//   hipcc -O3 --offload-arch=gfx950 -o xdl_probe tools/debug/xdl_coresidence_probe.hip
//   ./xdl_probe [repeats] [iterations] [variant bits 0-31]
//
// Prints, per MFMA mode and repeat, how many VALU lanes differ from mode 0
// (no MFMA stream) and the lane histogram of the differences.
// Diagnostic tool, not product code.
#include <hip/hip_runtime.h>

#ifndef WK_PROBE_CHAINS
#define WK_PROBE_CHAINS 8   // packed-fp32 chains per VALU lane (-DWK_PROBE_CHAINS=48: ~110 VGPRs, the front-end's register range)
#endif

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 1024, kValuWaves = 8, kChains = WK_PROBE_CHAINS;
constexpr int kLdsFloats = 24 * 1024;   // ~96 KB: one workgroup per CU

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul_swap_neg(f32x2 a, f32x2 b) {   // {-a.y * b.x, a.x * b.y}
  f32x2 d;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ f32x2 pk_fma_s(f32x2 a, f32x2 b_sgpr, f32x2 c) {   // a constant in an SGPR pair
  f32x2 d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_sgpr), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul_swap_neg_s(f32x2 a, f32x2 b_sgpr) {
  f32x2 d;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(a), "s"(b_sgpr));
  return d;
}
__device__ __forceinline__ float dpp_shr1_keep(float old, float x) {   // row_shr:1, bound_ctrl off: lane 0 of a row keeps old
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x),
                                                               0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_mirror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xf, 0xf, false));
}

// MODE 0: no MFMA stream, 1: K = 16 bf16 pair, 2: K = 32 bf16, 3: K = 32 f16.
// VAR bits (0 = VGPR constants, row_mirror only): 1 = SGPR-pair constants and
// the split's row_mirror -> row_shr:1 (bound_ctrl off) pair; 2 = v_log_f32 /
// v_exp_f32 and a lane select per iteration; 4 = the MFMA waves read their B
// operand from LDS and store their accumulators to LDS (the CNN role's epilogue
// stores), in their own LDS range.
// 8 = each iteration adds a value loaded from global memory (a buffer load into
// VGPRs, as the front-end's audio loads) and a 64-bit LDS table read (its
// twiddles); 16 = the MFMA waves leave ~3/4 of their issue time idle
// (s_sleep between groups of MFMAs, the CNN role's MFMA share) instead of a
// dense stream.
template <int MODE>
__global__ __launch_bounds__(kThreads) void probe_kernel(int iters, int VAR, const float* __restrict__ table,
                                                         float* __restrict__ out, float* __restrict__ mout,
                                                         unsigned* __restrict__ info) {
  __shared__ float lds[kLdsFloats];
  __shared__ unsigned done;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) done = 0;
  for (int i = tid; i < 1024; i += kThreads) lds[4096 + i] = 1e-3f * (float)((i * 37) % 101) - 0.05f;   // the LDS table
  __syncthreads();
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // hwreg(HW_REG_HW_ID)
  if (lane == 0) info[blockIdx.x * 16 + wave] = (hw >> 4) & 3u;   // the wave's SIMD
  if (wave < kValuWaves) {
    // rotations by a fixed angle: norm-preserving, so a perturbation persists
    const float c = 0.99875026f, s = 0.04997917f;   // cos / sin 0.05
    const f32x2 cc = {c, c}, ss = {s, s};
    f32x2 v[kChains];
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      const float a = 0.25f + 1e-3f * (float)((blockIdx.x * 64 + lane) % 977) + 0.01f * k;
      v[k] = f32x2{a, 1.0f - a};
    }
    float* my = lds + wave * 64 * 4;
    f32x2 sum = {0.0f, 0.0f};
    for (int it = 0; it < iters; ++it) {
      if (!(VAR & 1)) {
#pragma unroll
        for (int k = 0; k < kChains; ++k) v[k] = pk_fma(v[k], cc, pk_mul_swap_neg(v[k], ss));
      } else {
#pragma unroll
        for (int k = 0; k < kChains; ++k) v[k] = pk_fma_s(v[k], cc, pk_mul_swap_neg_s(v[k], ss));
      }
      // DPP exchange (the real-FFT split's partner fetch) and an LDS round trip
      float m = dpp_mirror(v[0].x);
      if (VAR & 1) m = dpp_shr1_keep(v[kChains - 1].y, m);
      if (VAR & 2) {
        const float l = __builtin_amdgcn_logf(fabsf(m) + 1.0f);
        m = (lane & 4) ? m : m + 1e-3f * __builtin_amdgcn_exp2f(-l);
      }
      if (VAR & 8) {
        const float g = table[(it * 64 + lane) & 4095];
        const f32x2 tw = reinterpret_cast<const f32x2*>(lds + 4096)[(it + lane) & 511];
        m = fmaf(g, tw.x, m) + tw.y;
      }
      my[lane] = m;
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
      const float back = my[63 - lane];
      sum = pk_fma(f32x2{m, back}, f32x2{1.0f, 1.0f}, sum);
    }
    f32x4* o = reinterpret_cast<f32x4*>(out) + ((size_t)blockIdx.x * kValuWaves + wave) * 64 * (kChains / 2 + 1);
#pragma unroll
    for (int k = 0; k < kChains; k += 2) o[(k / 2) * 64 + lane] = f32x4{v[k].x, v[k].y, v[k + 1].x, v[k + 1].y};
    o[(kChains / 2) * 64 + lane] = f32x4{sum.x, sum.y, 0.0f, 0.0f};
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0) atomicAdd(&done, 1u);
  } else {
    f32x4 acc[4] = {};
    s16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (short)(0x3f80 + ((lane + i) & 7));
      b[i] = (short)(0x3c00 + ((lane * 3 + i) & 7));
    }
    if (VAR & 4) {
      s16x8* dst = reinterpret_cast<s16x8*>(lds + 8192 + (wave - kValuWaves) * 1024);
      dst[lane] = b;
    }
    const int cap = 64 * iters + 4096;   // every wave leaves: bounded even if a VALU wave never signals
    if (MODE != 0) {
      for (int n = 0; n < cap; n += 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          f32x4& c = acc[j & 3];
          if (VAR & 4) {   // B from LDS (the waves' own range, beyond the VALU waves')
            const s16x8* src = reinterpret_cast<const s16x8*>(lds + 8192 + (wave - kValuWaves) * 1024);
            b = src[(lane + j) & 63];
          }
          if (MODE == 1) {
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 0, 1, 2, 3),
                                                          __builtin_shufflevector(b, b, 0, 1, 2, 3), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_shufflevector(a, a, 4, 5, 6, 7),
                                                          __builtin_shufflevector(b, b, 4, 5, 6, 7), c, 0, 0, 0);
          } else if (MODE == 2) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                        0, 0, 0);
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                       0, 0);
          }
        }
        if (VAR & 16) __builtin_amdgcn_s_sleep(8);
        if (VAR & 4) {   // epilogue-like stores of the accumulators
          f32x4* dst = reinterpret_cast<f32x4*>(lds + 8192 + (wave - kValuWaves) * 1024 + 256);
          dst[lane] = acc[0];
          dst[64 - 1 - lane] = acc[1];
        }
        if (__builtin_amdgcn_readfirstlane(*(volatile unsigned*)&done) >= (unsigned)kValuWaves) break;
      }
    }
    f32x4* o = reinterpret_cast<f32x4*>(mout) + ((size_t)blockIdx.x * (16 - kValuWaves) + (wave - kValuWaves)) * 64;
    o[lane] = acc[0] + acc[1] + acc[2] + acc[3];
  }
}

static void launch_mode(int mode, int var, int grid, int iters, const float* table, float* out, float* m,
                        unsigned* info) {
  switch (mode) {
    case 0: hipLaunchKernelGGL(probe_kernel<0>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 1: hipLaunchKernelGGL(probe_kernel<1>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    case 2: hipLaunchKernelGGL(probe_kernel<2>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
    default: hipLaunchKernelGGL(probe_kernel<3>, dim3(grid), dim3(kThreads), 0, 0, iters, var, table, out, m, info); break;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 4000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus;
  const size_t nv = (size_t)grid * kValuWaves * 64 * (kChains / 2 + 1) * 4, nm = (size_t)grid * 8 * 64 * 4;
  float *d_out, *d_m;
  unsigned* d_info;
  CHECK(hipMalloc(&d_out, nv * 4));
  CHECK(hipMalloc(&d_m, nm * 4));
  CHECK(hipMalloc(&d_info, (size_t)grid * 16 * 4));
  std::vector<float> ref(nv), got(nv), table(4096);
  for (int i = 0; i < 4096; ++i) table[i] = 1e-3f * (float)((i * 53) % 97) - 0.04f;
  float* d_table;
  CHECK(hipMalloc(&d_table, 4096 * 4));
  CHECK(hipMemcpy(d_table, table.data(), 4096 * 4, hipMemcpyHostToDevice));
  std::vector<unsigned> info((size_t)grid * 16);
  const int var = argc > 3 ? atoi(argv[3]) : 0;
  auto launch = [&](int mode) {
    CHECK(hipMemset(d_out, 0, nv * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    launch_mode(mode, var, grid, iters, d_table, d_out, d_m, d_info);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(got.data(), d_out, nv * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(info.data(), d_info, info.size() * 4, hipMemcpyDeviceToHost));
    return ms;
  };
  launch(0);
  ref = got;
  {   // the role placement: VALU and MFMA waves per SIMD in workgroup 0
    int cnt[4][2] = {};
    for (int w = 0; w < 16; ++w) cnt[info[w] & 3][w >= kValuWaves]++;
    printf("workgroup 0 placement (valu, mfma) per SIMD: (%d,%d) (%d,%d) (%d,%d) (%d,%d)\n", cnt[0][0], cnt[0][1],
           cnt[1][0], cnt[1][1], cnt[2][0], cnt[2][1], cnt[3][0], cnt[3][1]);
  }
  printf("valu variant %d, %d iterations\n", var, iters);
  const char* names[4] = {"none", "k16_bf16_pair", "k32_bf16", "k32_f16"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int r = 0; r < reps; ++r) {
      const float ms = launch(mode);
      long diff = 0;
      int hist[64] = {};
      const size_t per_wave = 64 * (kChains / 2 + 1) * 4;
      for (size_t i = 0; i < nv; ++i)
        if (memcmp(&got[i], &ref[i], 4) != 0) {
          ++diff;
          hist[(i % per_wave) / 4 % 64]++;
        }
      printf("mode %-14s rep %d: %.3f ms, differing values %ld", names[mode], r, ms, diff);
      if (diff) {
        printf("; by lane:");
        for (int l = 0; l < 64; ++l)
          if (hist[l]) printf(" %d:%d", l, hist[l]);
      }
      printf("\n");
      fflush(stdout);
    }
  }
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_m));
  CHECK(hipFree(d_info));
  return 0;
}
