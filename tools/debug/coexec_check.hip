// Co-execution correctness check (dev tool): do MFMAs on some waves of a SIMD
// change the results of VALU work on other waves of the same SIMD?
//   hipcc -O3 --offload-arch=gfx950 coexec_check.hip -o coexec_check && ./coexec_check
// Waves 0-3 (one per SIMD) run an MFMA loop of the given kind (or nothing);
// waves 4-11 run a deterministic VALU workload (plain fp32 FMA chains, packed
// fp32 v_pk_fma/v_pk_mul chains, DPP row moves) and store their final values.
// The VALU results must be bit-identical whatever the MFMA waves do.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

enum { K_NONE = 0, K_BF16_K16 = 1, K_BF16_K32 = 2, K_F32 = 3 };

template <int KIND>
__device__ void mfma_loop(int iters, float seed, float* out) {
  f32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  s4 a4, b4;
  bf8 a8, b8;
  for (int i = 0; i < 4; ++i) { a4[i] = (short)(0x3f80 + i); b4[i] = (short)(0x3f00 + i); }
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(seed + i); b8[i] = (__bf16)(seed - i); }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (KIND == K_BF16_K16) acc[q] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[q], 0, 0, 0);
      else if constexpr (KIND == K_BF16_K32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[q], 0, 0, 0);
      else if constexpr (KIND == K_F32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(seed, seed + 1.0f, acc[q], 0, 0, 0);
    }
  }
  float s = 0;
  for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  *out = s;
}

__device__ float valu_work2(int iters, int lane, int wave, float* lds) {
  // transcendentals, op_sel/neg packed FMA (the front-end's cmul2), and an
  // in-wave LDS transpose (ds_write then ds_read of other lanes' words, no waitcnt between)
  float x = 1.0f + 0.01f * lane + wave;
  f2 p = f2{x, 0.5f * x};
  float* row = lds + (wave - 4) * 64 * 17;
  for (int it = 0; it < iters; ++it) {
    float l = __builtin_amdgcn_logf(x + 1.0f) * 0.69314718f;
    float e = __builtin_amdgcn_exp2f(-l);
    x = __builtin_fmaf(l, 0.5f, e) + 1.0f;
    f2 t = p * f2{x, x};
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(p), "v"(f2{0.6f, 0.8f}), "v"(t));
    p = r * f2{0.5f, 0.5f} + f2{0.25f, -0.25f};
    row[(lane & 15) * 17 + (lane >> 4)] = p.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float q = row[(lane >> 4) * 17 + (lane & 15)];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    p.y += 1e-3f * q;
  }
  return x + p.x + p.y;
}

__device__ float valu_work(int iters, int lane, int wave) {
  float a[4];
  f2 p[4];
  for (int i = 0; i < 4; ++i) {
    a[i] = 0.1f * lane + 0.01f * i + wave;
    p[i] = f2{a[i], -a[i] * 0.5f};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = __builtin_fmaf(a[i], 0.9999f, 1e-3f * i);
      p[i] = __builtin_elementwise_fma(p[i], f2{0.99991f, 1.00003f}, f2{1e-4f, -2e-4f});
      p[i] = p[i] * f2{1.0000001f, 0.9999999f};
      const float r = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a[i]), 0x121, 0xF, 0xF, false));
      a[i] += 1e-7f * r;
    }
  }
  float s = 0;
  for (int i = 0; i < 4; ++i) s += a[i] + p[i].x + p[i].y;
  return s;
}

template <int KIND>
__global__ void k(float* out, float* sink, int m_iters, int v_iters) {
  __shared__ float lds[8 * 64 * 17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave < 4) {
    if constexpr (KIND != K_NONE) mfma_loop<KIND>(m_iters, lane * 1e-3f, sink + blockIdx.x * 256 + threadIdx.x);
  } else if (wave < 8) {
    out[(blockIdx.x * 8 + (wave - 4)) * 64 + lane] = valu_work(v_iters, lane, wave);
  } else {
    out[(blockIdx.x * 8 + (wave - 4)) * 64 + lane] = valu_work2(v_iters / 4, lane, wave, lds);
  }
}

int main() {
  const int ncu = 256, n = ncu * 8 * 64;
  float *out, *sink;
  hipMalloc(&out, n * 4);
  hipMalloc(&sink, ncu * 256 * 4);
  std::vector<float> ref(n), got(n);
  const int v_iters = 20000, m_iters = 20000;
  hipLaunchKernelGGL(k<K_NONE>, dim3(ncu), dim3(768), 0, 0, out, sink, m_iters, v_iters);
  hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost);
  const char* names[] = {"none", "bf16_16x16x16_1k", "bf16_16x16x32", "f32_16x16x4"};
  for (int kind = 0; kind < 4; ++kind)
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(out, 0, n * 4);
      if (kind == 0) hipLaunchKernelGGL(k<K_NONE>, dim3(ncu), dim3(768), 0, 0, out, sink, m_iters, v_iters);
      if (kind == 1) hipLaunchKernelGGL(k<K_BF16_K16>, dim3(ncu), dim3(768), 0, 0, out, sink, m_iters, v_iters);
      if (kind == 2) hipLaunchKernelGGL(k<K_BF16_K32>, dim3(ncu), dim3(768), 0, 0, out, sink, m_iters, v_iters);
      if (kind == 3) hipLaunchKernelGGL(k<K_F32>, dim3(ncu), dim3(768), 0, 0, out, sink, m_iters / 2, v_iters);
      hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int i = 0; i < n; ++i) bad += memcmp(&ref[i], &got[i], 4) != 0;
      printf("MFMA waves: %-18s rep %d: %d of %d VALU lane results differ from the MFMA-free run\n", names[kind], rep,
             bad, n);
    }
  return 0;
}
