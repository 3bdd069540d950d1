// VALU issue-rate microbenchmark (dev tool): waves/SIMD x {v_fma_f32, v_pk_fma_f32}.
//   hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ void k(float* out, int iters, unsigned long long* cyc) {
  float a[8];
  f2 b[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; b[i] = f2{a[i], a[i] + 1.0f}; }
  const float m = 0.999f, c = 1e-4f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (PK) b[i] = __builtin_elementwise_fma(b[i], f2{m - i * 1e-6f, m}, f2{c, c});
        else a[i] = __builtin_fmaf(a[i], m - i * 1e-6f, c);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += PK ? b[i].x + b[i].y : a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  int ncu = 256;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 1024 * 4 * 8);
  hipMalloc(&cyc, 8);
  const int iters = 4000;
  for (int pk = 0; pk < 2; ++pk)
    for (int w = 1; w <= 4; w *= 2) {
      const int threads = 64 * 4 * w;   // w waves per SIMD, 1 WG per CU
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (pk) hipLaunchKernelGGL(k<true>, dim3(ncu), dim3(threads), 0, 0, out, iters, cyc);
        else hipLaunchKernelGGL(k<false>, dim3(ncu), dim3(threads), 0, 0, out, iters, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      const double instr_per_wave = (double)iters * 64;
      const double cyc_per_instr_per_simd = (double)c / (instr_per_wave * w);
      printf("%s waves/SIMD=%d: %.2f cycles per wave-instruction per SIMD (wave0 %llu cyc, %.3f ms)\n",
             pk ? "v_pk_fma_f32" : "v_fma_f32   ", w, cyc_per_instr_per_simd, c, ms);
    }
  return 0;
}
