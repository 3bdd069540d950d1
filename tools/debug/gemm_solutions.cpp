// Time every rocBLAS solution for the CTC input-projection GEMM shape
// (gi[rows][768] = x[rows][K] . W_ih[768][K]^T, fp16 in/out, fp32 compute),
// as wk_ctc.hip's gemm_nt issues it.  Dev tool:
//   hipcc -O2 --offload-arch=gfx950 tools/debug/gemm_solutions.cpp -lrocblas -o /tmp/gs && /tmp/gs 1232896 128
#define ROCBLAS_BETA_FEATURES_API
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 1232896, K = argc > 2 ? atoi(argv[2]) : 128, N = 768;
  rocblas_handle h;
  rocblas_create_handle(&h);
  void *A, *W, *C;
  hipMalloc(&A, M * K * 2); hipMalloc(&W, N * K * 2); hipMalloc(&C, M * N * 2);
  hipMemset(A, 0x2C, M * K * 2); hipMemset(W, 0x2C, N * K * 2);
  const float one = 1.0f, zero = 0.0f;
  auto run = [&](rocblas_gemm_algo algo, int32_t sol, uint32_t flags) {
    return rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &one, W, rocblas_datatype_f16_r,
                           K, A, rocblas_datatype_f16_r, K, &zero, C, rocblas_datatype_f16_r, N, C, rocblas_datatype_f16_r, N,
                           rocblas_datatype_f32_r, algo, sol, flags);
  };
  rocblas_int n = 0;
  rocblas_gemm_ex_get_solutions(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &one, W,
                                rocblas_datatype_f16_r, K, A, rocblas_datatype_f16_r, K, &zero, C, rocblas_datatype_f16_r, N,
                                C, rocblas_datatype_f16_r, N, rocblas_datatype_f32_r, rocblas_gemm_algo_solution_index,
                                rocblas_gemm_flags_none, nullptr, &n);
  std::vector<rocblas_int> sols(n);
  rocblas_gemm_ex_get_solutions(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &one, W,
                                rocblas_datatype_f16_r, K, A, rocblas_datatype_f16_r, K, &zero, C, rocblas_datatype_f16_r, N,
                                C, rocblas_datatype_f16_r, N, rocblas_datatype_f32_r, rocblas_gemm_algo_solution_index,
                                rocblas_gemm_flags_none, sols.data(), &n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto time_it = [&](rocblas_gemm_algo algo, int32_t sol) -> float {
    if (run(algo, sol, 0) != rocblas_status_success) return -1.0f;
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) run(algo, sol, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
  };
  printf("M=%lld K=%lld N=%lld: %d solutions; default %.4f ms\n", (long long)M, (long long)K, (long long)N, n,
         time_it(rocblas_gemm_algo_standard, 0));
  std::vector<std::pair<float, int>> t;
  for (int i = 0; i < n; ++i) {
    const float ms = time_it(rocblas_gemm_algo_solution_index, sols[i]);
    if (ms > 0) t.push_back({ms, sols[i]});
  }
  std::sort(t.begin(), t.end());
  for (size_t i = 0; i < t.size() && i < 8; ++i) printf("  solution %d: %.4f ms\n", t[i].second, t[i].first);
  fflush(stdout);
  return 0;
}
