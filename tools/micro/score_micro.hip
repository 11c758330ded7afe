// Development micro-benchmark (not part of the library): the cov-mode score GEMM of a fast slot
// at d = 1000 (D = 1024: ((-mu) cov)^T read k-major times I - W, split-K slices) alone,
// hipEvent-timed back to back, against the split-K counts and rocBLAS dgemm of the same shape;
// "cold": the B operand rewritten by a kernel before each launch (as build_at does in the slot).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../midagma_amd/csrc
//          score_micro.hip ../../midagma_amd/csrc/gemm.hip -lrocblas -o score_micro
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>

#include "launch.h"

using namespace midagma;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void fill_kernel(double* p, int64_t n, uint64_t seed, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    p[i] = scale * ((double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5);
  }
}

template <class F>
static double time_us(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

int main() {
  const int64_t D = 1024, K = 1008;
  gemm_setup_attributes();
  double *A, *B, *C, *W;
  CK(hipMalloc(&A, 8 * D * D));
  CK(hipMalloc(&B, 8 * D * D));
  CK(hipMalloc(&W, 8 * D * D));
  CK(hipMalloc(&C, 8 * D * D * 8));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, A, D * D, 1, 1.0);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, B, D * D, 2, 1.0);
  const int reps = 200;
  const double f = 2.0 * D * D * K;
  for (int split : {1, 2, 4, 8}) {
    const double us = time_us([&] { launch_gemm(D, D, K, A, D, true, B, D, B_PLAIN, C, D, EPI_STORE, split, D * D,
                                                nullptr, 0, 0, nullptr, 0); }, reps);
    const double cold = time_us([&] {
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, B, D * D, 3, 1.0);
      launch_gemm(D, D, K, A, D, true, B, D, B_PLAIN, C, D, EPI_STORE, split, D * D, nullptr, 0, 0, nullptr, 0);
    }, reps);
    const double fill = time_us([&] { hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, B, D * D, 3, 1.0); },
                                reps);
    printf("split %d: %.2f us (%.1f TF) back to back; after a B rewrite %.2f us (fill alone %.2f)\n", split, us,
           f / us / 1e6, cold - fill, fill);
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  const double one = 1.0, zero = 0.0;
  const double us = time_us([&] {
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, D, D, K, &one, B, D, A, D, &zero, C, D);
  }, reps);
  printf("rocblas dgemm %ldx%ldx%ld: %.2f us (%.1f TF)\n", (long)D, (long)D, (long)K, us, f / us / 1e6);
  return 0;
}
