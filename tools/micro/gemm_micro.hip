// Development micro-benchmark (not part of the library): the data-mode FP64 GEMM shapes
//   xw : Y[n x D] = X (I - W)   (A = X^T stored D x n, the library's form)
//   xty: Z[D x D] = X^T Y        (split-K 16, slices summed separately)
// timed with hipEvents for the library kernel, experimental variants and rocBLAS dgemm.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../midagma_amd/csrc
//          gemm_micro.hip ../../midagma_amd/csrc/gemm.hip -lrocblas -o gemm_micro
//   run  : ./gemm_micro [n] [which...]   which in {xw, xty, blas}
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "launch.h"
#include "gemm_exp.h"

using namespace midagma;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void maxdiff_kernel(const double* a, const double* b, int64_t n, unsigned long long* out) {
  double m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmax(m, fabs(a[i] - b[i]));
  atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

static double maxdiff(const double* a, const double* b, int64_t n) {
  unsigned long long* d;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(maxdiff_kernel, dim3(4096), dim3(256), 0, 0, a, b, n, d);
  unsigned long long h = 0;
  CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  double r;
  memcpy(&r, &h, 8);
  return r;
}

__global__ void fill_kernel(double* p, int64_t n, uint64_t seed, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = scale * ((double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5);
  }
}

static void fill(double* p, int64_t n, uint64_t seed, double scale) {
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, p, n, seed, scale);
  CK(hipGetLastError());
}

template <class F>
static double time_ms(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000064;  // rows (multiple of 128)
  std::vector<std::string> which;
  for (int i = 2; i < argc; ++i) which.push_back(argv[i]);
  if (which.empty()) which = {"xw", "xty", "blas"};
  auto want = [&](const char* w) {
    for (auto& s : which)
      if (s == w) return true;
    return false;
  };
  const int64_t D = 1024;
  const int split = 16;
  const int reps = 5;
  gemm_setup_attributes();
  double *XT, *X, *W, *IW, *Y, *Z, *Z2;
  CK(hipMalloc(&XT, sizeof(double) * D * n));
  CK(hipMalloc(&X, sizeof(double) * D * n));
  CK(hipMalloc(&Y, sizeof(double) * D * n));
  CK(hipMalloc(&W, sizeof(double) * D * D));
  CK(hipMalloc(&IW, sizeof(double) * D * D));
  CK(hipMalloc(&Z, sizeof(double) * D * D * split));
  CK(hipMalloc(&Z2, sizeof(double) * D * D));
  fill(X, D * n, 1, 2.0);
  fill(W, D * D, 2, 0.1);
  launch_transpose(X, D, n, D, XT, n, 0);
  CK(hipDeviceSynchronize());
  const double f = 2.0 * n * D * D;
  auto report = [&](const char* name, double ms) {
    printf("%-28s %9.3f ms  %6.2f TF  (%.1f%% of 78.6)\n", name, ms, f / ms / 1e9, 100.0 * f / ms / 1e9 / 78.6);
    fflush(stdout);
  };
  if (want("xw")) {
    report("xw  lib gemm128<T,IMINUS>", time_ms([&] {
             launch_gemm(n, D, D, XT, n, true, W, D, B_IMINUS, Y, D, EPI_STORE, 1, 0, nullptr, 0, 0, nullptr, 0);
           }, reps));
  }
  if (want("xty")) {
    report("xty lib gemm128<T,PLAIN>/16", time_ms([&] {
             launch_gemm(D, D, n, X, D, true, Y, D, B_PLAIN, Z, D, EPI_STORE, split, D * D, nullptr, 0, 0, nullptr,
                         0);
           }, reps));
  }
  double* Yref = nullptr;
  if (want("xw2") || want("xty2") || want("xw3") || want("xty3")) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw2_kernel<1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw2Lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw2_kernel<0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw2Lds));
    CK(hipMalloc(&Yref, sizeof(double) * D * n));
    launch_gemm(n, D, D, XT, n, true, W, D, B_IMINUS, Yref, D, EPI_STORE, 1, 0, nullptr, 0, 0, nullptr, 0);
    CK(hipDeviceSynchronize());
  }
  if (want("xw2")) {
    const int tm = (int)(n / 128), tn = (int)(D / 128);
    report("xw  exp xw2<IMINUS>", time_ms([&] {
             hipLaunchKernelGGL(exp::xw2_kernel<1>, dim3(tm * tn), dim3(256), exp::kXw2Lds, 0, D, D, tm, tn, XT, n,
                                W, D, Y, D, (int64_t)0);
           }, reps));
    CK(hipDeviceSynchronize());
    printf("    max|Y - Yref| = %.3e\n", maxdiff(Y, Yref, D * n));
  }
  if (want("xw3")) {
    const int tm = (int)(n / 128), tn = (int)(D / 128);
    report("xw  exp xw3<IMINUS>", time_ms([&] {
             hipLaunchKernelGGL(exp::xw3_kernel<1>, dim3(tm * tn), dim3(256), exp::kXw3Lds, 0, D, D, tm, tn, XT, n,
                                W, D, Y, D, (int64_t)0);
           }, reps));
    CK(hipDeviceSynchronize());
    printf("    max|Y - Yref| = %.3e\n", maxdiff(Y, Yref, D * n));
  }
  if (want("xw3p")) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<1, 1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<0, 1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    const int tm = (int)(n / 128), tn = (int)(D / 128);
    report("xw  exp xw3<IMINUS,prio>", time_ms([&] {
             hipLaunchKernelGGL((exp::xw3_kernel<1, 1>), dim3(tm * tn), dim3(256), exp::kXw3Lds, 0, D, D, tm, tn, XT,
                                n, W, D, Y, D, (int64_t)0);
           }, reps));
    CK(hipDeviceSynchronize());
    printf("    max|Y - Yref| = %.3e\n", maxdiff(Y, Yref, D * n));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<0, 0, 8>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(exp::xw3_kernel<0, 0, 1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)exp::kXw3Lds));
    report("xw  exp xw3<PLAIN B, stag 8>", time_ms([&] {
             hipLaunchKernelGGL((exp::xw3_kernel<0, 0, 8>), dim3(tm * tn), dim3(256), exp::kXw3Lds, 0, D, D, tm, tn, XT,
                                n, W, D, Y, D, (int64_t)0);
           }, reps));
    report("xw  exp xw3<PLAIN B, stag 1>", time_ms([&] {
             hipLaunchKernelGGL((exp::xw3_kernel<0, 0, 1>), dim3(tm * tn), dim3(256), exp::kXw3Lds, 0, D, D, tm, tn, XT,
                                n, W, D, Y, D, (int64_t)0);
           }, reps));
    report("xw  exp xw3<PLAIN B>", time_ms([&] {
             hipLaunchKernelGGL((exp::xw3_kernel<0, 0>), dim3(tm * tn), dim3(256), exp::kXw3Lds, 0, D, D, tm, tn, XT,
                                n, W, D, Y, D, (int64_t)0);
           }, reps));
    const int64_t per16 = (n / 16 + split - 1) / split;
    const int nsplit = (int)((n / 16 + per16 - 1) / per16);
    report("xty exp xw3<PLAIN,prio>/16", time_ms([&] {
             hipLaunchKernelGGL((exp::xw3_kernel<0, 1>), dim3(64 * nsplit), dim3(256), exp::kXw3Lds, 0, n, per16 * 16,
                                8, 8, X, D, Yref, D, Z, D, D * D);
           }, reps));
  }
  if (want("xty3")) {
    double* Z3;
    double* Zs;
    CK(hipMalloc(&Z3, sizeof(double) * D * D * split));
    CK(hipMalloc(&Zs, sizeof(double) * D * D));
    launch_gemm(D, D, n, X, D, true, Yref, D, B_PLAIN, Z, D, EPI_STORE, split, D * D, nullptr, 0, 0, nullptr, 0);
    launch_sum_slices(Z, split, D * D, D * D, Z2, nullptr, 0);
    const int64_t per16 = (n / 16 + split - 1) / split;
    const int nsplit = (int)((n / 16 + per16 - 1) / per16);
    report("xty exp xw3<PLAIN>/16", time_ms([&] {
             hipLaunchKernelGGL(exp::xw3_kernel<0>, dim3(64 * nsplit), dim3(256), exp::kXw3Lds, 0, n, per16 * 16, 8,
                                8, X, D, Yref, D, Z3, D, D * D);
           }, reps));
    launch_sum_slices(Z3, nsplit, D * D, D * D, Zs, nullptr, 0);
    CK(hipDeviceSynchronize());
    printf("    max|Z - Zref| = %.3e (rel to max|Zref| %.3e)\n", maxdiff(Zs, Z2, D * D), 0.0);
  }
  if (want("xty2")) {
    launch_gemm(D, D, n, X, D, true, Yref, D, B_PLAIN, Z, D, EPI_STORE, split, D * D, nullptr, 0, 0, nullptr, 0);
    launch_sum_slices(Z, split, D * D, D * D, Z2, nullptr, 0);
    CK(hipDeviceSynchronize());
    double* Z3;
    double* Zs;
    CK(hipMalloc(&Z3, sizeof(double) * D * D * split));
    CK(hipMalloc(&Zs, sizeof(double) * D * D));
    const int64_t per16 = (n / 16 + split - 1) / split;
    const int nsplit = (int)((n / 16 + per16 - 1) / per16);
    report("xty exp xw2<PLAIN>/16", time_ms([&] {
             hipLaunchKernelGGL(exp::xw2_kernel<0>, dim3(64 * nsplit), dim3(256), exp::kXw2Lds, 0, n, per16 * 16, 8,
                                8, X, D, Yref, D, Z3, D, D * D);
           }, reps));
    launch_sum_slices(Z3, nsplit, D * D, D * D, Zs, nullptr, 0);
    CK(hipDeviceSynchronize());
    printf("    max|Z - Zref| = %.3e\n", maxdiff(Zs, Z2, D * D));
  }
  if (want("blas")) {
    rocblas_handle h;
    rocblas_create_handle(&h);
    const double one = 1.0, zero = 0.0;
    // column-major view: Y^T (D x n) = (I-W)^T-as-stored (D x D) * X^T-as-stored (D x n)
    report("xw  rocblas_dgemm NN", time_ms([&] {
             rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, D, n, D, &one, W, D, X, D, &zero, Y, D);
           }, reps));
    // Z^T (D x D) = Y_cm (D x n) * (X_cm)^T (n x D)
    report("xty rocblas_dgemm NT", time_ms([&] {
             rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, D, D, n, &one, Y, D, X, D, &zero,
                           Z2, D);
           }, reps));
    // Z^T (D x D) = Y_cm (D x n) * XT_cm (n x D, ld n): NN with both operands k-contiguous in B
    report("xty rocblas_dgemm NN (XT)", time_ms([&] {
             rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, D, D, n, &one, Y, D, XT, n, &zero, Z2,
                           D);
           }, reps));
    rocblas_destroy_handle(h);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
