// Development micro-benchmark (not part of the library): the fused DagmaMLP fc1 + tail forward
// and backward (csrc/mlp.hip, ABI 7) at config 5's shape (n = 1000, d = 200, m1 = 10), hipEvent-
// timed, with parts switched off by MLP_FUSED_PROBE (see mlp.hip) to locate the time.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMIDAGMA_EXPERIMENTS -I../../midagma_amd/csrc
//          -DMLP_FUSED_PROBE=<bits> mlp_micro.hip -o mlp_micro_<bits>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../midagma_amd/csrc/mlp.hip"

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
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    p[i] = scale * ((double)(x >> 11) / 9007199254740992.0 - 0.5);
  }
}

static double* dalloc(int64_t n, uint64_t seed, double scale) {
  double* p = nullptr;
  CK(hipMalloc(&p, n * sizeof(double)));
  hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, p, n, seed, scale);
  return p;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000, d = argc > 2 ? atoll(argv[2]) : 200;
  const int m1 = argc > 3 ? atoi(argv[3]) : 10;
  const int64_t dm = d * m1, np = mlp_fused_parts(n, d, m1), ns = mlp_fused_splits(n);
  double *X = dalloc(n * d, 1, 2.0), *W1 = dalloc(dm * d, 2, 0.05), *b1 = dalloc(dm, 3, 0.2), *w2 = dalloc(dm, 4, 0.5);
  double *b2 = dalloc(d, 5, 0.5), *S = dalloc(n * dm, 6, 1.0), *R = dalloc(n * d, 7, 1.0), *part = dalloc(np, 8, 1.0);
  double *gobj = dalloc(1, 9, 1.0), *lin = dalloc(ns * dm * d, 10, 1.0), *dw2 = dalloc(dm, 11, 1.0);
  double *db2 = dalloc(d, 12, 1.0), *db1 = dalloc(dm, 13, 1.0), *scr = dalloc(mlp_tail_scratch(n, d, m1), 14, 1.0);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  float ms = 0.f;
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) launch_mlp_fc1_tail_fwd(X, W1, b1, w2, b2, n, d, m1, S, R, part, 0);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  printf("probe=%d fwd %.2f us", MLP_FUSED_PROBE, ms * 1e3 / reps);
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
      launch_mlp_tail_bwd_lin(S, w2, R, X, part, np, gobj, 0.1, 0.5 * d, 1.0 / n, n, d, m1, lin, dw2, db2, db1, scr, 0);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  printf("  bwd+dw %.2f us\n", ms * 1e3 / reps);
  return 0;
}
