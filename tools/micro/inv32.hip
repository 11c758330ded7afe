// Microbenchmark: latency of one 32x32 unpivoted GJ tile inversion inside a workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NB = 32, SA32 = 34;

__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

// V1: 256 threads, 4 elements per thread (production version)
template <int NT>
__device__ void invert_v(double* img, double* scratch) {
  constexpr int EPT = NB * NB / NT, TPR = NB / EPT;
  const int tid = threadIdx.x;
  const int r = tid / TPR, c0 = (tid % TPR) * EPT;
  double* rowbuf = scratch;
  double* colbuf = scratch + 2 * NB;
  double a[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) a[e] = img[r * SA32 + c0 + e];
  for (int pb = 0; pb < NB; pb += EPT) {
#pragma unroll
    for (int pp = 0; pp < EPT; ++pp) {
      const int p = pb + pp;
      const int par = p & 1;
      if (r == p) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) rowbuf[par * NB + c0 + e] = a[e];
      }
      if (c0 == pb) colbuf[par * NB + r] = a[pp];
      if (NT > 64) __syncthreads(); else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      const double piv = rowbuf[par * NB + p];
      const double inv = fast_rcp(piv);
      const double arp = colbuf[par * NB + r];
      const double neg_arp_inv = -arp * inv;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int c = c0 + e;
        const double rpc = rowbuf[par * NB + c] * inv;
        if (r == p) a[e] = (c == p) ? inv : rpc;
        else a[e] = (c == p) ? neg_arp_inv : __builtin_fma(-arp, rpc, a[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) img[r * SA32 + c0 + e] = a[e];
  if (NT > 64) __syncthreads(); else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

template <int NT>
__global__ __launch_bounds__(NT) void bench(const double* A, double* out, int reps, long long* cycles) {
  __shared__ double img[NB * SA32];
  __shared__ double scratch[4 * NB];
  for (int i = threadIdx.x; i < NB * NB; i += NT) img[(i / NB) * SA32 + i % NB] = A[i];
  __syncthreads();
  long long t0 = clock64();
  for (int k = 0; k < reps; ++k) invert_v<NT>(img, scratch);  // inverts back and forth
  long long t1 = clock64();
  __syncthreads();
  for (int i = threadIdx.x; i < NB * NB; i += NT) out[i] = img[(i / NB) * SA32 + i % NB];
  if (threadIdx.x == 0) cycles[0] = t1 - t0;
}

int main() {
  std::vector<double> A(NB * NB);
  for (int i = 0; i < NB; ++i) for (int j = 0; j < NB; ++j) A[i * NB + j] = (i == j ? 1.0 : 0.0) - 0.01 * std::sin(i * 7 + j * 3);
  double *dA, *dO; long long* dc;
  CHECK(hipMalloc(&dA, NB * NB * 8)); CHECK(hipMalloc(&dO, NB * NB * 8)); CHECK(hipMalloc(&dc, 8));
  CHECK(hipMemcpy(dA, A.data(), NB * NB * 8, hipMemcpyHostToDevice));
  const int reps = 200;
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  auto run = [&](auto kern, int nt, const char* name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(nt), 0, 0, dA, dO, 2, dc);
    CHECK(hipDeviceSynchronize());
    std::vector<double> o(NB * NB);
    CHECK(hipMemcpy(o.data(), dO, NB * NB * 8, hipMemcpyDeviceToHost));
    double err = 0; for (int i = 0; i < NB * NB; ++i) err = std::fmax(err, std::fabs(o[i] - A[i]));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(1), dim3(nt), 0, 0, dA, dO, reps, dc);
    CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    long long cyc; CHECK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
    printf("%s: %.3f us per inversion, %.0f cycles (clock64) per inversion, double-inverse err %.2e\n", name, ms * 1e3 / reps, (double)cyc / reps, err);
    return 0;
  };
  run(bench<256>, 256, "256 threads x4");
  run(bench<64>, 64, "64 threads x16");
  run(bench<1024>, 1024, "1024 threads x1");
  run(bench<128>, 128, "128 threads x8");
  return 0;
}
