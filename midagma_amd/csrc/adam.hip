// Gated Adam step for DagmaNonlinear (nonlinear.py:213-224 through torch.optim.Adam, the
// single-tensor algorithm with L2 weight decay):
//     g = grad + wd * p;  m = m + (1 - b1) (g - m)  [lerp];  v = v * b2 + (1 - b2) * g * g
//     p = p + (-step_size) * m / (sqrt(v) / sqrt(1 - b2^t) + eps),  step_size = lr / (1 - b1^t)
// skipped when *gate < 0: the reference leaves minimize before stepping when h(W) < 0
// (nonlinear.py:216-218), so a negative h freezes the parameters -- and with them h -- for the
// rest of the call, and the host reads h only at checkpoints instead of every step.
#include <hip/hip_runtime.h>

#include "launch.h"

namespace midagma {
namespace {

__global__ __launch_bounds__(NTHREADS) void adam_gated_kernel(double* __restrict__ p, const double* __restrict__ g,
                                                              double* __restrict__ m, double* __restrict__ v,
                                                              int64_t n, AdamCoef c,
                                                              const double* __restrict__ gate) {
  if (gate && !(*gate >= 0.0)) return;
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTHREADS) {
    double gi = g[i];
    const double pi = p[i];
    if (c.wd != 0.0) gi = gi + c.wd * pi;
    const double mi = m[i] + c.w1 * (gi - m[i]);
    const double vi = v[i] * c.beta2 + c.c2 * gi * gi;
    const double denom = sqrt(vi) / c.bc2_sqrt + c.eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + (-c.step_size) * mi / denom;
  }
}

// the same step with (step_size, sqrt(1 - b2^t)) from a per-step table at the device step
// counter: one captured step serves every replay of a hipGraph
__global__ __launch_bounds__(NTHREADS) void adam_gated_table_kernel(double* __restrict__ p,
                                                                    const double* __restrict__ g,
                                                                    double* __restrict__ m, double* __restrict__ v,
                                                                    int64_t n, AdamCoef c,
                                                                    const double* __restrict__ table,
                                                                    const int64_t* __restrict__ counter,
                                                                    const double* __restrict__ gate) {
  if (gate && !(*gate >= 0.0)) return;
  const int64_t t = *counter;
  c.step_size = table[2 * t];
  c.bc2_sqrt = table[2 * t + 1];
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTHREADS) {
    double gi = g[i];
    const double pi = p[i];
    if (c.wd != 0.0) gi = gi + c.wd * pi;
    const double mi = m[i] + c.w1 * (gi - m[i]);
    const double vi = v[i] * c.beta2 + c.c2 * gi * gi;
    const double denom = sqrt(vi) / c.bc2_sqrt + c.eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + (-c.step_size) * mi / denom;
  }
}

// the table step over up to ADAM_MULTI tensors in one launch (grid-stride over their
// concatenation; the same per-element arithmetic as adam_gated_table_kernel)
__global__ __launch_bounds__(NTHREADS) void adam_gated_table_multi_kernel(AdamSet set, AdamCoef c,
                                                                          const double* __restrict__ table,
                                                                          const int64_t* __restrict__ counter,
                                                                          const double* __restrict__ gate) {
  if (gate && !(*gate >= 0.0)) return;
  const int64_t t = *counter;
  c.step_size = table[2 * t];
  c.bc2_sqrt = table[2 * t + 1];
  const int64_t total = set.off[set.k];
  for (int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * NTHREADS) {
    int q = 0;
    while (e >= set.off[q + 1]) ++q;
    const int64_t i = e - set.off[q];
    double* __restrict__ p = set.p[q];
    double* __restrict__ m = set.m[q];
    double* __restrict__ v = set.v[q];
    double gi = set.g[q][i];
    const double pi = p[i];
    if (c.wd != 0.0) gi = gi + c.wd * pi;
    const double mi = m[i] + c.w1 * (gi - m[i]);
    const double vi = v[i] * c.beta2 + c.c2 * gi * gi;
    const double denom = sqrt(vi) / c.bc2_sqrt + c.eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + (-c.step_size) * mi / denom;
  }
}

__global__ void counter_advance_kernel(int64_t* counter) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *counter += 1;
}

}  // namespace

void launch_adam_gated_table(double* p, const double* g, double* m, double* v, int64_t n, const AdamCoef& c,
                             const double* table, const int64_t* counter, const double* gate, hipStream_t stream) {
  const int64_t blocks = std::min<int64_t>((n + NTHREADS - 1) / NTHREADS, 2048);
  hipLaunchKernelGGL(adam_gated_table_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(NTHREADS), 0,
                     stream, p, g, m, v, n, c, table, counter, gate);
  HIP_TRY(hipGetLastError());
}

void launch_adam_gated_table_multi(const AdamSet& set, const AdamCoef& c, const double* table, const int64_t* counter,
                                   const double* gate, hipStream_t stream) {
  const int64_t n = set.off[set.k];
  const int64_t blocks = std::min<int64_t>((n + NTHREADS - 1) / NTHREADS, 2048);
  hipLaunchKernelGGL(adam_gated_table_multi_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(NTHREADS), 0,
                     stream, set, c, table, counter, gate);
  HIP_TRY(hipGetLastError());
}

void launch_counter_advance(int64_t* counter, hipStream_t stream) {
  hipLaunchKernelGGL(counter_advance_kernel, dim3(1), dim3(64), 0, stream, counter);
  HIP_TRY(hipGetLastError());
}

void launch_adam_gated(double* p, const double* g, double* m, double* v, int64_t n, const AdamCoef& c,
                       const double* gate, hipStream_t stream) {
  const int64_t blocks = std::min<int64_t>((n + NTHREADS - 1) / NTHREADS, 2048);
  hipLaunchKernelGGL(adam_gated_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(NTHREADS), 0, stream, p, g,
                     m, v, n, c, gate);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
