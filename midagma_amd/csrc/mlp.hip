// The DagmaMLP tail for BASELINE config 5 (dims [d, m1, 1]), fused: from the fc1 output
// Z (n x d*m1, nonlinear.py:99-100) through sigmoid, the width-1 LocallyConnected layer and
// its bias (locally_connected.py:55-85, nonlinear.py:101-104) to the squared residual sum the
// log-MSE score takes (nonlinear.py:139-159):
//     S = sigmoid(Z),  Xhat[r, j] = sum_m S[r, j, m] w2[j, m] + b2[j],  ssq = sum (Xhat - X)^2
// and its backward for d(ssq) = g:
//     dXhat = 2 g (Xhat - X),  dZ = dXhat w2 S (1 - S),  dw2[j, m] = sum_r dXhat S,  db2 = sum_r dXhat.
// Four launches replace the ~20 elementwise/reduction kernels PyTorch runs for the same
// forward and backward.  Sums over rows run in a fixed order (deterministic).
#include "launch.h"

namespace midagma {
namespace {

__device__ __forceinline__ double sigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

// thread per (row, j): residual R and per-workgroup partial of R^2
__global__ __launch_bounds__(NTHREADS) void mlp_tail_fwd_kernel(const double* __restrict__ Z,
                                                                const double* __restrict__ w2,
                                                                const double* __restrict__ b2,
                                                                const double* __restrict__ X, int64_t n, int64_t d,
                                                                int m1, double* __restrict__ R,
                                                                double* __restrict__ part) {
  __shared__ double red[NTHREADS];
  const int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  double r2 = 0.0;
  if (t < n * d) {
    const int64_t row = t / d, j = t % d;
    const double* z = Z + row * d * m1 + j * m1;
    const double* w = w2 + j * m1;
    double acc = 0.0;
    for (int m = 0; m < m1; ++m) acc += sigmoid(z[m]) * w[m];
    const double r = (acc + b2[j]) - X[t];
    R[t] = r;
    r2 = r * r;
  }
  red[threadIdx.x] = r2;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// one workgroup: out[0] = sum of the np partials (fixed order)
__global__ __launch_bounds__(NTHREADS) void mlp_sum_kernel(const double* __restrict__ part, int64_t np,
                                                           double* __restrict__ out) {
  __shared__ double red[NTHREADS];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += NTHREADS) a += part[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// thread per (row, j): dZ[row, j, :]
__global__ __launch_bounds__(NTHREADS) void mlp_tail_dz_kernel(const double* __restrict__ Z,
                                                               const double* __restrict__ w2,
                                                               const double* __restrict__ R,
                                                               const double* __restrict__ g, int64_t n, int64_t d,
                                                               int m1, double* __restrict__ dZ) {
  const int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (t >= n * d) return;
  const int64_t row = t / d, j = t % d;
  const double dxh = 2.0 * g[0] * R[t];
  const double* z = Z + row * d * m1 + j * m1;
  const double* w = w2 + j * m1;
  double* dz = dZ + row * d * m1 + j * m1;
  for (int m = 0; m < m1; ++m) {
    const double s = sigmoid(z[m]);
    dz[m] = dxh * w[m] * (s * (1.0 - s));
  }
}

// workgroup per node j: dw2[j, :] and db2[j], sums over the rows in a fixed order
template <int MAXM>
__global__ __launch_bounds__(NTHREADS) void mlp_tail_dw_kernel(const double* __restrict__ Z,
                                                               const double* __restrict__ R,
                                                               const double* __restrict__ g, int64_t n, int64_t d,
                                                               int m1, double* __restrict__ dw2,
                                                               double* __restrict__ db2) {
  __shared__ double red[NTHREADS];
  const int64_t j = blockIdx.x;
  double acc[MAXM + 1];
#pragma unroll
  for (int m = 0; m <= MAXM; ++m) acc[m] = 0.0;
  const double g2 = 2.0 * g[0];
  for (int64_t row = threadIdx.x; row < n; row += NTHREADS) {
    const double dxh = g2 * R[row * d + j];
    const double* z = Z + row * d * m1 + j * m1;
#pragma unroll
    for (int m = 0; m < MAXM; ++m)
      if (m < m1) acc[m] += dxh * sigmoid(z[m]);
    acc[MAXM] += dxh;
  }
#pragma unroll
  for (int m = 0; m <= MAXM; ++m) {
    if (m < m1 || m == MAXM) {
      red[threadIdx.x] = acc[m];
      __syncthreads();
      for (int s = NTHREADS / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        if (m == MAXM)
          db2[j] = red[0];
        else
          dw2[j * m1 + m] = red[0];
      }
      __syncthreads();
    }
  }
}

}  // namespace

void launch_mlp_tail_fwd(const double* Z, const double* w2, const double* b2, const double* X, int64_t n, int64_t d,
                         int m1, double* R, double* part, double* ssq, hipStream_t stream) {
  const int64_t blocks = (n * d + NTHREADS - 1) / NTHREADS;
  hipLaunchKernelGGL(mlp_tail_fwd_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, Z, w2, b2, X, n, d, m1,
                     R, part);
  hipLaunchKernelGGL(mlp_sum_kernel, dim3(1), dim3(NTHREADS), 0, stream, part, blocks, ssq);
  HIP_TRY(hipGetLastError());
}

void launch_mlp_tail_bwd(const double* Z, const double* w2, const double* R, const double* g, int64_t n, int64_t d,
                         int m1, double* dZ, double* dw2, double* db2, hipStream_t stream) {
  if (m1 > MLP_TAIL_MAXM) throw std::invalid_argument("mlp tail: hidden width above 16");
  const int64_t blocks = (n * d + NTHREADS - 1) / NTHREADS;
  hipLaunchKernelGGL(mlp_tail_dz_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, Z, w2, R, g, n, d, m1, dZ);
  hipLaunchKernelGGL(mlp_tail_dw_kernel<MLP_TAIL_MAXM>, dim3((unsigned)d), dim3(NTHREADS), 0, stream, Z, R, g, n, d,
                     m1, dw2, db2);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
