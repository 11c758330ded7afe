// fit()'s data preparation on the device (linear.py:406-428): the column sums behind the l2
// centring `X -= X.mean(axis=0)` (411), the centring itself, and cov's Gram matrix X^T X (428)
// from a row-major X of any leading dimension, on device or host memory.
//
// The Gram streams X through a zero-padded staging buffer in chunks of rows (so any ld and any
// row count reach the 128 x 128 pipelined MFMA GEMM, whose shapes must be tile multiples) and
// keeps a running sum: each chunk's split-K slices and the accumulator are summed in a fixed
// order, so the result is deterministic and independent of the device's timing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "launch.h"

namespace midagma {

namespace {

constexpr int CS_COLS = 64;   // columns per colsum workgroup (one per lane of a wave)
constexpr int CS_WAVES = NTHREADS / 64;

// part[(blockIdx.y * 4 + wave) * d + j] = sum of X[r, j] over this workgroup's row range,
// rows r = r0 + wave, r0 + wave + 4, ...: a wave reads 64 consecutive doubles of one row
__global__ void colsum_part_kernel(const double* __restrict__ X, int64_t n, int64_t d, int64_t ldx,
                                   int64_t rows_per, double* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * CS_COLS + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = std::min<int64_t>(n, r0 + rows_per);
  if (j >= d) return;
  double acc = 0.0;
#pragma unroll 8
  for (int64_t r = r0 + wave; r < r1; r += CS_WAVES) acc += X[r * ldx + j];
  part[((int64_t)blockIdx.y * CS_WAVES + wave) * d + j] = acc;
}

// out[j] = sum_p part[p * d + j] in ascending p
__global__ void colsum_final_kernel(const double* __restrict__ part, int64_t np, int64_t d,
                                    double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (j >= d) return;
  double acc = 0.0;
  for (int64_t p = 0; p < np; ++p) acc += part[p * d + j];
  out[j] = acc;
}

// X[r, j] -= colsum[j] / n  (X.mean(axis=0) is the column sum over n: linear.py:411)
__global__ void center_kernel(double* __restrict__ X, int64_t n, int64_t d, int64_t ldx,
                              const double* __restrict__ colsum, double nrows) {
  const int64_t j = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (j >= d) return;
  const double mean = colsum[j] / nrows;
  for (int64_t r = blockIdx.y; r < n; r += gridDim.y) X[r * ldx + j] -= mean;
}

// S[r, c] (ld D) = X[r, c] for r < rows, c < d; 0 elsewhere in the rpad x D chunk.  *flag |= 1
// when a copied value is not finite (scipy's check_finite on the operands of linear.py:428).
__global__ void stage_rows_kernel(const double* __restrict__ X, int64_t ldx, int64_t rows, int64_t d,
                                  double* __restrict__ S, int64_t D, int64_t rpad, int* __restrict__ flag) {
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  int bad = 0;
  if (c < D) {
    for (int64_t r = blockIdx.y; r < rpad; r += gridDim.y) {
      double v = 0.0;
      if (r < rows && c < d) {
        v = X[r * ldx + c];
        bad |= std::isfinite(v) ? 0 : 1;
      }
      S[r * D + c] = v;
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// *flag |= 1 if any of the rows x cols block (ld) is not finite (the host-copied chunks)
__global__ void nonfinite_or_kernel(const double* __restrict__ S, int64_t rows, int64_t cols, int64_t ld,
                                    int* __restrict__ flag) {
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  int bad = 0;
  if (c < cols)
    for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) bad |= std::isfinite(S[r * ld + c]) ? 0 : 1;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// out[r, c] (ldo) = in[r, c] (ldi) / divisor for r, c < d; *flag |= 1 on a non-finite result
__global__ void div_block_kernel(const double* __restrict__ in, int64_t ldi, double divisor, int64_t d,
                                 double* __restrict__ out, int64_t ldo, int* __restrict__ flag) {
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  int bad = 0;
  if (c < d)
    for (int64_t r = blockIdx.y; r < d; r += gridDim.y) {
      const double v = in[r * ldi + c] / divisor;
      bad |= std::isfinite(v) ? 0 : 1;
      out[r * ldo + c] = v;
    }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

unsigned row_grid(int64_t rows) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(rows, 4096)); }

}  // namespace

int64_t colsum_parts(int64_t n) {
  const int64_t groups = std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256));
  return groups * CS_WAVES;
}

void launch_colsum(const double* X, int64_t n, int64_t d, int64_t ldx, double* part, double* out,
                   hipStream_t stream) {
  const int64_t groups = colsum_parts(n) / CS_WAVES;
  const int64_t rows_per = std::max<int64_t>(1, (n + groups - 1) / groups);
  const int64_t used = std::max<int64_t>(1, (n + rows_per - 1) / rows_per);
  dim3 grid((unsigned)((d + CS_COLS - 1) / CS_COLS), (unsigned)used);
  if (n > 0) {
    hipLaunchKernelGGL(colsum_part_kernel, grid, dim3(NTHREADS), 0, stream, X, n, d, ldx, rows_per, part);
    HIP_TRY(hipGetLastError());
  }
  const int64_t np = n > 0 ? used * CS_WAVES : 0;
  hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((d + NTHREADS - 1) / NTHREADS)), dim3(NTHREADS), 0, stream,
                     part, np, d, out);
  HIP_TRY(hipGetLastError());
}

void launch_center(double* X, int64_t n, int64_t d, int64_t ldx, const double* colsum, double nrows,
                   hipStream_t stream) {
  if (n < 1) return;
  dim3 grid((unsigned)((d + NTHREADS - 1) / NTHREADS), row_grid(n));
  hipLaunchKernelGGL(center_kernel, grid, dim3(NTHREADS), 0, stream, X, n, d, ldx, colsum, nrows);
  HIP_TRY(hipGetLastError());
}

void launch_stage_rows(const double* X, int64_t ldx, int64_t rows, int64_t d, double* S, int64_t D, int64_t rpad,
                       int* flag, hipStream_t stream) {
  dim3 grid((unsigned)((D + NTHREADS - 1) / NTHREADS), row_grid(rpad));
  hipLaunchKernelGGL(stage_rows_kernel, grid, dim3(NTHREADS), 0, stream, X, ldx, rows, d, S, D, rpad, flag);
  HIP_TRY(hipGetLastError());
}

void launch_nonfinite_or(const double* S, int64_t rows, int64_t cols, int64_t ld, int* flag, hipStream_t stream) {
  if (rows < 1) return;
  dim3 grid((unsigned)((cols + NTHREADS - 1) / NTHREADS), row_grid(rows));
  hipLaunchKernelGGL(nonfinite_or_kernel, grid, dim3(NTHREADS), 0, stream, S, rows, cols, ld, flag);
  HIP_TRY(hipGetLastError());
}

void launch_div_block(const double* in, int64_t ldi, double divisor, int64_t d, double* out, int64_t ldo, int* flag,
                      hipStream_t stream) {
  dim3 grid((unsigned)((d + NTHREADS - 1) / NTHREADS), row_grid(d));
  hipLaunchKernelGGL(div_block_kernel, grid, dim3(NTHREADS), 0, stream, in, ldi, divisor, d, out, ldo, flag);
  HIP_TRY(hipGetLastError());
}

GramPlan gram_plan(int64_t n, int64_t d, int64_t chunk_rows) {
  GramPlan p;
  p.D = (d + 127) / 128 * 128;
  const int64_t tiles = (p.D / 128) * (p.D / 128);
  // split-K so one chunk's GEMM has >= ~1024 workgroups; a power of two, and chunks padded to a
  // multiple of 256 rows, so every split slice gets the same whole number of 16-row k-tiles
  int split = 1;
  while (split < 16 && tiles * split < 1024) split *= 2;
  p.split = split;
  const int64_t cap = std::max<int64_t>(256, chunk_rows / 256 * 256);
  p.chunk = std::min<int64_t>(cap, std::max<int64_t>(256, (n + 255) / 256 * 256));
  p.nchunks = n > 0 ? (n + p.chunk - 1) / p.chunk : 0;
  return p;
}

}  // namespace midagma
