// FP64 matrix-core building blocks for 64 x 64 tiles (gfx950, v_mfma_f64_16x16x4_f64).
//
// A 256-thread workgroup = 4 waves; wave w owns the 32 x 32 output quadrant
// (wm, wn) = (w >> 1, w & 1) as a 2 x 2 grid of 16 x 16 MFMA accumulators.
// Operand images live in LDS (strides SA / SB in common.h).
#pragma once

#include "common.h"

namespace midagma {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// Row of accumulator register t held by `lane` (16x16x4 f64 C/D map):
// col = lane & 15, row = (lane >> 4) + 4 * t  (cdna_hip_programming.md sec. 3).
#ifndef MIDAGMA_F64_ROW_MAJOR_QUAD
__device__ __forceinline__ int acc_row(int lane, int t) { return (lane >> 4) + 4 * t; }
#else
__device__ __forceinline__ int acc_row(int lane, int t) { return 4 * (lane >> 4) + t; }
#endif
__device__ __forceinline__ int acc_col(int lane) { return lane & 15; }

struct Quad {
  dbl4 c[2][2];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) c[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
  }
};

// acc += A(64 x 64) * B(64 x 64) restricted to this wave's quadrant.
// A_KM = false: As is an [m][k] image (stride SA); true: a [k][m] image (stride SB).
// Bs is a [k][n] image (stride SB).  kdepth: number of k (multiple of 4, <= 64).
template <bool A_KM>
__device__ __forceinline__ void quad_mma(const double* __restrict__ As, const double* __restrict__ Bs,
                                         Quad& q, int kdepth = TILE) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int m0 = (w >> 1) * 32, n0 = (w & 1) * 32;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < kdepth; k0 += 4) {
    const int kk = k0 + kq;
    double a0, a1;
    if (A_KM) {
      a0 = As[kk * SB + m0 + r];
      a1 = As[kk * SB + m0 + 16 + r];
    } else {
      a0 = As[(m0 + r) * SA + kk];
      a1 = As[(m0 + 16 + r) * SA + kk];
    }
    const double b0 = Bs[kk * SB + n0 + r];
    const double b1 = Bs[kk * SB + n0 + 16 + r];
    q.c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, q.c[0][0], 0, 0, 0);
    q.c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, q.c[0][1], 0, 0, 0);
    q.c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, q.c[1][0], 0, 0, 0);
    q.c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, q.c[1][1], 0, 0, 0);
  }
}

// Visit every (row, col, value) of this wave's quadrant.  f(row, col, double&)
template <class F>
__device__ __forceinline__ void quad_foreach(Quad& q, F&& f) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int m0 = (w >> 1) * 32, n0 = (w & 1) * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        double tmp = q.c[i][j][t];
        f(m0 + 16 * i + acc_row(lane, t), n0 + 16 * j + acc_col(lane), tmp);
        q.c[i][j][t] = tmp;
      }
}

// Copy a 64 x 64 tile from global (row-major, leading dim ld) into an LDS
// image with row stride S, applying op(row, col, value) -> value.
template <int S, class Op>
__device__ __forceinline__ void tile_to_lds(double* __restrict__ dst, const double* __restrict__ src, int64_t ld,
                                            Op op) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int item = it * NTHREADS + threadIdx.x;  // 2048 double2 items
    const int row = item >> 5, c = (item & 31) * 2;
    const double2 v = *reinterpret_cast<const double2*>(src + row * ld + c);
    double2 o;
    o.x = op(row, c, v.x);
    o.y = op(row, c + 1, v.y);
    *reinterpret_cast<double2*>(dst + row * S + c) = o;
  }
}

// Transposed copy: dst[c][r] = op(r, c, src[r][c]) (image stride S).
template <int S, class Op>
__device__ __forceinline__ void tile_to_lds_t(double* __restrict__ dst, const double* __restrict__ src, int64_t ld,
                                              Op op) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int item = it * NTHREADS + threadIdx.x;
    const int row = item >> 5, c = (item & 31) * 2;
    const double2 v = *reinterpret_cast<const double2*>(src + row * ld + c);
    dst[c * S + row] = op(row, c, v.x);
    dst[(c + 1) * S + row] = op(row, c + 1, v.y);
  }
}

struct Ident {
  __device__ __forceinline__ double operator()(int, int, double v) const { return v; }
};
struct Negate {
  __device__ __forceinline__ double operator()(int, int, double v) const { return -v; }
};

}  // namespace midagma
