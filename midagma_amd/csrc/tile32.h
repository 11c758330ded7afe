// 32 x 32 FP64 tile building blocks shared by the Gauss-Jordan (gj.hip) and the two-level
// blocked inverse (blockinv.hip): LDS images, the 16x16x4 f64 MFMA tile product of a
// 256-thread workgroup (wave w owns the 16 x 16 quadrant (w >> 1, w & 1)), DPP reductions
// and the write-through store used for data the next launch reads.
#pragma once

#include "mfma64.h"

namespace midagma {

constexpr int NB = 32;  // tile edge (block size of the 32-level elimination)

// Every 32 x 32 LDS image has row stride ST = 34 (= 2 mod 32 doubles): conflict-free as
// an MFMA A operand ([m][k], lanes walk rows) and 2-way on one ds_read_b64 lane group as
// a B operand ([k][n], lanes walk columns) -- one image then serves both roles, which the
// warm-started inverse needs (X is the B operand of S X and the A operand of X R).
constexpr int ST = 34;

// ---- 32 x 32 tile helpers --------------------------------------------------------
// Wave w owns the 16 x 16 quadrant (wm, wn) = (w >> 1, w & 1) of a 32 x 32 output.
__device__ __forceinline__ int q_m0() { return (threadIdx.x >> 7) * 16; }
__device__ __forceinline__ int q_n0() { return ((threadIdx.x >> 6) & 1) * 16; }

// acc += Ls * Rs, both 32 x 32 LDS images (row stride ST).  Four independent MFMA
// chains (k mod 16) summed at the end: a dependent chain leaves the SIMD's matrix pipe
// idle between its MFMAs, and co-resident workgroups' MFMAs take those slots -- with
// independent chains a high-priority wave (the diagonal owner) keeps the pipe.
__device__ __forceinline__ void mma32(const double* __restrict__ Ls, const double* __restrict__ Rs, dbl4& acc) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const double* La = Ls + (q_m0() + r) * ST + kq;
  const double* Rb = Rs + kq * ST + q_n0() + r;
  const dbl4 z = {0.0, 0.0, 0.0, 0.0};
  dbl4 c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[0], Rb[0], acc, 0, 0, 0);
  dbl4 c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[4], Rb[4 * ST], z, 0, 0, 0);
  dbl4 c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[8], Rb[8 * ST], z, 0, 0, 0);
  dbl4 c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[12], Rb[12 * ST], z, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[16], Rb[16 * ST], c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[20], Rb[20 * ST], c1, 0, 0, 0);
  c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[24], Rb[24 * ST], c2, 0, 0, 0);
  c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[28], Rb[28 * ST], c3, 0, 0, 0);
  acc = (c0 + c1) + (c2 + c3);
}

template <class F>
__device__ __forceinline__ void acc_foreach(dbl4& acc, F&& f) {
  const int lane = threadIdx.x & 63;
  const int m0 = q_m0(), n0 = q_n0();
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    double v = acc[t];
    f(m0 + acc_row(lane, t), n0 + acc_col(lane), v);
    acc[t] = v;
  }
}

// 32 x 32 global tile (leading dim ld) -> LDS image (stride ST), scaled by `sc`
__device__ __forceinline__ void tile32_to_lds(double* __restrict__ dst, const double* __restrict__ src, int64_t ld,
                                              double sc) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int item = it * NTHREADS + threadIdx.x;  // 512 double2 items
    const int row = item >> 4, c = (item & 15) * 2;
    double2 v = *reinterpret_cast<const double2*>(src + row * ld + c);
    v.x *= sc;
    v.y *= sc;
    *reinterpret_cast<double2*>(dst + row * ST + c) = v;
  }
}

__device__ __forceinline__ void tile32_copy(double* __restrict__ dst, int64_t ldd, const double* __restrict__ src,
                                            int64_t lds) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int item = it * NTHREADS + threadIdx.x;
    const int row = item >> 4, c = (item & 15) * 2;
    *reinterpret_cast<double2*>(dst + row * ldd + c) = *reinterpret_cast<const double2*>(src + row * lds + c);
  }
}

// Store for data the NEXT launch reads: write-through (sc1), so the tile does not sit
// dirty in this XCD's L2 and the kernel boundary has nothing of it to write back
// (MI355X_MICROARCH.md price list: a boundary pays dirty bytes / ~6 TB/s).
__device__ __forceinline__ void st_wt(double* p, double v) {
#ifdef MIDAGMA_GJ_PLAIN_STORES
  *p = v;
#else
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// max over the 64 lanes of a wave of a non-negative float: DPP within each row of 16
// (quad swaps, half-row and row mirrors: single v_max_f32_dpp ops), then the four row
// results by readlane.  No LDS round trip.
template <int CTRL>
__device__ __forceinline__ float dpp_max(float v) {
  return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false)));
}
__device__ __forceinline__ float wave_max(float v) {
  v = dpp_max<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_max<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_max<0x141>(v);  // row_half_mirror
  v = dpp_max<0x140>(v);  // row_mirror
  const int b = __float_as_int(v);
  return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(b, 0)), __int_as_float(__builtin_amdgcn_readlane(b, 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(b, 32)), __int_as_float(__builtin_amdgcn_readlane(b, 48))));
}

// Two independent 32 x 32 products in one pass (their MFMA chains interleave):
//   c1 += A1 * B1,  c2 += A2 * B2   (LDS images, stride ST)
__device__ __forceinline__ void mma32x2(const double* __restrict__ A1, const double* __restrict__ B1, dbl4& c1,
                                        const double* __restrict__ A2, const double* __restrict__ B2, dbl4& c2) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int ao = (q_m0() + r) * ST + kq, bo = kq * ST + q_n0() + r;
#pragma unroll
  for (int k0 = 0; k0 < NB; k0 += 4) {
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(A1[ao + k0], B1[bo + k0 * ST], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(A2[ao + k0], B2[bo + k0 * ST], c2, 0, 0, 0);
  }
}


// A^T tile builder: At[J][I] = (I == J ? s : 0) - f(X[I][J]) on the logical d x d block (f =
// square for W, identity for a given A), identity padding; source tile (rows bi, cols bj) through
// the LDS tile; IW (nullable) = I - X untransposed (the data-mode score GEMM's B operand).
// w32: W is float32 (common.h sw_entry / one_minus).
// build_at_kernel (gj.hip) and the fast slot's build_resid0_kernel (blockinv.hip).
template <bool SQUARE, int BT = 32>
__device__ __forceinline__ void build_at_tile(int bi, int bj, const double* __restrict__ X, int64_t ldx,
                                              double* __restrict__ At, int64_t D, int64_t d, double s,
                                              double* __restrict__ IW, double (&tile)[BT][BT + 1],
                                              bool w32 = false) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < BT * BT / NTHREADS; ++it) {
    const int e = it * NTHREADS + tid;
    const int r = e / BT, c = e % BT;
    const int64_t I = (int64_t)bi * BT + r, J = (int64_t)bj * BT + c;
    double v;
    const double x = (I < d && J < d) ? X[I * ldx + J] : 0.0;
    if (I < d && J < d) {
      v = SQUARE ? sw_entry(I == J, s, x, w32) : (I == J ? s : 0.0) - x;
    } else {
      v = (I == J) ? 1.0 : 0.0;
    }
    if (IW) IW[I * D + J] = one_minus(I == J, x, w32);
    tile[c][r] = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < BT * BT / NTHREADS; ++it) {
    const int e = it * NTHREADS + tid;
    const int r = e / BT, c = e % BT;  // r: row of At tile (= source col)
    At[((int64_t)bj * BT + r) * D + (int64_t)bi * BT + c] = tile[r][c];
  }
}

}  // namespace midagma
