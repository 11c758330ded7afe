// Experimental FP64 GEMM variants for the micro-benchmark (development only).
//
// xw2: C[M x N] (+ split-K slices) = op(A) op(B), op(A) from A stored [k][m] (lda), staged
// through a double-buffered LDS image; op(B) = B or I - B ([k][n], ldb) loaded straight into
// the MFMA B-fragment registers, one k-tile ahead.  128 x 128 tile, 4 waves side by side in N
// (wave w: all 128 rows x 32 columns = 8 x 2 accumulators of 16 x 16).
#pragma once

#include "mfma64.h"

namespace midagma {
namespace exp {

constexpr int X_S = 144;  // [k][m] image stride (16 mod 32 doubles: conflict-free fragment reads)

__device__ __forceinline__ int xcd_remap2(int w, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = w % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
}

template <int BMODE>
__global__ __launch_bounds__(256, 2) void xw2_kernel(int64_t K, int64_t kslice, int tiles_m, int tiles_n,
                                                     const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ B, int64_t ldb,
                                                     double* __restrict__ C, int64_t ldc, int64_t slice_stride) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = xcd_remap2(blockIdx.x, gridDim.x);
  const int per_slice = tiles_m * tiles_n;
  const int z = t / per_slice, rem = t % per_slice;
  const int bm = rem / tiles_n, bn = rem % tiles_n;
  const int64_t m0 = (int64_t)bm * 128, n0 = (int64_t)bn * 128;
  const int64_t k_begin = (int64_t)z * kslice;
  const int64_t k_end = (k_begin + kslice < K) ? k_begin + kslice : K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int64_t nw = n0 + 32 * w;

  const double* Ablk = A + m0;
  int offA[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i_ = it * 256 + tid;
    offA[it] = (i_ >> 6) * (int)lda + 2 * (i_ & 63);
  }
  const double* Bw = B + (int64_t)kq * ldb + nw + r;
  double2 ra0, ra1, ra2, ra3;
  double bn_[8], bc[8];
#define XW2_LOAD(KT)                                                                   \
  {                                                                                    \
    const double* ap_ = Ablk + (KT) * lda;                                             \
    ra0 = *reinterpret_cast<const double2*>(ap_ + offA[0]);                            \
    ra1 = *reinterpret_cast<const double2*>(ap_ + offA[1]);                            \
    ra2 = *reinterpret_cast<const double2*>(ap_ + offA[2]);                            \
    ra3 = *reinterpret_cast<const double2*>(ap_ + offA[3]);                            \
    const double* bp_ = Bw + (KT) * ldb;                                               \
    _Pragma("unroll") for (int kk_ = 0; kk_ < 4; ++kk_)                                \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_) {                                 \
      double v_ = bp_[(int64_t)(4 * kk_) * ldb + 16 * j_];                             \
      if (BMODE == 1) {                                                                \
        const int64_t kg_ = (KT) + 4 * kk_ + kq, ng_ = nw + 16 * j_ + r;               \
        v_ = (kg_ == ng_ ? 1.0 : 0.0) - v_;                                            \
      }                                                                                \
      bn_[2 * kk_ + j_] = v_;                                                          \
    }                                                                                  \
  }
#define XW2_STORE(AS)                                                                  \
  {                                                                                    \
    *reinterpret_cast<double2*>((AS) + ((0 * 256 + tid) >> 6) * X_S + 2 * (tid & 63)) = ra0; \
    *reinterpret_cast<double2*>((AS) + ((1 * 256 + tid) >> 6) * X_S + 2 * (tid & 63)) = ra1; \
    *reinterpret_cast<double2*>((AS) + ((2 * 256 + tid) >> 6) * X_S + 2 * (tid & 63)) = ra2; \
    *reinterpret_cast<double2*>((AS) + ((3 * 256 + tid) >> 6) * X_S + 2 * (tid & 63)) = ra3; \
  }

  dbl4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  double* As0 = smem;
  double* As1 = smem + 16 * X_S;
  if (k_begin < k_end) {
    XW2_LOAD(k_begin)
    XW2_STORE(As0)
#pragma unroll
    for (int q = 0; q < 8; ++q) bc[q] = bn_[q];
  }
  __syncthreads();
  for (int64_t kt = k_begin; kt < k_end; kt += 16) {
    const int64_t kn = (kt + 16 < k_end) ? kt + 16 : kt;
    XW2_LOAD(kn)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = As0[(4 * kk + kq) * X_S + 16 * i + r];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bc[2 * kk + j], acc[i][j], 0, 0, 0);
    }
    XW2_STORE(As1)
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) bc[q] = bn_[q];
    double* tmp = As0;
    As0 = As1;
    As1 = tmp;
  }
#undef XW2_LOAD
#undef XW2_STORE
  double* Ct = C + (int64_t)z * slice_stride;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int64_t row = m0 + 16 * i + acc_row(lane, tt);
        const int64_t col = nw + 16 * j + acc_col(lane);
        Ct[row * ldc + col] = acc[i][j][tt];
      }
}

constexpr size_t kXw2Lds = 2 * 16 * X_S * sizeof(double);

// xw3: the xw2 split (A through LDS shared by the 4 waves, B straight to registers) with
// a software pipeline in the style of the vendor DGEMM:
//   * k permuted inside a 16-deep tile: lane quarter kq takes k = 4 kq + kk at k-step kk, so a
//     lane's B values of one k-step come from one row of B and its two columns (2r, 2r + 1)
//     are one 16-B load (dwordx4) -- output column c of accumulator j is n = 2c + j;
//   * A image [k][m], row stride 132 (k rows 4 apart differ by 16 mod 32 doubles: the two
//     kq halves of a 32-lane group use disjoint banks -> conflict-free ds_read_b64);
//   * A fragments read one k-step ahead, the next tile's A staged into the other LDS buffer
//     during k-step 1, one barrier per tile placed before the last k-step so that the next
//     tile's first fragments are read while that k-step's MFMAs run.
constexpr int X3_S = 132;
constexpr int X3_IMG = 16 * X3_S;

template <int BMODE, int PRIO = 0, int STAG = 0>
__global__ __launch_bounds__(256, 2) void xw3_kernel(int64_t K, int64_t kslice, int tiles_m, int tiles_n,
                                                     const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ B, int64_t ldb,
                                                     double* __restrict__ C, int64_t ldc, int64_t slice_stride) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = xcd_remap2(blockIdx.x, gridDim.x);
  const int per_slice = tiles_m * tiles_n;
  const int z = t / per_slice, rem = t % per_slice;
  const int bm = rem / tiles_n, bn = rem % tiles_n;
  const int64_t m0 = (int64_t)bm * 128, n0 = (int64_t)bn * 128;
  const int64_t k_begin = (int64_t)z * kslice;
  const int64_t k_end = (k_begin + kslice < K) ? k_begin + kslice : K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int64_t nw = n0 + 32 * w;

  // A staging: item i_ = it * 256 + tid -> tile row k = i_ >> 6, columns m = 2 (i_ & 63) + {0,1}
  const double* Ablk = A + m0;
  int offA[4], ldsA[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i_ = it * 256 + tid;
    offA[it] = (i_ >> 6) * (int)lda + 2 * (i_ & 63);
    ldsA[it] = (i_ >> 6) * X3_S + 2 * (i_ & 63);
  }
  // B: row kt + 4 kq + kk, columns nw + 2r, nw + 2r + 1
  const double* Bw = B + (int64_t)(4 * kq) * ldb + nw + 2 * r;
  // A fragment of block i at k-step kk: image row 4 kq + kk, column 16 i + r
  const int fo = 4 * kq * X3_S + r;

  double2 ra0, ra1, ra2, ra3;
  double2 fb[4];  // raw B rows (I - B applied at use); row kk reloaded for the next tile right
                  // after its k-step's MFMAs are issued (no loop-carried copies)
  double fa0[8], fa1[8];
#define XW3_LOADA(KT)                                                                  \
  {                                                                                    \
    const double* ap_ = Ablk + (KT) * lda;                                             \
    ra0 = *reinterpret_cast<const double2*>(ap_ + offA[0]);                            \
    ra1 = *reinterpret_cast<const double2*>(ap_ + offA[1]);                            \
    ra2 = *reinterpret_cast<const double2*>(ap_ + offA[2]);                            \
    ra3 = *reinterpret_cast<const double2*>(ap_ + offA[3]);                            \
  }
#define XW3_LOADB1(KT, KK) fb[KK] = *reinterpret_cast<const double2*>(Bw + ((KT) + (KK)) * ldb);
#define XW3_STOREA(AS)                                                                 \
  {                                                                                    \
    *reinterpret_cast<double2*>((AS) + ldsA[0]) = ra0;                                 \
    *reinterpret_cast<double2*>((AS) + ldsA[1]) = ra1;                                 \
    *reinterpret_cast<double2*>((AS) + ldsA[2]) = ra2;                                 \
    *reinterpret_cast<double2*>((AS) + ldsA[3]) = ra3;                                 \
  }
#define XW3_FRAG(DST, AS, KK)                                                          \
  {                                                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) DST[i_] = (AS)[fo + (KK) * X3_S + 16 * i_]; \
  }
#define XW3_MMA(FA, KT, KK)                                                            \
  {                                                                                    \
    double b0_ = fb[KK].x, b1_ = fb[KK].y;                                             \
    if (BMODE == 1) {                                                                  \
      const int64_t kg_ = (KT) + 4 * kq + (KK), ng_ = nw + 2 * r;                      \
      b0_ = (kg_ == ng_ ? 1.0 : 0.0) - b0_;                                            \
      b1_ = (kg_ == ng_ + 1 ? 1.0 : 0.0) - b1_;                                        \
    }                                                                                  \
    _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) {                                 \
      acc[i_][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(FA[i_], b0_, acc[i_][0], 0, 0, 0); \
      acc[i_][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(FA[i_], b1_, acc[i_][1], 0, 0, 0); \
    }                                                                                  \
  }

  dbl4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  // k-tile order: tile it of this slice is (it + stagger) mod ntile; with STAG the rotation
  // differs between row panels, so concurrent workgroups stream different rows of B
  const int64_t ntile = (k_end - k_begin) / 16;
  const int64_t stagger = STAG && ntile > 0 ? ((int64_t)bm * STAG) % ntile : 0;
#define KOF(I) (k_begin + 16 * (((I) + stagger) % ntile))
  double* As0 = smem;
  double* As1 = smem + X3_IMG;
  if (k_begin < k_end) {
    XW3_LOADA(KOF(0))
#pragma unroll
    for (int q = 0; q < 4; ++q) XW3_LOADB1(KOF(0), q)
    XW3_STOREA(As0)
    XW3_LOADA(KOF(ntile > 1 ? 1 : 0))
    __syncthreads();
    XW3_FRAG(fa0, As0, 0)
  }
  // per k-step: the next k-step's 8 fragment reads interleaved with the first MFMAs, then
  // NW ds_writes and NV global loads interleaved with the following ones
#define XW3_SCHED(NW, NV)                                                              \
  {                                                                                    \
    _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_) {                                 \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                               \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                               \
    }                                                                                  \
    _Pragma("unroll") for (int q_ = 0; q_ < (NW); ++q_) {                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                               \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                               \
    }                                                                                  \
    _Pragma("unroll") for (int q_ = 0; q_ < (NV); ++q_) {                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                               \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                               \
    }                                                                                  \
    __builtin_amdgcn_sched_group_barrier(0x008, 16 - 8 - (NW) - (NV), 0);             \
  }
  if (PRIO) __builtin_amdgcn_s_setprio(3);
  for (int64_t it = 0; it < ntile; ++it) {
    const int64_t kt = KOF(it);
    const int64_t k1 = KOF(it + 1 < ntile ? it + 1 : it);
    const int64_t k2 = KOF(it + 2 < ntile ? it + 2 : (it + 1 < ntile ? it + 1 : it));
    // k-step 0
    XW3_FRAG(fa1, As0, 1)
    XW3_MMA(fa0, kt, 0)
    XW3_LOADB1(k1, 0)
    XW3_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    // k-step 1: stage the next tile (loaded one tile ago), then issue the one after it
    XW3_STOREA(As1)
    XW3_FRAG(fa0, As0, 2)
    XW3_MMA(fa1, kt, 1)
    XW3_LOADB1(k1, 1)
    XW3_LOADA(k2)
    XW3_SCHED(4, 5)
    __builtin_amdgcn_sched_barrier(0);
    // k-step 2
    XW3_FRAG(fa1, As0, 3)
    XW3_MMA(fa0, kt, 2)
    XW3_LOADB1(k1, 2)
    XW3_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (PRIO) __builtin_amdgcn_s_setprio(3);
    // k-step 3: the next tile's first fragments are read while these MFMAs run
    XW3_FRAG(fa0, As1, 0)
    XW3_MMA(fa1, kt, 3)
    XW3_LOADB1(k1, 3)
    XW3_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    double* tmp = As0;
    As0 = As1;
    As1 = tmp;
  }
#undef XW3_SCHED
#undef KOF
#undef XW3_LOADA
#undef XW3_LOADB1
#undef XW3_STOREA
#undef XW3_FRAG
#undef XW3_MMA
  double* Ct = C + (int64_t)z * slice_stride;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int64_t row = m0 + 16 * i + acc_row(lane, tt);
      const int64_t col = nw + 2 * acc_col(lane);
      *reinterpret_cast<double2*>(Ct + row * ldc + col) = double2{acc[i][0][tt], acc[i][1][tt]};
    }
}

constexpr size_t kXw3Lds = 2 * X3_IMG * sizeof(double);

}  // namespace exp
}  // namespace midagma
