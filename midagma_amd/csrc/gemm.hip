// FP64 MFMA GEMM for the score gradients (linear.py:244, 246).
//
//   cov mode  : rhs = ((-mu) cov) @ (I - W)                   (d x d x d)
//   data mode : Y = X_k @ (I - W)  then  Z_k = X_k^T @ Y      (l2, row shard k)
//   logistic  : Y = expit(X_k @ W)  then  Z_k = X_k^T @ Y      (+ loss partials)
//
// 64 x 64 output tile per 256-thread workgroup, 64-deep K tiles staged through
// LDS in conflict-free images (mfma64.h); I - W is formed while staging B, the
// sigmoid and the logistic loss are fused into the epilogue.  Long K (= rows of
// the shard) is split over blockIdx.z into fixed slices summed in fixed order.
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "binv_tile.h"
#include "control.h"
#include "launch.h"
#include "mfma64.h"
#include "nm_series.h"

namespace midagma {

struct IMinus {
  int64_t k0, n0;
  __device__ __forceinline__ double operator()(int r, int c, double v) const {
    return ((k0 + r) == (n0 + c) ? 1.0 : 0.0) - v;
  }
};

// numpy.logaddexp(0, x) (npy_math: log1p/exp split on the sign of the difference)
__device__ __forceinline__ double logaddexp0(double x) {
  if (x == 0.0) return 0.69314718055994530942;
  const double t = -x;
  if (t > 0) return log1p(exp(-t));
  return x + log1p(exp(t));
}

template <bool ATRANS, int BMODE, int EPI>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(int64_t K, int64_t kslice, const double* __restrict__ A,
                                                        int64_t lda, const double* __restrict__ B, int64_t ldb,
                                                        double* __restrict__ C, int64_t ldc, int64_t slice_stride,
                                                        double* __restrict__ loss_part, int64_t m_valid,
                                                        int64_t n_valid, const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Ls = smem;            // [64][SA] or [64][SB] image of op(A)
  double* Bs = smem + 64 * SB;  // [64][SB] image of op(B)
  const int64_t bm = blockIdx.y, bn = blockIdx.x, z = blockIdx.z;
  const int64_t k_begin = z * kslice;
  const int64_t k_end = (k_begin + kslice < K) ? k_begin + kslice : K;
  Quad q;
  q.zero();
  for (int64_t kt = k_begin; kt < k_end; kt += 64) {
    __syncthreads();
    if (ATRANS)
      tile_to_lds<SB>(Ls, A + kt * lda + bm * 64, lda, Ident());
    else
      tile_to_lds<SA>(Ls, A + bm * 64 * lda + kt, lda, Ident());
    if (BMODE == B_IMINUS)
      tile_to_lds<SB>(Bs, B + kt * ldb + bn * 64, ldb, IMinus{kt, bn * 64});
    else
      tile_to_lds<SB>(Bs, B + kt * ldb + bn * 64, ldb, Ident());
    __syncthreads();
    quad_mma<ATRANS>(Ls, Bs, q);
  }
  double* Ct = C + z * slice_stride + bm * 64 * ldc + bn * 64;
  if (EPI == EPI_STORE) {
    quad_foreach(q, [&](int row, int col, double& v) { Ct[(int64_t)row * ldc + col] = v; });
    return;
  }
  // EPI_SIGMOID (A = X row-major, not transposed)
  const bool want_loss = loss_part != nullptr && (st == nullptr || st->ckpt_pending);
  double part = 0.0;
  quad_foreach(q, [&](int row, int col, double& v) {
    const int64_t gi = bm * 64 + row, gj = bn * 64 + col;
    if (want_loss && gi < m_valid && gj < n_valid) {
      const double x = A[gi * lda + gj];
      part += logaddexp0(v) - x * v;
    }
    Ct[(int64_t)row * ldc + col] = 1.0 / (1.0 + exp(-v));
  });
  if (!want_loss) return;
  __shared__ double red[NTHREADS];
  red[threadIdx.x] = part;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss_part[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

// ---- 128 x 128 tile GEMM (the data-mode and large-d workhorse) ---------------------------
// 4 waves in 2 x 2, each owning a 64 x 64 sub-tile = 4 x 4 accumulators of 16 x 16 (64 f64
// accumulator values per lane).  BK = 16, LDS double-buffered with register prefetch of the
// next k-tile (one barrier per k-tile).  LDS images (strides in doubles, conflict-free for
// the MFMA fragment reads of a 32-lane group):
//   op(A) from A[m][k] : [m][k] image, stride 17  (34 r dwords: distinct banks mod 64 for
//                        ds_read_b64 AND mod 32 for the ds_read2_b64 hipcc forms from two
//                        k-steps; stride 18 gave a 2-way conflict there: SQ_LDS_BANK_CONFLICT)
//   op(A) from A[k][m] : [k][m] image, stride 144 (= 16 mod 32)
//   op(B)              : [k][n] image, stride 144
// Workgroups are remapped so consecutive tiles (which share an A panel) run on one XCD.
constexpr int G_BM = 128, G_BN = 128, G_BK = 16;
constexpr int G_SMK = 17, G_SKM = 144;
constexpr int G_IMG = 16 * 144;  // doubles per operand image (>= 128 * 17)

__device__ __forceinline__ int xcd_remap(int w, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = w % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
}

template <bool ATRANS, int BMODE, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm128_kernel(int64_t K, int64_t kslice, int tiles_m, int tiles_n,
                                                              const double* __restrict__ A, int64_t lda,
                                                              const double* __restrict__ B, int64_t ldb,
                                                              double* __restrict__ C, int64_t ldc,
                                                              int64_t slice_stride, double* __restrict__ loss_part,
                                                              int64_t m_valid, int64_t n_valid,
                                                              const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int per_slice = tiles_m * tiles_n;
  const int z = t / per_slice, rem = t % per_slice;
  int bm = rem / tiles_n, bn = rem % tiles_n;
  if (EPI == EPI_SUB_BAND || EPI == EPI_SUB_PRE || EPI == EPI_SUB_MID) {
    // trailing update of the blocked inverse: the tile grid skips the pivot band
    // [m_valid, m_valid + n_valid) (in 128-tiles) in both rows and columns
    bm += bm >= (int)m_valid ? (int)n_valid : 0;
    bn += bn >= (int)m_valid ? (int)n_valid : 0;
  }
  const int64_t m0 = (int64_t)bm * G_BM, n0 = (int64_t)bn * G_BN;
  const int64_t k_begin = (int64_t)z * kslice;
  const int64_t k_end = (k_begin + kslice < K) ? k_begin + kslice : K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int mb = (w >> 1) * 64, nbs = (w & 1) * 64;

  // Register prefetch of the next k-tile.  Straight-line code (no lambdas, no conditional
  // loads) so the staging registers stay in VGPRs; the last iteration re-loads its own
  // tile into the idle buffer, which is harmless.
  double2 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
  // tile-invariant per-thread offsets (32-bit) and uniform tile bases
  const double* Ablk = ATRANS ? A + m0 : A + m0 * lda;
  const int64_t a_kstride = ATRANS ? lda : 1;
  const double* Bblk = B + n0;
  int offA[4], offB[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i_ = it * NTHREADS + tid;
    offA[it] = ATRANS ? (i_ >> 6) * (int)lda + 2 * (i_ & 63) : (i_ >> 3) * (int)lda + 2 * (i_ & 7);
    offB[it] = (i_ >> 6) * (int)ldb + 2 * (i_ & 63);
  }
#define G128_LOAD1(IT, RA, RB, KT)                                                              \
  {                                                                                             \
    const int i_ = (IT) * NTHREADS + tid;                                                       \
    RA = *reinterpret_cast<const double2*>(Ablk + (KT) * a_kstride + offA[IT]);                 \
    double2 v_ = *reinterpret_cast<const double2*>(Bblk + (KT) * ldb + offB[IT]);               \
    if (BMODE == B_IMINUS) {                                                                    \
      const int64_t kg_ = (KT) + (i_ >> 6), ng_ = n0 + 2 * (i_ & 63);                            \
      v_.x = (kg_ == ng_ ? 1.0 : 0.0) - v_.x;                                                    \
      v_.y = (kg_ == ng_ + 1 ? 1.0 : 0.0) - v_.y;                                                \
    }                                                                                           \
    RB = v_;                                                                                    \
  }
#define G128_STORE1(IT, RA, RB, AS, BS)                                                        \
  {                                                                                             \
    const int i_ = (IT) * NTHREADS + tid;                                                       \
    if (ATRANS)                                                                                 \
      *reinterpret_cast<double2*>((AS) + (i_ >> 6) * G_SKM + 2 * (i_ & 63)) = RA;               \
    else {                                                                                      \
      double* a_ = (AS) + (i_ >> 3) * G_SMK + 2 * (i_ & 7); /* odd stride: 8-byte aligned */    \
      a_[0] = RA.x;                                                                             \
      a_[1] = RA.y;                                                                             \
    }                                                                                           \
    *reinterpret_cast<double2*>((BS) + (i_ >> 6) * G_SKM + 2 * (i_ & 63)) = RB;                 \
  }
#define G128_LOAD(KT)                 \
  G128_LOAD1(0, ra0, rb0, KT)         \
  G128_LOAD1(1, ra1, rb1, KT)         \
  G128_LOAD1(2, ra2, rb2, KT)         \
  G128_LOAD1(3, ra3, rb3, KT)
#define G128_STORE(AS, BS)            \
  G128_STORE1(0, ra0, rb0, AS, BS)    \
  G128_STORE1(1, ra1, rb1, AS, BS)    \
  G128_STORE1(2, ra2, rb2, AS, BS)    \
  G128_STORE1(3, ra3, rb3, AS, BS)

  dbl4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  double* As0 = smem;
  double* As1 = smem + 2 * G_IMG;
  if (k_begin < k_end) {
    G128_LOAD(k_begin)
    G128_STORE(As0, As0 + G_IMG)
  }
  __syncthreads();
  for (int64_t kt = k_begin; kt < k_end; kt += G_BK) {
    const int64_t kn = (kt + G_BK < k_end) ? kt + G_BK : kt;
    G128_LOAD(kn)
    // keep the prefetch issued ahead of the MFMA block (hipcc otherwise sinks the loads next to
    // their LDS stores, serializing memory latency and compute)
    __builtin_amdgcn_sched_barrier(0);
    const double* As = As0;
    const double* Bs = As0 + G_IMG;
#pragma unroll
    for (int kk = 0; kk < G_BK / 4; ++kk) {
      const int k = kk * 4 + kq;
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = ATRANS ? As[k * G_SKM + mb + i * 16 + r] : As[(mb + i * 16 + r) * G_SMK + k];
        b[i] = Bs[k * G_SKM + nbs + i * 16 + r];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    G128_STORE(As1, As1 + G_IMG)
    __syncthreads();
    double* tmp = As0;
    As0 = As1;
    As1 = tmp;
  }
#undef G128_LOAD
#undef G128_STORE
#undef G128_LOAD1
#undef G128_STORE1

  double* Ct = C + (int64_t)z * slice_stride;
  if (EPI == EPI_SUB_BAND) {  // C = C0 - acc, C0 passed as loss_part; slice_stride = check flags
    const double* C0 = loss_part;
    int flag = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int64_t row = m0 + mb + i * 16 + acc_row(lane, tt);
          const int64_t col = n0 + nbs + j * 16 + acc_col(lane);
          const double v = C0[row * ldc + col] - acc[i][j][tt];
          C[row * ldc + col] = v;
          flag |= (v + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v) ? 0 : 2);
        }
    if (slice_stride && flag) atomicOr(const_cast<int32_t*>(&st->flags), flag);
    return;
  }
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int64_t row = m0 + mb + i * 16 + acc_row(lane, tt);
          const int64_t col = n0 + nbs + j * 16 + acc_col(lane);
          Ct[row * ldc + col] = acc[i][j][tt];
        }
    return;
  }
  // (sigmoid: the accumulators pass through a per-lane LDS stage so that the transcendental
  // loop can stay rolled without demoting acc to scratch; see gemm_pipe_kernel)
  const bool want_loss = loss_part != nullptr && (st == nullptr || st->ckpt_pending);
  double part = 0.0;
  __syncthreads();
  double* stg = smem + (tid >> 6) * 1024 + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) stg[(4 * j + tt) * 64] = acc[i][j][tt];
#pragma unroll 1
    for (int jt = 0; jt < 16; ++jt) {
      const int j = jt >> 2, tt = jt & 3;
      {
        const int64_t row = m0 + mb + i * 16 + acc_row(lane, tt);
        const int64_t col = n0 + nbs + j * 16 + acc_col(lane);
        const double v = stg[jt * 64];
        if (want_loss && row < m_valid && col < n_valid)  // X[row][col]: A's (m, k) = (row, col)
          part += logaddexp0(v) - (ATRANS ? A[col * lda + row] : A[row * lda + col]) * v;
        Ct[row * ldc + col] = 1.0 / (1.0 + exp(-v));
      }
    }
  }
  if (!want_loss) return;
  __syncthreads();
  double* red = smem;
  red[tid] = part;
  __syncthreads();
  for (int s2 = NTHREADS / 2; s2 > 0; s2 >>= 1) {
    if (tid < s2) red[tid] += red[tid + s2];
    __syncthreads();
  }
  if (tid == 0) loss_part[EPI == EPI_SIGMOID_SPLIT ? blockIdx.x - per_slice : blockIdx.x] = red[0];
}

constexpr size_t kGemm128Lds = 4 * G_IMG * sizeof(double);

// ---- pipelined 128 x 128 tile GEMM (data-mode and cov-mode score GEMMs) --------------------
// The A tile goes through a double-buffered LDS image shared by the 4 waves; each wave owns all
// 128 rows x 32 columns (8 x 2 accumulators) and loads its B values straight into MFMA operand
// registers.  The software pipeline follows the vendor DGEMM's (measured: rocBLAS 94% on the
// X(I-W) shape where the 2 x 2-wave gemm128 above reached 83%):
//   * k is permuted inside a 16-deep tile: lane quarter kq takes k = 4 kq + kk at k-step kk, so
//     one lane's B values of a k-step sit in one row of B, and its two columns 2r, 2r+1 (output
//     column c of accumulator j is n = 2c + j) are one 16-B load;
//   * A image [k][m] with row stride 132 doubles: rows 4 apart differ by 16 mod 32 doubles, so
//     the two kq halves of a 32-lane group use disjoint banks (conflict-free fragment reads);
//   * fragments are read one k-step ahead, interleaved with the MFMAs by sched_group_barrier;
//     the next tile is staged into the other LDS buffer during k-step 1 from registers loaded
//     one tile earlier; one barrier per tile, before the last k-step, so the next tile's first
//     fragments are read while that k-step's MFMAs run;
//   * B row kk of the next tile is reloaded into the same registers right after k-step kk's
//     MFMAs are issued (no loop-carried register copies, which made hipcc drain the loads).
// AMODE 1: A stored [k][m] (lda), AMODE 0: A stored [m][k].  BMODE B_IMINUS forms I - B in
// registers.  Split-K slices as gemm128.  Measured at n = 1e6, d = 1000 (MI355X): X(I-W) from
// X^T 29.1 ms (B = I - W pre-formed, 91.7% of FP64 peak), X^T Y split 16 28.7 ms (92.8%).
constexpr int P_S = 132;
constexpr int P_IMG = 16 * P_S;
constexpr size_t kGemmPipeLds = 2 * P_IMG * sizeof(double);

// The serial split sigmoid GEMM's per-tile hand-off (EPI_SIGMOID_SPLIT).  Every launch pairs
// exactly one signal with exactly one take per tile, whatever the status word does during the
// launch: a first half always signals (SIG_RAN after its partial is stored and released,
// SIG_SKIPPED when it is gated off), a second half always takes the word and clears it, and uses
// the partial only after SIG_RAN.  So every word is 0 again when the launch ends, and a take can
// never see an earlier launch's signal.  Both halves of a tile sit on one XCD (launch_gemm: tiles
// % 8 == 0), and every first half precedes every second half in the grid, so each wait is on a
// workgroup already dispatched; the wait is bounded (50 ms) all the same, and an expired one
// sets ST_HANDOFF_TIMEOUT, on which the host clears the words and raises.
enum SigSplitWord : int { SIG_RAN = 1, SIG_SKIPPED = 2 };

__device__ __forceinline__ void sig_split_signal(int* flag, int word) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// returns the first half's word (0: the wait expired); sh: one int of LDS
__device__ __forceinline__ int sig_split_take(int* flag, const State* st, int* sh) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int got = 0;
    for (;;) {
      got = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (got != 0) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000) break;  // 50 ms
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (got != 0)
      __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (st)
      __hip_atomic_store(const_cast<int32_t*>(&st->status), (int32_t)ST_HANDOFF_TIMEOUT, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    *sh = got;
  }
  __syncthreads();
  return *sh;
}

// One 128 x 128 output tile (t: its index after the XCD remap) of the pipelined GEMM; smem:
// kGemmPipeLds bytes.  The body of gemm_pipe_kernel, and of the launch that runs the cov score
// GEMM beside the blocked inverse's last trailing update (gemm_trail_kernel).
template <int AMODE, int BMODE, int EPI>
__device__ __forceinline__ void gemm_pipe_tile(int t, int64_t K, int64_t kslice, int tiles_m, int tiles_n,
                                               const double* __restrict__ A, int64_t lda,
                                               const double* __restrict__ B, int64_t ldb, double* __restrict__ C,
                                               int64_t ldc, int64_t slice_stride, double* __restrict__ loss_part,
                                               int64_t m_valid, int64_t n_valid, const State* __restrict__ st,
                                               double* __restrict__ smem) {
  const int per_slice = tiles_m * tiles_n;
  const int z = t / per_slice, rem = t % per_slice;
  int bm, bn;
  if (EPI == EPI_SUB_CROSS || EPI == EPI_SUB_CROSS_MID) {
    // look-ahead part of a trailing update (launch_trail128_split): the tiles in the row or column
    // band of the NEXT outer block, which sits right after the pivot band b = m_valid, nb =
    // n_valid tiles wide; tiles_m = the trailing grid's edge (pivot band skipped), tiles_n = 2 nb
    // (so that tiles_m tiles_n covers the grid and z = 0)
    const int b = (int)m_valid, nb = (int)n_valid, tm = tiles_m;
    if (t < nb * tm) {
      bm = b + t / tm;
      bn = t % tm;
    } else {
      const int u = t - nb * tm, ri = u / nb;
      bm = ri < b ? ri : ri + nb;
      bn = b + u % nb;
    }
    bm += bm >= b ? nb : 0;  // skip the pivot band
    bn += bn >= b ? nb : 0;
  } else if (tiles_n > 8) {
    // grouped order: the 64 consecutive tiles one XCD holds resident (32 CUs x 2) form an
    // 8 x 8 block, so its L2 serves each A row panel and B column panel to 8 tiles (row-major
    // order put 40 different B panels in flight per XCD at d = 5000)
    const int gsz = 8 * tiles_n, g = rem / gsz, w_ = rem - g * gsz;
    const int fm = g * 8, rows = tiles_m - fm < 8 ? tiles_m - fm : 8;
    bm = fm + w_ % rows;
    bn = w_ / rows;
  } else {
    bm = rem / tiles_n;
    bn = rem % tiles_n;
  }
  if (EPI == EPI_SUB_BAND || EPI == EPI_SUB_PRE || EPI == EPI_SUB_MID) {
    // trailing update of the blocked inverse: the tile grid skips the pivot band
    // [m_valid, m_valid + n_valid) (in 128-tiles) in both rows and columns
    bm += bm >= (int)m_valid ? (int)n_valid : 0;
    bn += bn >= (int)m_valid ? (int)n_valid : 0;
  }
  const int64_t m0 = (int64_t)bm * 128, n0 = (int64_t)bn * 128;
  const int64_t k_begin = (int64_t)z * kslice;
  const int64_t k_end = (k_begin + kslice < K) ? k_begin + kslice : K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int64_t nw = n0 + 32 * w;

  // A staging, 4 x 16 B per thread per tile.  AMODE 1: item i_ -> k = i_ >> 6, m = 2 (i_ & 63)
  // (+1), one ds_write_b128.  AMODE 0: item i_ -> k = 2 (i_ >> 7) (+1), m = i_ & 127, two
  // ds_write_b64 (consecutive lanes on consecutive m: conflict-free).
  const double* Ablk = AMODE ? A + m0 : A + m0 * lda;
  int offA[4], ldsA[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i_ = it * NTHREADS + tid;
    if (AMODE) {
      offA[it] = (i_ >> 6) * (int)lda + 2 * (i_ & 63);
      ldsA[it] = (i_ >> 6) * P_S + 2 * (i_ & 63);
    } else {
      offA[it] = (i_ & 127) * (int)lda + 2 * (i_ >> 7);
      ldsA[it] = 2 * (i_ >> 7) * P_S + (i_ & 127);
    }
  }
  const int64_t a_kstride = AMODE ? lda : 1;
  const double* Bw = B + (int64_t)(4 * kq) * ldb + nw + 2 * r;
  const int fo = 4 * kq * P_S + r;  // fragment of block i at k-step kk: fo + kk P_S + 16 i

  double2 ra0, ra1, ra2, ra3;
  double2 fb[4];
  double fa0[8], fa1[8];
#define GP_LOADA(KT)                                                                              \
  {                                                                                               \
    const double* ap_ = Ablk + (KT) * a_kstride;                                                  \
    ra0 = *reinterpret_cast<const double2*>(ap_ + offA[0]);                                       \
    ra1 = *reinterpret_cast<const double2*>(ap_ + offA[1]);                                       \
    ra2 = *reinterpret_cast<const double2*>(ap_ + offA[2]);                                       \
    ra3 = *reinterpret_cast<const double2*>(ap_ + offA[3]);                                       \
  }
#define GP_LOADB1(KT, KK) fb[KK] = *reinterpret_cast<const double2*>(Bw + ((KT) + (KK)) * ldb);
#define GP_STA1(AS, I, RA)                                                                        \
  if (AMODE) {                                                                                    \
    *reinterpret_cast<double2*>((AS) + ldsA[I]) = RA;                                             \
  } else {                                                                                        \
    (AS)[ldsA[I]] = RA.x;                                                                         \
    (AS)[ldsA[I] + P_S] = RA.y;                                                                   \
  }
#define GP_STOREA(AS)                                                                             \
  {                                                                                               \
    GP_STA1(AS, 0, ra0) GP_STA1(AS, 1, ra1) GP_STA1(AS, 2, ra2) GP_STA1(AS, 3, ra3)               \
  }
#define GP_FRAG(DST, AS, KK)                                                                      \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) DST[i_] = (AS)[fo + (KK) * P_S + 16 * i_];   \
  }
#define GP_MMA(FA, KT, KK)                                                                        \
  {                                                                                               \
    double b0_ = fb[KK].x, b1_ = fb[KK].y;                                                        \
    if (BMODE == B_IMINUS) {                                                                      \
      const int64_t kg_ = (KT) + 4 * kq + (KK), ng_ = nw + 2 * r;                                 \
      b0_ = (kg_ == ng_ ? 1.0 : 0.0) - b0_;                                                       \
      b1_ = (kg_ == ng_ + 1 ? 1.0 : 0.0) - b1_;                                                   \
    }                                                                                             \
    if (EPI == EPI_SUB_PRE) {                                                                     \
      b0_ = -b0_;                                                                                 \
      b1_ = -b1_;                                                                                 \
    }                                                                                             \
    _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) {                                            \
      acc[i_][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(FA[i_], b0_, acc[i_][0], 0, 0, 0);         \
      acc[i_][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(FA[i_], b1_, acc[i_][1], 0, 0, 0);         \
    }                                                                                             \
  }
  // instruction interleave of one k-step: its 8 fragment reads (for the next k-step) between the
  // first MFMAs, then NW LDS stores and NV global loads between the following ones
#define GP_SCHED(NW, NV)                                                                          \
  {                                                                                               \
    _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_) {                                            \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    }                                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < (NW); ++q_) {                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                          \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                                          \
    }                                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < (NV); ++q_) {                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                          \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    }                                                                                             \
    __builtin_amdgcn_sched_group_barrier(0x008, 16 - 8 - (NW) - (NV), 0);                        \
  }

  dbl4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  double* As0 = smem;
  double* As1 = smem + P_IMG;
  if (k_begin < k_end) {
    GP_LOADA(k_begin)
#pragma unroll
    for (int q = 0; q < 4; ++q) GP_LOADB1(k_begin, q)
    if (EPI == EPI_SUB_PRE) {
      // C = C0 + sum (-a) b: the accumulators start from C0 (loads issued behind the first
      // operand tile, so they overlap the prologue instead of a load-then-store epilogue)
      const double* C0 = loss_part;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int64_t row = m0 + 16 * i + acc_row(lane, tt);
          const int64_t col = nw + 2 * acc_col(lane);
          const double2 c0 = *reinterpret_cast<const double2*>(C0 + row * ldc + col);
          acc[i][0][tt] = c0.x;
          acc[i][1][tt] = c0.y;
        }
    }
    GP_STOREA(As0)
    GP_LOADA((k_begin + 16 < k_end) ? k_begin + 16 : k_begin)
    __syncthreads();
    GP_FRAG(fa0, As0, 0)
  }
  // EPI_SUB_MID (K = 256 exactly, 16 K-tiles): C0 is read in 16 half-blocks (8 rows x 16
  // columns of each of a lane's two accumulator columns) over the 16 K-tiles, each loaded one K-tile ahead of its fold
  // acc -= C0 (8 extra VGPRs), so the C0 traffic overlaps the MFMAs instead of the epilogue's
  // burst of every resident tile at once; acc ends as A B - C0 and is stored negated
  constexpr bool kFold = EPI == EPI_SUB_MID || EPI == EPI_SUB_CROSS_MID;
  const int nit = kFold ? 16 : (int)((k_end - k_begin + 15) / 16);
  const double* C0m = loss_part;
  double2 c0r[2];
  // (addresses: a wave-uniform row base (SGPRs) plus one per-lane 32-bit offset, so the 32 loads
  // of the unrolled loop hold no 64-bit address registers)
  const int64_t nwu = n0 + 32 * __builtin_amdgcn_readfirstlane(w);
  const int c0lane = acc_row(lane, 0) * (int)ldc + 2 * acc_col(lane);
  const int c0dt = acc_row(lane, 1) - acc_row(lane, 0);  // row step of accumulator element tt
#define GP_C0LOAD(H)                                                                              \
  {                                                                                               \
    _Pragma("unroll") for (int u_ = 0; u_ < 2; ++u_) c0r[u_] = *reinterpret_cast<const double2*>(  \
        C0m + ((m0 + 16 * ((H) >> 1) + c0dt * (2 * ((H) & 1) + u_)) * ldc + nwu) + c0lane);       \
  }
#define GP_C0FOLD(H)                                                                              \
  {                                                                                               \
    _Pragma("unroll") for (int u_ = 0; u_ < 2; ++u_) {                                            \
      acc[(H) >> 1][0][2 * ((H) & 1) + u_] -= c0r[u_].x;                                          \
      acc[(H) >> 1][1][2 * ((H) & 1) + u_] -= c0r[u_].y;                                          \
    }                                                                                             \
  }
  // (the MID loop is unrolled over its fixed 16 K-tiles, so every fold and load index is a
  // constant and acc stays in registers; a run-time switch over the folds spilled it)
  constexpr int kUnroll = kFold ? 16 : 1;
  const int nit_loop = kFold ? 16 : nit;
  __builtin_amdgcn_s_setprio(3);
#pragma unroll kUnroll
  for (int it = 0; it < nit_loop; ++it) {
    const int64_t kt = k_begin + 16 * (int64_t)it;
    const int64_t k1 = kt + 16 < k_end ? kt + 16 : kt;
    const int64_t k2 = kt + 32 < k_end ? kt + 32 : k1;
    if (kFold) {
      const int h = it - (nit - 16) - 1;  // half-block folded in this K-tile (15: after the loop)
      switch (h) {
        case 0: GP_C0FOLD(0) break;
        case 1: GP_C0FOLD(1) break;
        case 2: GP_C0FOLD(2) break;
        case 3: GP_C0FOLD(3) break;
        case 4: GP_C0FOLD(4) break;
        case 5: GP_C0FOLD(5) break;
        case 6: GP_C0FOLD(6) break;
        case 7: GP_C0FOLD(7) break;
        case 8: GP_C0FOLD(8) break;
        case 9: GP_C0FOLD(9) break;
        case 10: GP_C0FOLD(10) break;
        case 11: GP_C0FOLD(11) break;
        case 12: GP_C0FOLD(12) break;
        case 13: GP_C0FOLD(13) break;
        case 14: GP_C0FOLD(14) break;
        default: break;
      }
      if (h >= -1 && h < 15) GP_C0LOAD(h + 1)
      __builtin_amdgcn_sched_barrier(0);
    }
    GP_FRAG(fa1, As0, 1)  // k-step 0
    GP_MMA(fa0, kt, 0)
    GP_LOADB1(k1, 0)
    GP_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    GP_STOREA(As1)  // k-step 1: stage the next tile, then load the one after it
    GP_FRAG(fa0, As0, 2)
    GP_MMA(fa1, kt, 1)
    GP_LOADB1(k1, 1)
    GP_LOADA(k2)
    GP_SCHED(AMODE ? 4 : 8, 5)
    __builtin_amdgcn_sched_barrier(0);
    GP_FRAG(fa1, As0, 3)  // k-step 2
    GP_MMA(fa0, kt, 2)
    GP_LOADB1(k1, 2)
    GP_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    __builtin_amdgcn_s_setprio(3);
    GP_FRAG(fa0, As1, 0)  // k-step 3, reading the next tile's first fragments meanwhile
    GP_MMA(fa1, kt, 3)
    GP_LOADB1(k1, 3)
    GP_SCHED(0, 1)
    __builtin_amdgcn_sched_barrier(0);
    double* tmp = As0;
    As0 = As1;
    As1 = tmp;
  }
  __builtin_amdgcn_s_setprio(0);
#undef GP_LOADA
#undef GP_LOADB1
#undef GP_STA1
#undef GP_STOREA
#undef GP_FRAG
#undef GP_MMA
#undef GP_SCHED
  if (kFold) {  // acc = A B - C0 once the last half-block is folded; slice_stride = check
    GP_C0FOLD(15)
    int flag = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int64_t row = m0 + 16 * i + acc_row(lane, tt);
        const int64_t col = nw + 2 * acc_col(lane);
        const double2 v = double2{-acc[i][0][tt], -acc[i][1][tt]};
        *reinterpret_cast<double2*>(C + row * ldc + col) = v;
        flag |= (v.x + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.x) ? 0 : 2);
        flag |= (v.y + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.y) ? 0 : 2);
      }
    if (slice_stride && flag) atomicOr(const_cast<int32_t*>(&st->flags), flag);
    return;
  }
#undef GP_C0LOAD
#undef GP_C0FOLD
  if (EPI == EPI_SUB_PRE) {  // acc = C0 - A B already; slice_stride = check
    int flag = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int64_t row = m0 + 16 * i + acc_row(lane, tt);
        const int64_t col = nw + 2 * acc_col(lane);
        const double2 v = double2{acc[i][0][tt], acc[i][1][tt]};
        *reinterpret_cast<double2*>(C + row * ldc + col) = v;
        flag |= (v.x + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.x) ? 0 : 2);
        flag |= (v.y + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.y) ? 0 : 2);
      }
    if (slice_stride && flag) atomicOr(const_cast<int32_t*>(&st->flags), flag);
    return;
  }
  if (EPI == EPI_SUB_BAND || EPI == EPI_SUB_CROSS) {  // C = C0 - acc, C0 as loss_part; slice_stride = check
    const double* C0 = loss_part;
    int flag = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int64_t row = m0 + 16 * i + acc_row(lane, tt);
        const int64_t col = nw + 2 * acc_col(lane);
        const double2 c0 = *reinterpret_cast<const double2*>(C0 + row * ldc + col);
        const double2 v = double2{c0.x - acc[i][0][tt], c0.y - acc[i][1][tt]};
        *reinterpret_cast<double2*>(C + row * ldc + col) = v;
        flag |= (v.x + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.x) ? 0 : 2);
        flag |= (v.y + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v.y) ? 0 : 2);
      }
    if (slice_stride && flag) atomicOr(const_cast<int32_t*>(&st->flags), flag);
    return;
  }
  double* Ct = C + (int64_t)z * slice_stride;
  if (EPI == EPI_SIGMOID_SPLIT) {
    // serial split-K of the sigmoid GEMM (two K halves; launch_gemm: grids of few tiles): the
    // first half stores its partial at C + slice_stride and hands it over through the tile's flag
    // (int words after the partial; protocol: sig_split_signal / sig_split_take); the second half
    // adds it while staging the epilogue, which then runs on the full sum and writes C.
    int* flag = reinterpret_cast<int*>(C + 2 * slice_stride) + rem;
    if (z == 0) {
      double* Pt = C + slice_stride;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int64_t row = m0 + 16 * i + acc_row(lane, tt);
          const int64_t col = nw + 2 * acc_col(lane);
          *reinterpret_cast<double2*>(Pt + row * ldc + col) = double2{acc[i][0][tt], acc[i][1][tt]};
        }
      sig_split_signal(flag, SIG_RAN);
      return;
    }
    __syncthreads();  // (every wave is done with the A images: the take's word overlays them)
    if (sig_split_take(flag, st, reinterpret_cast<int*>(smem)) != SIG_RAN) return;
    Ct = C;
  }
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int64_t row = m0 + 16 * i + acc_row(lane, tt);
        const int64_t col = nw + 2 * acc_col(lane);
        *reinterpret_cast<double2*>(Ct + row * ldc + col) = double2{acc[i][0][tt], acc[i][1][tt]};
      }
    return;
  }
  // EPI_SIGMOID: C = expit(acc); loss partial sum(logaddexp(0, acc) - X * acc) over the valid
  // block, X = op(A) at (row, col).
  // The 64 accumulators stay in registers only while every index into acc is a compile-time
  // constant, and the f64 exp / log bodies are too large to unroll 64 times: hipcc then keeps
  // acc in scratch for the whole kernel (544 B/lane, the GEMM 5x slower).  So each 16-row block
  // is parked in a per-lane LDS stage with constant indices, and a rolled loop does the
  // transcendental work.  A lane reads back only its own slots (no barrier inside).
  const bool want_loss = loss_part != nullptr && (st == nullptr || st->ckpt_pending);
  double part = 0.0;
  __syncthreads();  // every wave is done with the A images the stage overlays
  double* stg = smem + w * 512 + lane;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      if (EPI == EPI_SIGMOID_SPLIT) {  // the first K half's partial + this half (fixed order)
        const int64_t row = m0 + 16 * i + acc_row(lane, tt), col = nw + 2 * acc_col(lane);
        const double2 p = *reinterpret_cast<const double2*>(C + slice_stride + row * ldc + col);
        stg[(2 * tt) * 64] = p.x + acc[i][0][tt];
        stg[(2 * tt + 1) * 64] = p.y + acc[i][1][tt];
      } else {
        stg[(2 * tt) * 64] = acc[i][0][tt];
        stg[(2 * tt + 1) * 64] = acc[i][1][tt];
      }
    }
#pragma unroll 1
    for (int tt = 0; tt < 4; ++tt) {
      const int64_t row = m0 + 16 * i + acc_row(lane, tt);
      const int64_t col = nw + 2 * acc_col(lane);
      double2 o;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double v = stg[(2 * tt + j) * 64];
        if (want_loss && row < m_valid && col + j < n_valid)
          part += logaddexp0(v) - (AMODE ? A[(col + j) * lda + row] : A[row * lda + col + j]) * v;
        (j ? o.y : o.x) = 1.0 / (1.0 + exp(-v));
      }
      *reinterpret_cast<double2*>(Ct + row * ldc + col) = o;
    }
  }
  if (!want_loss) return;
  __syncthreads();
  double* red = smem;
  red[tid] = part;
  __syncthreads();
  for (int s2 = NTHREADS / 2; s2 > 0; s2 >>= 1) {
    if (tid < s2) red[tid] += red[tid + s2];
    __syncthreads();
  }
  if (tid == 0) loss_part[EPI == EPI_SIGMOID_SPLIT ? blockIdx.x - per_slice : blockIdx.x] = red[0];
}

template <int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_pipe_kernel(int64_t K, int64_t kslice, int tiles_m, int tiles_n,
                                                                const double* __restrict__ A, int64_t lda,
                                                                const double* __restrict__ B, int64_t ldb,
                                                                double* __restrict__ C, int64_t ldc,
                                                                int64_t slice_stride, double* __restrict__ loss_part,
                                                                int64_t m_valid, int64_t n_valid,
                                                                const State* __restrict__ st) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  int t = xcd_remap(blockIdx.x, gridDim.x);
  if (EPI == EPI_SIGMOID_SPLIT) {  // (serial split: the K halves in grid order, z-major)
    const int per = tiles_m * tiles_n, b = blockIdx.x, z = b >= per ? 1 : 0;
    t = z * per + xcd_remap(b - z * per, per);
    if (st && st->status != ST_RUNNING) {
      // a gated-off half still takes part in its tile's hand-off, so every flag a launch sets is
      // also cleared by it (the status may leave ST_RUNNING mid-launch: a hand-back of the
      // inverse forked beside this GEMM)
      int* flag = reinterpret_cast<int*>(C + 2 * slice_stride) + (t - z * per);
      if (z == 0)
        sig_split_signal(flag, SIG_SKIPPED);
      else
        (void)sig_split_take(flag, st, reinterpret_cast<int*>(smem));
      return;
    }
  } else if (st && st->status != ST_RUNNING) {
    return;
  }
  gemm_pipe_tile<AMODE, BMODE, EPI>(t, K, kslice, tiles_m, tiles_n, A, lda, B, ldb, C, ldc, slice_stride, loss_part,
                                    m_valid, n_valid, st, smem);
}


// The cov score GEMM and the blocked inverse's LAST trailing update in one launch: the first
// n_gemm workgroups run gemm_pipe_tile (the GEMM's own launch, bit-identical), the rest the
// 32 x 32 trailing tiles (binv_trail_tile).  The GEMM reads W and cov only, so it needs nothing
// of the inverse; the trailing tiles (≈12 us at d = 1000) run beside it instead of as a
// launch of their own.
struct GemmTrailArgs {
  int64_t K, kslice;
  int tm, tn, n_gemm;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  double* C;
  int64_t ldc, slice_stride;
  const double* Ain;
  double* Aout;
  int64_t D;
  int B2, g, check, pf;
  State* st;
  const Params* pr;         // control folded into the launch (ticket non-null; control.h)
  const double* bc_table;
  int* ticket;
};
constexpr size_t kGemmTrailLds = (4 * NB * ST * sizeof(double) > kGemmPipeLds) ? 4 * NB * ST * sizeof(double)
                                                                                : kGemmPipeLds;

// a gated-off launch with the control folded in: the control kernel's NOOP for this slot
__device__ __forceinline__ bool gemm_trail_gated(const GemmTrailArgs& a) {
  if (a.st->status == ST_RUNNING) return false;
  if (a.ticket && blockIdx.x == 0 && threadIdx.x == 0) a.st->action = ACT_NOOP;
  return true;
}

template <int AMODE, int BMODE>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_trail_kernel(GemmTrailArgs a) {
  if (gemm_trail_gated(a)) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  if (b < a.n_gemm) {
    gemm_pipe_tile<AMODE, BMODE, EPI_STORE>(xcd_remap(b, a.n_gemm), a.K, a.kslice, a.tm, a.tn, a.A, a.lda, a.B, a.ldb,
                                            a.C, a.ldc, a.slice_stride, nullptr, 0, 0, a.st, smem);
  } else {
    binv_trail_tile(xcd_spread(b - a.n_gemm, (int)gridDim.x - a.n_gemm), a.Ain, a.Aout, a.D, a.B2, a.g, a.check, a.st,
                    a.pf, smem, smem + NB * ST, smem + 2 * NB * ST, smem + 3 * NB * ST);
  }
  if (a.ticket) control_fold_tail(a.pr, a.st, a.bc_table, a.ticket);
}

// experiment knob MIDAGMA_EXP_TRAIL_EPI=1: C0 read in the epilogue at every B2
// (the 128-tile trailing updates; B2 = 256 otherwise folds it in during the K loop)
static bool trail_mid() {
  static const bool epi = knob_set("MIDAGMA_EXP_TRAIL_EPI");
  return !epi;
}

// The same pairing at large D, where the trailing update itself runs on the 128-tile GEMM
// (launch_trail128): the score GEMM's tiles, then the band-skipping C0 - A B tiles.
struct Gemm2Args {
  GemmTrailArgs g;  // the score GEMM (its trailing-update fields unused)
  int tm2;          // trailing tiles per dimension: (D - B2) / 128
  int mid;          // B2 = 256: C0 folded in during the K loop (EPI_SUB_MID, launch_trail128)
};

template <int AMODE, int BMODE>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_trail128_kernel(Gemm2Args a2) {
  const GemmTrailArgs& a = a2.g;
  if (gemm_trail_gated(a)) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  if (b < a.n_gemm) {
    gemm_pipe_tile<AMODE, BMODE, EPI_STORE>(xcd_remap(b, a.n_gemm), a.K, a.kslice, a.tm, a.tn, a.A, a.lda, a.B, a.ldb,
                                            a.C, a.ldc, a.slice_stride, nullptr, 0, 0, a.st, smem);
  } else {
    const int64_t G0 = (int64_t)a.g * a.B2;
    if (a2.mid)
      gemm_pipe_tile<0, B_PLAIN, EPI_SUB_MID>(xcd_remap(b - a.n_gemm, (int)gridDim.x - a.n_gemm), a.B2, a.B2, a2.tm2,
                                              a2.tm2, a.Ain + G0, a.D, a.Aout + G0 * a.D, a.D, a.Aout, a.D,
                                              (int64_t)a.check, const_cast<double*>(a.Ain), G0 / 128, a.B2 / 128,
                                              a.st, smem);
    else
      gemm_pipe_tile<0, B_PLAIN, EPI_SUB_BAND>(xcd_remap(b - a.n_gemm, (int)gridDim.x - a.n_gemm), a.B2, a.B2, a2.tm2,
                                               a2.tm2, a.Ain + G0, a.D, a.Aout + G0 * a.D, a.D, a.Aout, a.D,
                                               (int64_t)a.check, const_cast<double*>(a.Ain), G0 / 128, a.B2 / 128,
                                               a.st, smem);
  }
  if (a.ticket) control_fold_tail(a.pr, a.st, a.bc_table, a.ticket);
}

constexpr size_t kGemmLds = (2 * 64 * SB) * sizeof(double);

template <bool AT, int BM, int EP>
static void set_attr() {
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<AT, BM, EP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemmLds));
}

template <bool AT, int BM, int EP>
static void set_attr128() {
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm128_kernel<AT, BM, EP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemm128Lds));
}

template <int AM, int BM, int EP>
static void set_attr_pipe() {
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pipe_kernel<AM, BM, EP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemmPipeLds));
}

template <int AM, int BM>
static void set_attr_gt() {
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_trail_kernel<AM, BM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemmTrailLds));
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_trail128_kernel<AM, BM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemmPipeLds));
}

void gemm_setup_attributes() {
  set_attr_gt<1, B_PLAIN>();
  set_attr_gt<1, B_IMINUS>();
  set_attr_gt<0, B_PLAIN>();
  set_attr_gt<0, B_IMINUS>();
  set_attr_pipe<1, B_PLAIN, EPI_STORE>();
  set_attr_pipe<1, B_IMINUS, EPI_STORE>();
  set_attr_pipe<0, B_PLAIN, EPI_STORE>();
  set_attr_pipe<0, B_IMINUS, EPI_STORE>();
  set_attr_pipe<1, B_PLAIN, EPI_SIGMOID>();
  set_attr_pipe<0, B_PLAIN, EPI_SIGMOID>();
  set_attr_pipe<1, B_PLAIN, EPI_SIGMOID_SPLIT>();
  set_attr_pipe<0, B_PLAIN, EPI_SIGMOID_SPLIT>();
  set_attr_pipe<0, B_PLAIN, EPI_SUB_BAND>();
  set_attr_pipe<0, B_PLAIN, EPI_SUB_CROSS>();
  set_attr_pipe<0, B_PLAIN, EPI_SUB_CROSS_MID>();
#ifdef MIDAGMA_EXPERIMENTS
  set_attr_pipe<0, B_PLAIN, EPI_SUB_PRE>();
#endif
  set_attr128<false, B_PLAIN, EPI_STORE>();
  set_attr128<false, B_IMINUS, EPI_STORE>();
  set_attr128<true, B_PLAIN, EPI_STORE>();
  set_attr128<true, B_IMINUS, EPI_STORE>();
  set_attr128<false, B_PLAIN, EPI_SIGMOID>();
  set_attr128<true, B_PLAIN, EPI_SIGMOID>();
  set_attr128<false, B_PLAIN, EPI_SUB_BAND>();
  set_attr<false, B_PLAIN, EPI_STORE>();
  set_attr<false, B_IMINUS, EPI_STORE>();
  set_attr<true, B_PLAIN, EPI_STORE>();
  set_attr<true, B_IMINUS, EPI_STORE>();
  set_attr<false, B_PLAIN, EPI_SIGMOID>();
}

void launch_gemm(int64_t M, int64_t N, int64_t K, const double* A, int64_t lda, bool a_trans, const double* B,
                 int64_t ldb, GemmB bmode, double* C, int64_t ldc, GemmEpi epi, int split, int64_t slice_stride,
                 double* loss_part, int64_t m_valid, int64_t n_valid, const State* st, hipStream_t stream) {
  // (K % 16 suffices for the pipelined kernel: the k loop of a padded problem may stop at the
  // first 16-multiple past the logical size, the rest of A's k range being zero)
  if (M % 64 || N % 64 || K % 16 || split < 1) throw std::invalid_argument("launch_gemm: bad shape");
  static const bool force64 = knob_set("MIDAGMA_EXP_GEMM64");  // experiment knobs (knobs.h)
  static const bool no_pipe = knob_set("MIDAGMA_EXP_NO_PIPE");
  if (M % 128 == 0 && N % 128 == 0 && K % 16 == 0 && !force64 && !no_pipe &&
      (epi == EPI_STORE || (epi == EPI_SIGMOID && (split == 1 || split == 2) && bmode == B_PLAIN))) {
    const int64_t ktiles16 = K / 16;
    const int64_t per16 = (ktiles16 + split - 1) / split;
    const int nsplit = (int)((ktiles16 + per16 - 1) / per16);
    const int tm = (int)(M / 128), tn = (int)(N / 128);
    const int64_t nwg = (int64_t)tm * tn * nsplit;
    const int64_t kslice = per16 * 16;
    if (epi == EPI_SIGMOID && nsplit > 1 && (nsplit != 2 || (tm * tn) % 8 || slice_stride < M * ldc))
      throw std::invalid_argument("launch_gemm: the serial split sigmoid needs 2 slices, tiles % 8 == 0 and C with "
                                  "room for the partial and the flags");
#define MIDAGMA_GEMMP(AM, BM, EP)                                                                         \
  hipLaunchKernelGGL((gemm_pipe_kernel<AM, BM, EP>), dim3((unsigned)nwg), dim3(NTHREADS), kGemmPipeLds, stream, K, \
                     kslice, tm, tn, A, lda, B, ldb, C, ldc, slice_stride, loss_part, m_valid, n_valid, st)
    if (epi == EPI_SIGMOID) {
      if (K > N) throw std::invalid_argument("launch_gemm: sigmoid form (op(A) is X: K <= N)");
      if (nsplit > 1 && a_trans)
        MIDAGMA_GEMMP(1, B_PLAIN, EPI_SIGMOID_SPLIT);
      else if (nsplit > 1)
        MIDAGMA_GEMMP(0, B_PLAIN, EPI_SIGMOID_SPLIT);
      else if (a_trans)
        MIDAGMA_GEMMP(1, B_PLAIN, EPI_SIGMOID);
      else
        MIDAGMA_GEMMP(0, B_PLAIN, EPI_SIGMOID);
    } else if (a_trans && bmode == B_PLAIN) {
      MIDAGMA_GEMMP(1, B_PLAIN, EPI_STORE);
    } else if (a_trans) {
      MIDAGMA_GEMMP(1, B_IMINUS, EPI_STORE);
    } else if (bmode == B_PLAIN) {
      MIDAGMA_GEMMP(0, B_PLAIN, EPI_STORE);
    } else {
      MIDAGMA_GEMMP(0, B_IMINUS, EPI_STORE);
    }
#undef MIDAGMA_GEMMP
    HIP_TRY(hipGetLastError());
    return;
  }
  // the older kernels step K by 64: a k extent cut at a 16-multiple (Kd(): the operands' rows
  // past it are zero and allocated up to the 64-padded size) is rounded back up
  if (K % 64) K = (K + 63) / 64 * 64;
  if (M % 128 == 0 && N % 128 == 0 && K % 128 == 0 && !force64) {
    const int64_t ktiles16 = K / G_BK;
    const int64_t per16 = (ktiles16 + split - 1) / split;
    const int nsplit = (int)((ktiles16 + per16 - 1) / per16);
    const int tm = (int)(M / G_BM), tn = (int)(N / G_BN);
    const int64_t nwg = (int64_t)tm * tn * nsplit;
    const int64_t kslice = per16 * G_BK;
#define MIDAGMA_GEMM128(AT, BM, EP)                                                                       \
  hipLaunchKernelGGL((gemm128_kernel<AT, BM, EP>), dim3((unsigned)nwg), dim3(NTHREADS), kGemm128Lds, stream, K, \
                     kslice, tm, tn, A, lda, B, ldb, C, ldc, slice_stride, loss_part, m_valid, n_valid, st)
    if (epi == EPI_SIGMOID) {
      // (a_trans: the epilogue reads X[m][n] from X^T's row n < N; X^T has D >= N rows, zero past d,
      // so the k loop may stop short of N as in the pipelined kernel)
      if (bmode != B_PLAIN || nsplit != 1 || (a_trans && K > N))
        throw std::invalid_argument("launch_gemm: sigmoid form");
      if (a_trans)
        MIDAGMA_GEMM128(true, B_PLAIN, EPI_SIGMOID);
      else
        MIDAGMA_GEMM128(false, B_PLAIN, EPI_SIGMOID);
    } else if (epi == EPI_SUB_BAND) {
      throw std::invalid_argument("launch_gemm: use launch_trail128");
    } else if (!a_trans && bmode == B_PLAIN) {
      MIDAGMA_GEMM128(false, B_PLAIN, EPI_STORE);
    } else if (!a_trans) {
      MIDAGMA_GEMM128(false, B_IMINUS, EPI_STORE);
    } else if (bmode == B_PLAIN) {
      MIDAGMA_GEMM128(true, B_PLAIN, EPI_STORE);
    } else {
      MIDAGMA_GEMM128(true, B_IMINUS, EPI_STORE);
    }
#undef MIDAGMA_GEMM128
    HIP_TRY(hipGetLastError());
    return;
  }
  const int64_t ktiles = K / 64;
  const int64_t per = (ktiles + split - 1) / split;
  const int nsplit = (int)((ktiles + per - 1) / per);
  dim3 grid((unsigned)(N / 64), (unsigned)(M / 64), (unsigned)nsplit);
  const int64_t kslice = per * 64;
#define MIDAGMA_GEMM(AT, BM, EP)                                                                         \
  hipLaunchKernelGGL((gemm_kernel<AT, BM, EP>), grid, dim3(NTHREADS), kGemmLds, stream, K, kslice, A, lda, B, \
                     ldb, C, ldc, slice_stride, loss_part, m_valid, n_valid, st)
  if (epi == EPI_SIGMOID) {
    if (a_trans || bmode != B_PLAIN || nsplit != 1) throw std::invalid_argument("launch_gemm: sigmoid form");
    MIDAGMA_GEMM(false, B_PLAIN, EPI_SIGMOID);
  } else if (!a_trans && bmode == B_PLAIN) {
    MIDAGMA_GEMM(false, B_PLAIN, EPI_STORE);
  } else if (!a_trans) {
    MIDAGMA_GEMM(false, B_IMINUS, EPI_STORE);
  } else if (bmode == B_PLAIN) {
    MIDAGMA_GEMM(true, B_PLAIN, EPI_STORE);
  } else {
    MIDAGMA_GEMM(true, B_IMINUS, EPI_STORE);
  }
#undef MIDAGMA_GEMM
  HIP_TRY(hipGetLastError());
}

// The EPI_SUB_MID / EPI_SUB_CROSS_MID tile bodies fold C0 over exactly 16 K-tiles of one K slice
// (the loop is unrolled with compile-time fold indices), and a workgroup past the tile count would
// fold nothing: every launcher of them checks that shape on the host.
static void check_mid_shape(int64_t K, int64_t kslice, int64_t tiles, int64_t grid, const char* who) {
  if (K != 256 || kslice != K || grid > tiles)
    throw std::invalid_argument(std::string(who) + ": the C0 fold needs K = kslice = 256 and grid <= tiles");
}

bool gemm_trail_supported(const GemmSpec& gs) {
  return gs.M % 128 == 0 && gs.N % 128 == 0 && gs.K % 16 == 0 && gs.split >= 1 &&
         !knob_set("MIDAGMA_EXP_GEMM64") && !knob_set("MIDAGMA_EXP_NO_PIPE");
}

// n_trail < 0: the trailing update of the 128-tile kind (launch_trail128's grid)
void launch_gemm_trail(const GemmSpec& gs, const double* Ain, double* Aout, int64_t D, int B2, int g, bool check,
                       State* st, int pf, int n_trail, hipStream_t stream) {
  if (!gemm_trail_supported(gs)) throw std::invalid_argument("launch_gemm_trail: shape");
  const int64_t ktiles16 = gs.K / 16;
  const int64_t per16 = (ktiles16 + gs.split - 1) / gs.split;
  const int nsplit = (int)((ktiles16 + per16 - 1) / per16);
  GemmTrailArgs a{};
  a.K = gs.K;
  a.kslice = per16 * 16;
  a.tm = (int)(gs.M / 128);
  a.tn = (int)(gs.N / 128);
  a.n_gemm = a.tm * a.tn * nsplit;
  a.A = gs.A;
  a.lda = gs.lda;
  a.B = gs.B;
  a.ldb = gs.ldb;
  a.C = gs.C;
  a.ldc = gs.ldc;
  a.slice_stride = gs.slice_stride;
  a.Ain = Ain;
  a.Aout = Aout;
  a.D = D;
  a.B2 = B2;
  a.g = g;
  a.check = check ? 1 : 0;
  a.pf = pf;
  a.st = st;
  a.pr = gs.ctl_pr;
  a.bc_table = gs.ctl_table;
  a.ticket = gs.ctl_ticket;
  if (a.ticket && (!a.pr || !a.bc_table)) throw std::invalid_argument("launch_gemm_trail: folded control needs pr, table");
  if (n_trail < 0) {
    if (D % 128 || B2 % 128) throw std::invalid_argument("launch_gemm_trail: D, B2 must be multiples of 128");
    Gemm2Args a2{a, (int)((D - B2) / 128), (B2 == 256 && trail_mid()) ? 1 : 0};
    const dim3 grid2((unsigned)(a.n_gemm + a2.tm2 * a2.tm2));
    if (a2.mid) check_mid_shape(B2, B2, (int64_t)a2.tm2 * a2.tm2, grid2.x - a.n_gemm, "launch_gemm_trail");
#define MIDAGMA_GT2(AM, BM) \
  hipLaunchKernelGGL((gemm_trail128_kernel<AM, BM>), grid2, dim3(NTHREADS), kGemmPipeLds, stream, a2)
    if (gs.a_trans && gs.bmode == B_PLAIN)
      MIDAGMA_GT2(1, B_PLAIN);
    else if (gs.a_trans)
      MIDAGMA_GT2(1, B_IMINUS);
    else if (gs.bmode == B_PLAIN)
      MIDAGMA_GT2(0, B_PLAIN);
    else
      MIDAGMA_GT2(0, B_IMINUS);
#undef MIDAGMA_GT2
    HIP_TRY(hipGetLastError());
    return;
  }
  const dim3 grid((unsigned)(a.n_gemm + n_trail));
#define MIDAGMA_GT(AM, BM) \
  hipLaunchKernelGGL((gemm_trail_kernel<AM, BM>), grid, dim3(NTHREADS), kGemmTrailLds, stream, a)
  if (gs.a_trans && gs.bmode == B_PLAIN)
    MIDAGMA_GT(1, B_PLAIN);
  else if (gs.a_trans)
    MIDAGMA_GT(1, B_IMINUS);
  else if (gs.bmode == B_PLAIN)
    MIDAGMA_GT(0, B_PLAIN);
  else
    MIDAGMA_GT(0, B_IMINUS);
#undef MIDAGMA_GT
  HIP_TRY(hipGetLastError());
}

// B2 = 256 (16 K-tiles) folds C0 in during the K loop (EPI_SUB_MID; D = 5120: 219 -> 203 us, D =
// 3072: 77.6 -> 68.9 us, tools/micro/trail_micro.hip), other B2 read it in the epilogue
static void launch_trail128_epi(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, bool check,
                                const State* st, hipStream_t stream, bool mid) {
  if (D % 128 || B2 % 128) throw std::invalid_argument("launch_trail128: D, B2 must be multiples of 128");
  const int tm = (int)((D - B2) / 128);
  if (tm <= 0) return;
  const int64_t G0 = g * B2;
  // A = Ain[:, G] (lda D), B = Aout[G, :] (the row panel), C = Aout, C0 = Ain; K = B2
  static const bool no_pipe = knob_set("MIDAGMA_EXP_NO_PIPE");  // experiment knob
  const dim3 grid((unsigned)(tm * tm));
  const int64_t chk = check ? 1 : 0, b0 = G0 / 128, nb = B2 / 128;
  if (!no_pipe && mid && B2 == 256) {
    check_mid_shape(B2, B2, (int64_t)tm * tm, grid.x, "launch_trail128");
    hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_MID>), grid, dim3(NTHREADS), kGemmPipeLds, stream, B2,
                       B2, tm, tm, Ain + G0, D, Aout + G0 * D, D, Aout, D, chk, const_cast<double*>(Ain), b0, nb, st);
  } else if (!no_pipe)
    hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_BAND>), grid, dim3(NTHREADS), kGemmPipeLds, stream, B2,
                       B2, tm, tm, Ain + G0, D, Aout + G0 * D, D, Aout, D, chk, const_cast<double*>(Ain), b0, nb, st);
  else
    hipLaunchKernelGGL((gemm128_kernel<false, B_PLAIN, EPI_SUB_BAND>), grid, dim3(NTHREADS), kGemm128Lds, stream, B2,
                       B2, tm, tm, Ain + G0, D, Aout + G0 * D, D, Aout, D, chk, const_cast<double*>(Ain), b0, nb, st);
  HIP_TRY(hipGetLastError());
}

void launch_trail128(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, bool check, const State* st,
                     hipStream_t stream) {
  launch_trail128_epi(Ain, Aout, D, B2, g, check, st, stream, trail_mid());
}

// ---- the trailing update with the next block's series in the same launch (large D) ---------
// At d = 5000 the 19 trailing updates of a slot (1444 tiles, 2.8 rounds, ~194 us each) are
// followed by block g + 1's series: a residual and two pass launches of 256 workgroups, each
// 6-7 us of mostly operand latency (0.4 ms a slot).  The series needs only block g + 1's
// diagonal, which the trailing update writes in four of its tiles; those run first, and the
// series runs on `workers` workgroups placed after the first round of tiles (they start as the
// first tiles finish, when the diagonal is ready), beside the rest of the update.
struct TrailSeriesArgs {
  const double* Ain;
  double* Aout;
  int64_t D;
  int g, check, tm, woff;
  int diag[4];                    // slots 0..3: block g + 1's diagonal tiles
  int exc_slot[4], exc_tile[4];   // the other slots whose tile is not xcd_remap's (-1: none)
  TrailSeries ts;
  State* st;
  // trail_panel_kernel only (np = 0 elsewhere)
  TrailPanel tp;
  int np, nband, nband_pad, nrest, njobs;
};

constexpr uint64_t TS_TIMEOUT = 5000000;  // device real-time ticks (100 MHz): 50 ms

// lane 0 polls the counter (relaxed agent loads) until it reaches `target` or the time runs out;
// then one agent acquire, its wait, and the barrier (MI355X_MICROARCH.md: Consumer, always)
__device__ __forceinline__ bool ts_wait(const int* ctr, int target, int* go) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 0;
    for (;;) {
      if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
        ok = 1;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > TS_TIMEOUT) break;
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *go = ok;
  }
  __syncthreads();
  return *go != 0;
}
// every wave's stores drained, the barrier, then lane 0: one counter add, behind an agent release
// when the handed-off bytes were plain stores (the diagonal tiles: the release writes back the XCD
// L2's dirty lines, the trailing tiles' too), without one when every handed-off byte was stored
// write-through (sc1: the series' Y, Q, P, row partials; MI355X_MICROARCH.md, "(2) without an
// agent release") -- a release per worker and phase flushed the L2s under the running update
__device__ __forceinline__ void ts_signal(int* ctr, bool release) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (release) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// a bounded wait ran out: the slot goes back to the host's pivoted path (every later launch of
// the slot is a no-op; P and *done of this series are not used), and sync[224] counts it
__device__ __forceinline__ void ts_abort(const TrailSeriesArgs& a) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(&a.st->status, (int32_t)ST_NEED_GJ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(a.ts.sync + 224, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// worker w of the series of block g + 1: tiles w, w + workers, ... of each phase (nm_tile's
// XCD placement holds: workers is a multiple of 8 and woff too)
__device__ void ts_worker(const TrailSeriesArgs& a, int w, double* smem) {
  const TrailSeries& s = a.ts;
  double* red = smem;
  float* red4 = reinterpret_cast<float*>(smem + 4 * 256);
  int* go = reinterpret_cast<int*>(smem + 4 * 256 + 4);
  const int64_t GN0 = (int64_t)(a.g + 1) * 256;
  if (!ts_wait(s.sync, 4, go)) return ts_abort(a);
  const double* S = a.Aout + GN0 * a.D + GN0;
  for (int wg = w; wg < 256; wg += s.workers) {
    __syncthreads();  // red is reused by consecutive tiles
    nm_resid_body<16, 4, false>(wg, S, a.D, SFromW{}, s.Pe, s.Po, s.Y[0], s.Q[0], s.part, s.done, a.st, s.xmap, red);
  }
  for (int p = 1; p <= s.passes; ++p) {
    ts_signal(s.sync + 32 * p, false);
    if (!ts_wait(s.sync + 32 * p, s.workers, go)) return ts_abort(a);
    for (int wg = w; wg < 256; wg += s.workers) {
      __syncthreads();
      nm_pass_body<16, 4>(wg, s.Y[(p - 1) & 1], s.Q[(p - 1) & 1], s.Y[p & 1], s.Q[p & 1], s.P,
                          s.part + (int64_t)(p - 1) * PART_STRIDE, s.part + (int64_t)p * PART_STRIDE, s.done, p,
                          a.st, s.xmap, red, red4);
    }
  }
  if (a.np > 0) ts_signal(s.sync + TS_FIN, false);  // P and done are in (write-through stores)
}

__global__ __launch_bounds__(NTHREADS, 2) void trail_series_kernel(TrailSeriesArgs a) {
  if (a.st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x, nw = a.ts.workers;
  if (b >= a.woff && b < a.woff + nw) {
    ts_worker(a, b - a.woff, smem);
    return;
  }
  const int s = b < a.woff ? b : b - nw, ntiles = a.tm * a.tm;
  int t = s < 4 ? a.diag[s] : xcd_remap(s, ntiles);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (s == a.exc_slot[k]) t = a.exc_tile[k];
  const int64_t G0 = (int64_t)a.g * 256;
  gemm_pipe_tile<0, B_PLAIN, EPI_SUB_MID>(t, 256, 256, a.tm, a.tm, a.Ain + G0, a.D, a.Aout + G0 * a.D, a.D, a.Aout,
                                          a.D, (int64_t)a.check, const_cast<double*>(a.Ain), G0 / 128, 2, a.st, smem);
  if (s < 4) ts_signal(a.ts.sync, true);  // block g + 1's diagonal tile is in Aout (plain stores)
}

// ---- ... and block g + 1's panel in the same launch (large D) -----------------------------------
// The panel launch of block g + 1 (≈35 us at D = 5120, its 2496 32 x 32 jobs latency-bound) needs
// block g + 1's P (the series above) and block g + 1's row and column bands of Aout (148 of the
// update's tiles); it writes those bands of Ain, which only the same 148 tiles read.  So the band
// tiles run first (the EPI_SUB_CROSS_MID tile body: block g + 1's bands), the rest after them (the
// EPI_SUB_MID body with both bands skipped), the series workers after the first round, and `np`
// panel workgroups at the end of the grid: dispatched as the update's last round frees slots,
// they wait for the band tiles and the series, then claim panel jobs from a counter.  Every job
// runs binv_panel_job's arithmetic, so W is bit-identical to the separate launches.
__device__ void tp_panel(const TrailSeriesArgs& a, double* smem) {
  double* img = smem;  // 4 images of NB x ST doubles, then the hand-off word
  int* go = reinterpret_cast<int*>(smem + 4 * NB * ST);
  int* sync = a.ts.sync;
  if (!ts_wait(sync + TS_BAND, a.nband, go)) return ts_abort(a);
  if (!ts_wait(sync + TS_FIN, a.ts.workers, go)) return ts_abort(a);
  if (__hip_atomic_load(&a.st->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ST_RUNNING) return;
  if (__hip_atomic_load(a.ts.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {  // (the panel launch's test)
    if (threadIdx.x == 0)
      __hip_atomic_store(&a.st->status, (int32_t)ST_NEED_GJ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  for (;;) {
    if (threadIdx.x == 0) *go = __hip_atomic_fetch_add(sync + TS_JOB, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int job = *go;
    __syncthreads();  // (go is rewritten next round)
    if (job >= a.njobs) return;
    binv_panel_job<0>(job, a.Aout, const_cast<double*>(a.Ain), a.D, 256, a.g + 1, a.ts.P, 256, a.tp.Ppe, a.tp.Ppo,
                      a.tp.pcheck, a.st, a.tp.pf, nullptr, nullptr, img, img + NB * ST, img + 2 * NB * ST,
                      img + 3 * NB * ST);
    __syncthreads();  // the images are reused by the next job
  }
}

__device__ __forceinline__ void zero_sync2(int* z) {
  if (threadIdx.x < 8) {
    const int w = threadIdx.x <= NM_PASSES ? 32 * threadIdx.x
                                           : (threadIdx.x == 5 ? TS_FIN : threadIdx.x == 6 ? TS_BAND : TS_JOB);
    __hip_atomic_store(z + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(NTHREADS, 2) void trail_panel_kernel(TrailSeriesArgs a) {
  if (a.st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x, nw = a.ts.workers;
  if (b == 0 && a.tp.zsync2) zero_sync2(a.tp.zsync2);  // block g + 2's words, for the next launch
  if (b >= a.woff && b < a.woff + nw) {
    ts_worker(a, b - a.woff, smem);
    return;
  }
  const int s = b < a.woff ? b : b - nw;
  if (s >= a.nband_pad + a.nrest) return tp_panel(a, smem);
  const int64_t G0 = (int64_t)a.g * 256;
  const int b0 = 2 * a.g;
  if (s < a.nband) {
    gemm_pipe_tile<0, B_PLAIN, EPI_SUB_CROSS_MID>(s, 256, 256, a.tm, 4, a.Ain + G0, a.D, a.Aout + G0 * a.D, a.D,
                                                  a.Aout, a.D, (int64_t)a.check, const_cast<double*>(a.Ain), b0, 2,
                                                  a.st, smem);
    // (the tile decode: s < 2 tm are block g + 1's rows, columns s % tm; b0, b0 + 1 is its diagonal)
    const bool diag = s < 2 * a.tm && (s % a.tm == b0 || s % a.tm == b0 + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {  // plain stores: one agent release, then the counters
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (diag) __hip_atomic_fetch_add(a.ts.sync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a.ts.sync + TS_BAND, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (s >= a.nband_pad) {
    // the rest: the grid without the pivot band and block g + 1's (4 tile rows and columns from b0)
    const int r = s - a.nband_pad;
    gemm_pipe_tile<0, B_PLAIN, EPI_SUB_MID>(xcd_remap(r, a.nrest), 256, 256, a.tm - 2, a.tm - 2, a.Ain + G0, a.D,
                                            a.Aout + G0 * a.D, a.D, a.Aout, a.D, (int64_t)a.check,
                                            const_cast<double*>(a.Ain), b0, 4, a.st, smem);
  }
}

size_t trail_panel_lds() { return std::max(kGemmPipeLds, (size_t)(4 * NB * ST) * sizeof(double) + 16); }

void launch_trail128_panel(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, State* st,
                           const TrailSeries& ts, const TrailPanel& tp, hipStream_t stream) {
  if (D % 128) throw std::invalid_argument("launch_trail128_panel: D must be a multiple of 128");
  const int tm = (int)((D - 256) / 128), K2 = (int)(D / 256);
  if (g + 1 >= K2 || tm < 8 || ts.workers <= 0 || ts.workers % 8 || ts.passes < 1 || ts.passes > NM_PASSES ||
      tp.workers < 0)
    throw std::invalid_argument("launch_trail128_panel: needs a next block, workers a multiple of 8, 1..4 passes");
  const int nband = 2 * (2 * tm - 2), nrest = (tm - 2) * (tm - 2);
  check_mid_shape(256, 256, (int64_t)tm * 4, nband, "launch_trail128_panel");
  check_mid_shape(256, 256, (int64_t)nrest, nrest, "launch_trail128_panel");
  TrailSeriesArgs a{};
  a.Ain = Ain;
  a.Aout = Aout;
  a.D = D;
  a.g = (int)g;
  a.check = check ? 1 : 0;
  a.tm = tm;
  for (int k = 0; k < 4; ++k) a.diag[k] = a.exc_slot[k] = a.exc_tile[k] = -1;
  a.ts = ts;
  a.st = st;
  a.tp = tp;
  a.np = tp.workers;
  a.nband = nband;
  a.nband_pad = (nband + 7) & ~7;  // the rest starts on an XCD boundary (xcd_remap)
  a.nrest = nrest;
  const int gb = 256 / NB, mb = (int)(D / NB) - gb;
  a.njobs = 2 * gb * mb + gb * gb;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int ntiles = a.nband_pad + nrest;
  a.woff = std::min(ntiles, 2 * cus) & ~7;  // the series workers after the first round of tiles
  static bool attr = false;
  if (!attr) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(trail_panel_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)trail_panel_lds()));
    attr = true;
  }
  hipLaunchKernelGGL(trail_panel_kernel, dim3((unsigned)(ntiles + ts.workers + tp.workers)), dim3(NTHREADS),
                     trail_panel_lds(), stream, a);
  HIP_TRY(hipGetLastError());
}

// linear index of tile (bm, bn) (pivot band skipped) in gemm_pipe_tile's order for tm x tm tiles
static int pipe_tile_index(int bm, int bn, int tm) {
  if (tm > 8) {
    const int fm = (bm / 8) * 8, rows = tm - fm < 8 ? tm - fm : 8;
    return fm * tm + bn * rows + (bm - fm);
  }
  return bm * tm + bn;
}
static int host_xcd_remap(int w, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = w % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
}

void launch_trail128_series(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, State* st,
                            const TrailSeries& ts, hipStream_t stream) {
  if (D % 128) throw std::invalid_argument("launch_trail128_series: D must be a multiple of 128");
  const int tm = (int)((D - 256) / 128), K2 = (int)(D / 256);
  if (g + 1 >= K2 || tm < 4 || ts.workers <= 0 || ts.workers % 8 || ts.passes < 1 || ts.passes > NM_PASSES)
    throw std::invalid_argument("launch_trail128_series: needs a next block, workers a multiple of 8, 1..4 passes");
  check_mid_shape(256, 256, (int64_t)tm * tm, (int64_t)tm * tm, "launch_trail128_series");
  const int ntiles = tm * tm;
  TrailSeriesArgs a{};
  a.Ain = Ain;
  a.Aout = Aout;
  a.D = D;
  a.g = (int)g;
  a.check = check ? 1 : 0;
  a.tm = tm;
  // block g + 1 sits right after the skipped pivot band: tiles 2g, 2g + 1 in both dimensions
  const int b0 = 2 * (int)g;
  std::vector<int> perm(ntiles);
  for (int s = 0; s < ntiles; ++s) perm[s] = host_xcd_remap(s, ntiles);
  for (int k = 0; k < 4; ++k) {
    a.diag[k] = pipe_tile_index(b0 + k / 2, b0 + k % 2, tm);
    const int j = (int)(std::find(perm.begin() + k, perm.end(), a.diag[k]) - perm.begin());
    std::swap(perm[k], perm[j]);
  }
  int ne = 0;
  for (int k = 0; k < 4; ++k) a.exc_slot[k] = a.exc_tile[k] = -1;
  for (int s = 4; s < ntiles; ++s)
    if (perm[s] != host_xcd_remap(s, ntiles)) {
      if (ne == 4) throw std::logic_error("launch_trail128_series: tile permutation");
      a.exc_slot[ne] = s;
      a.exc_tile[ne++] = perm[s];
    }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  // the workers' place in the grid: after the first round of tiles (2 workgroups per CU; they start
  // as the first tiles finish), or (experiment knob MIDAGMA_EXP_TS_WOFF=0) after all tiles, in
  // the slots the last round leaves idle
  const int woff = (knob("MIDAGMA_EXP_TS_WOFF", 1) != 0 ? std::min(ntiles, 2 * cus) : ntiles) & ~7;
  a.woff = woff;
  a.ts = ts;
  a.st = st;
  hipLaunchKernelGGL(trail_series_kernel, dim3((unsigned)(ntiles + ts.workers)), dim3(NTHREADS), kGemmPipeLds, stream,
                     a);
  HIP_TRY(hipGetLastError());
}

#ifdef MIDAGMA_EXPERIMENTS
#include "../../experiments/gemm_exp.inc"
#endif

// The trailing update of outer step g in two parts (the cov-mode look-ahead, blockinv.hip):
// part 0 the tiles in the row / column band of block g + 1 (what its series and panel read),
// part 1 the rest (both bands skipped).  The same tile bodies as launch_trail128.
void launch_trail128_split(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, int part,
                           const State* st, hipStream_t stream) {
  if (D % 128 || B2 % 128 || (g + 2) * B2 > D) throw std::invalid_argument("launch_trail128_split: shape");
  const int tm = (int)((D - B2) / 128), nb = (int)(B2 / 128);
  const int64_t G0 = g * B2;
  const bool mid = B2 == 256 && trail_mid();  // the tile bodies of launch_trail128 (bit-identical)
  if (part == 0) {
    const int n = nb * (2 * tm - nb);
    // (tiles_n = 2 nb: tiles_m tiles_n >= n, so every tile is in K slice 0)
    if (mid) check_mid_shape(B2, B2, (int64_t)tm * 2 * nb, n, "launch_trail128_split");
    if (mid)
      hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_CROSS_MID>), dim3((unsigned)n), dim3(NTHREADS),
                         kGemmPipeLds, stream, B2, B2, tm, 2 * nb, Ain + G0, D, Aout + G0 * D, D, Aout, D, (int64_t)0,
                         const_cast<double*>(Ain), (int64_t)(G0 / 128), (int64_t)nb, st);
    else
      hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_CROSS>), dim3((unsigned)n), dim3(NTHREADS), kGemmPipeLds,
                         stream, B2, B2, tm, 2 * nb, Ain + G0, D, Aout + G0 * D, D, Aout, D, (int64_t)0,
                         const_cast<double*>(Ain), (int64_t)(G0 / 128), (int64_t)nb, st);
  } else {
    const int tr = tm - nb;
    if (tr <= 0) return;
    if (mid) check_mid_shape(B2, B2, (int64_t)tr * tr, (int64_t)tr * tr, "launch_trail128_split");
    if (mid)
      hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_MID>), dim3((unsigned)(tr * tr)), dim3(NTHREADS),
                         kGemmPipeLds, stream, B2, B2, tr, tr, Ain + G0, D, Aout + G0 * D, D, Aout, D, (int64_t)0,
                         const_cast<double*>(Ain), (int64_t)(G0 / 128), (int64_t)(2 * nb), st);
    else
      hipLaunchKernelGGL((gemm_pipe_kernel<0, B_PLAIN, EPI_SUB_BAND>), dim3((unsigned)(tr * tr)), dim3(NTHREADS),
                         kGemmPipeLds, stream, B2, B2, tr, tr, Ain + G0, D, Aout + G0 * D, D, Aout, D, (int64_t)0,
                         const_cast<double*>(Ain), (int64_t)(G0 / 128), (int64_t)(2 * nb), st);
  }
  HIP_TRY(hipGetLastError());
}

// dst[c][r] = src[r][c] for r < rows, c < cols (64 x 64 tiles through LDS)
__global__ __launch_bounds__(NTHREADS) void transpose_kernel(const double* __restrict__ src, int64_t ld_src,
                                                             int64_t rows, int64_t cols, double* __restrict__ dst,
                                                             int64_t ld_dst) {
  __shared__ double t[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[r * ld_src + c] : 0.0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[c * ld_dst + r] = t[tx][i];
  }
}

void launch_transpose(const double* src, int64_t ld_src, int64_t rows, int64_t cols, double* dst, int64_t ld_dst,
                      hipStream_t stream) {
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((rows + 63) / 64), (unsigned)((cols + 63) / 64)),
                     dim3(NTHREADS), 0, stream, src, ld_src, rows, cols, dst, ld_dst);
  HIP_TRY(hipGetLastError());
}

__global__ __launch_bounds__(NTHREADS) void sum_slices_kernel(const double* __restrict__ parts, int split,
                                                              int64_t stride, int64_t count,
                                                              double* __restrict__ out,
                                                              const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < count; i += (int64_t)gridDim.x * NTHREADS) {
    double acc = parts[i];
    for (int z = 1; z < split; ++z) acc += parts[z * stride + i];
    out[i] = acc;
  }
}

__global__ __launch_bounds__(NTHREADS) void sum_vector_kernel(const double* __restrict__ v, int64_t n,
                                                              double* __restrict__ out,
                                                              const State* __restrict__ st) {
  // (with a State: the logistic loss partials, which the sigmoid GEMM writes and the controller
  // reads on checkpoint slots only)
  if (st && (st->status != ST_RUNNING || !st->ckpt_pending)) return;
  __shared__ double red[NTHREADS];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += NTHREADS) acc += v[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

void launch_sum_slices(const double* parts, int split, int64_t stride, int64_t count, double* out,
                       const State* st, hipStream_t stream) {
  int64_t blocks = (count + NTHREADS - 1) / NTHREADS;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sum_slices_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, parts, split, stride,
                     count, out, st);
  HIP_TRY(hipGetLastError());
}

void launch_sum_vector(const double* v, int64_t n, double* out, const State* st, hipStream_t stream) {
  hipLaunchKernelGGL(sum_vector_kernel, dim3(1), dim3(NTHREADS), 0, stream, v, n, out, st);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
