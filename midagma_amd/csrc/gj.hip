// Blocked Gauss-Jordan inverse + log-det of sI - W∘W on FP64 matrix cores.
//
// Replaces `sla.inv(s*I - W*W)` (LAPACK dgetrf+dgetri, linear.py:226, 240),
// `la.slogdet` (linear.py:114) and torch `slogdet` (nonlinear.py:85).
//
// In the M-matrix domain sI - W∘W is a nonsingular M-matrix, so elimination
// WITHOUT pivoting is stable and every pivot is > 0.
// The kernels run on A^T so the result is inv(A)^T = M^T, exactly the operand
// of the gradient 2 W∘M^T (linear.py:248), read coalesced by the fused update.
//
// Block Gauss-Jordan with NB = 32 (K = D/32 block steps), ONE launch per step.
// Step k reads three side panels published by step k-1 (double-buffered by
// parity): P = inv(A_kk), the column tiles C_i = A_ik and the row tiles
// R_j = A_kj, and updates every tile of A in place:
//     A_ij -= C_i (P R_j)      A_kj = P R_j      A_ik = -C_i P      A_kk = P
// Tiles landing in block column/row k+1 are also published as the next step's
// panels, and the workgroup owning tile (k+1, k+1) inverts it right away
// (unpivoted GJ in registers + LDS, pivots -> log|p|), so the only serial
// chain per step is one 32x32 inversion plus one kernel boundary.
#include "launch.h"
#include "mfma64.h"

namespace midagma {

constexpr int NB = 32;        // block size of the elimination
constexpr int SA32 = 34;      // [m][k] LDS image stride for 32-wide tiles (= 2 mod 32)
constexpr int SB32 = 48;      // [k][n] LDS image stride (= 16 mod 32)
constexpr int EPT = NB * NB / NTHREADS;   // elements per thread in the tile inversion (4)
constexpr int TPR = NB / EPT;             // threads per tile row (8)

// A^T tile builder: At[J][I] = (I == J ? s : 0) - f(X[I][J]) on the logical
// d x d block (f = square for W, identity for a given A), identity padding.
template <bool SQUARE>
__global__ __launch_bounds__(NTHREADS) void build_at_kernel(const double* __restrict__ X, int64_t ldx,
                                                            double* __restrict__ At, int64_t D, int64_t d,
                                                            double s_arg, const Params* __restrict__ pr,
                                                            const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  // s comes from device Params when given: graph replays must see each call's s
  const double s = pr ? pr->s : s_arg;
  __shared__ double tile[64][65];
  const int bi = blockIdx.y, bj = blockIdx.x;  // source tile (rows bi, cols bj)
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = it * NTHREADS + tid;
    const int r = e >> 6, c = e & 63;
    const int64_t I = (int64_t)bi * 64 + r, J = (int64_t)bj * 64 + c;
    double v;
    if (I < d && J < d) {
      const double x = X[I * ldx + J];
      const double f = SQUARE ? x * x : x;
      v = (I == J ? s : 0.0) - f;
    } else {
      v = (I == J) ? 1.0 : 0.0;
    }
    tile[c][r] = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = it * NTHREADS + tid;
    const int r = e >> 6, c = e & 63;  // r: row of At tile (= source col)
    At[((int64_t)bj * 64 + r) * D + (int64_t)bi * 64 + c] = tile[r][c];
  }
}

// ---- 32 x 32 tile helpers --------------------------------------------------------
// Wave w owns the 16 x 16 quadrant (wm, wn) = (w >> 1, w & 1) of a 32 x 32 output.
__device__ __forceinline__ int q_m0() { return (threadIdx.x >> 7) * 16; }
__device__ __forceinline__ int q_n0() { return ((threadIdx.x >> 6) & 1) * 16; }

// acc += Ls(32 x 32, [m][k] stride SA32) * Rs(32 x 32, [k][n] stride SB32)
__device__ __forceinline__ void mma32(const double* __restrict__ Ls, const double* __restrict__ Rs, dbl4& acc) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const int m0 = q_m0(), n0 = q_n0();
#pragma unroll
  for (int k0 = 0; k0 < NB; k0 += 4) {
    const double a = Ls[(m0 + r) * SA32 + k0 + kq];
    const double b = Rs[(k0 + kq) * SB32 + n0 + r];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
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

// 32 x 32 global tile (leading dim ld) -> LDS image with stride S, scaled by `sc`
template <int S>
__device__ __forceinline__ void tile32_to_lds(double* __restrict__ dst, const double* __restrict__ src, int64_t ld,
                                              double sc) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int item = it * NTHREADS + threadIdx.x;  // 512 double2 items
    const int row = item >> 4, c = (item & 15) * 2;
    double2 v = *reinterpret_cast<const double2*>(src + row * ld + c);
    v.x *= sc;
    v.y *= sc;
    *reinterpret_cast<double2*>(dst + row * S + c) = v;
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

// Reciprocal to ~1 ulp: hardware seed + two Newton steps (no IEEE division chain).
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

// In-place unpivoted GJ inverse of the 32 x 32 tile held in `img` (row stride SA32)
// by the whole workgroup; writes the inverse to Pout (ld NB) and log|pivot| to plog.
// `scratch` needs 4*NB doubles.  Ends with a barrier.
__device__ void invert_tile32(double* __restrict__ img, double* __restrict__ Pout, double* __restrict__ plog,
                              double* __restrict__ scratch) {
  const int tid = threadIdx.x;
  const int r = tid / TPR, c0 = (tid % TPR) * EPT;
  double* rowbuf = scratch;           // [2][NB]
  double* colbuf = scratch + 2 * NB;  // [2][NB]
  double a[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) a[e] = img[r * SA32 + c0 + e];
  double pivs = 0.0;  // lane p of wave 0 keeps pivot p (p < 32)
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
      __syncthreads();
      const double piv = rowbuf[par * NB + p];
      const double inv = fast_rcp(piv);
      const double arp = colbuf[par * NB + r];
      const double neg_arp_inv = -arp * inv;
      if (tid == p) pivs = piv;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int c = c0 + e;
        const double rpc = rowbuf[par * NB + c] * inv;
        if (r == p)
          a[e] = (c == p) ? inv : rpc;
        else
          a[e] = (c == p) ? neg_arp_inv : __builtin_fma(-arp, rpc, a[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) Pout[r * NB + c0 + e] = a[e];
  if (plog && tid < NB) plog[tid] = log(fabs(pivs));
  __syncthreads();
}

// Warm-started Newton-Schulz inverse of the 32 x 32 tile S (LDS image Sl, [m][k] stride SA32):
//   X <- X + X (I - S X), starting from X0 = the same block's inverse one Adam step earlier
//   (W moves by ~lr per step, so ||I - S X0|| is ~1e-3).  ||R_new|| <= ||R||^2, so once
//   32 max|R_ij| (>= ||R||_inf) <= 1e-8 the update lands at residual <= 1e-16 and we stop.
// Returns false (caller falls back to Gauss-Jordan) if the start is too far or does not
// converge in 4 updates.  On success the inverse is in `x` (accumulator layout).
// LDS: Xl [m][k] (SA32), Xr / Rr [k][n] (SB32), red[4].  All threads must call it.
__device__ bool ns_invert_tile32(const double* __restrict__ Sl, const double* __restrict__ X0, double* Xl,
                                 double* Xr, double* Rr, double* red, dbl4& x) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  acc_foreach(x, [&](int row, int col, double& v) {
    v = X0[row * NB + col];
    Xl[row * SA32 + col] = v;
    Xr[row * SB32 + col] = v;
  });
  __syncthreads();
  for (int it = 0; it < 5; ++it) {
    dbl4 sx = {0.0, 0.0, 0.0, 0.0};
    mma32(Sl, Xr, sx);
    double amax = 0.0;
    acc_foreach(sx, [&](int row, int col, double& v) {
      v = (row == col ? 1.0 : 0.0) - v;  // R = I - S X
      amax = fmax(amax, fabs(v)) + (isfinite(v) ? 0.0 : 1e300);
      Rr[row * SB32 + col] = v;
    });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmax(amax, __shfl_xor(amax, off));
    if (lane == 0) red[w] = amax;
    __syncthreads();  // Rr complete, red complete
    const double rho = 32.0 * fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    if (!(rho <= 0.25)) return false;  // too far from the warm start (or NaN)
    dbl4 xr = {0.0, 0.0, 0.0, 0.0};
    mma32(Xl, Rr, xr);
    __syncthreads();  // all reads of Xl / Xr / Rr / red done
#pragma unroll
    for (int t = 0; t < 4; ++t) x[t] = x[t] + xr[t];
    if (rho <= 1e-8) return true;
    if (it == 4) return false;
    acc_foreach(x, [&](int row, int col, double& v) {
      Xl[row * SA32 + col] = v;
      Xr[row * SB32 + col] = v;
    });
    __syncthreads();
  }
  return false;
}

// Invert the 32 x 32 tile `acc` (accumulator layout) into Pn (+ Pstore), Gauss-Jordan when
// pivots are wanted or no warm start exists, else warm-started Newton-Schulz.
__device__ void invert_diag_tile(dbl4& acc, double* __restrict__ Pn, double* __restrict__ Pstore,
                                 double* __restrict__ plog, bool want_gj, double* L0, double* L1, double* R0,
                                 double* T0, double* scratch) {
  __syncthreads();  // operand images of the caller are free
  acc_foreach(acc, [&](int row, int col, double& v) { L0[row * SA32 + col] = v; });
  __syncthreads();
  if (!want_gj) {
    dbl4 x;
    if (ns_invert_tile32(L0, Pstore, L1, R0, T0, scratch, x)) {
      acc_foreach(x, [&](int row, int col, double& v) {
        Pn[row * NB + col] = v;
        Pstore[row * NB + col] = v;
      });
      return;
    }
    __syncthreads();
  }
  invert_tile32(L0, Pn, plog, scratch);
  if (Pstore) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < NB * NB / NTHREADS; ++it) {
      const int e = it * NTHREADS + tid;
      Pstore[e] = Pn[e];
    }
  }
}

// Prologue: publish step 0's panels and invert A_00.
__global__ __launch_bounds__(NTHREADS) void gj_prologue_kernel(const double* __restrict__ A, int64_t D,
                                                               double* __restrict__ Cside,
                                                               double* __restrict__ Rside,
                                                               double* __restrict__ Pside,
                                                               double* __restrict__ pivlog,
                                                               double* __restrict__ Pstore,
                                                               const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  __shared__ __attribute__((aligned(16))) double L0[NB * SA32];
  __shared__ __attribute__((aligned(16))) double L1[NB * SA32];
  __shared__ __attribute__((aligned(16))) double R0[NB * SB32];
  __shared__ __attribute__((aligned(16))) double T0[NB * SB32];
  __shared__ double scratch[4 * NB];
  const int t = blockIdx.x;
  tile32_copy(Cside + (int64_t)t * NB * NB, NB, A + (int64_t)t * NB * D, D);  // column 0
  tile32_copy(Rside + (int64_t)t * NB, D, A + (int64_t)t * NB, D);            // row 0
  if (t != 0) return;
  dbl4 acc;
  acc_foreach(acc, [&](int row, int col, double& v) { v = A[(int64_t)row * D + col]; });
  const bool want_gj = st == nullptr || Pstore == nullptr || st->ckpt_pending || !st->warm_valid;
  invert_diag_tile(acc, Pside, Pstore, pivlog, want_gj, L0, L1, R0, T0, scratch);
}

// One block step of the elimination (see file header).
//   side buffers: Cside[2] (D x NB), Rside[2] (NB x D), Pside[2] (NB x NB), parity k & 1 read.
//   Every operand is requested from memory at kernel entry, so each step pays one
//   global-load latency before its MFMA chain.
__global__ __launch_bounds__(NTHREADS) void gj_step_kernel(double* __restrict__ A, int64_t D, int k,
                                                           double* __restrict__ Cside0, double* __restrict__ Cside1,
                                                           double* __restrict__ Rside0, double* __restrict__ Rside1,
                                                           double* __restrict__ Pside0, double* __restrict__ Pside1,
                                                           double* __restrict__ pivlog, double* __restrict__ Pstore,
                                                           const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  __shared__ __attribute__((aligned(16))) double L0[NB * SA32];   // P   ([m][k])
  __shared__ __attribute__((aligned(16))) double L1[NB * SA32];   // -C_i ([m][k])
  __shared__ __attribute__((aligned(16))) double R0[NB * SB32];   // R_j or P ([k][n])
  __shared__ __attribute__((aligned(16))) double T0[NB * SB32];   // P R_j ([k][n])
  __shared__ double scratch[4 * NB];
  const int bi = blockIdx.y, bj = blockIdx.x;
  const int K = (int)(D / NB);
  const bool odd = k & 1;
  const double* Cs = odd ? Cside1 : Cside0;
  const double* Rs = odd ? Rside1 : Rside0;
  const double* P = odd ? Pside1 : Pside0;
  double* Cn = odd ? Cside0 : Cside1;
  double* Rn = odd ? Rside0 : Rside1;
  double* Pn = odd ? Pside0 : Pside1;
  double* Aij = A + (int64_t)bi * NB * D + (int64_t)bj * NB;

  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  if (bi == k && bj == k) {
    acc_foreach(acc, [&](int row, int col, double& v) { v = P[row * NB + col]; });  // A_kk = P
  } else if (bi == k) {
    tile32_to_lds<SA32>(L0, P, NB, 1.0);  // A_kj = P R_j
    tile32_to_lds<SB32>(R0, Rs + (int64_t)bj * NB, D, 1.0);
    __syncthreads();
    mma32(L0, R0, acc);
  } else if (bj == k) {
    tile32_to_lds<SA32>(L1, Cs + (int64_t)bi * NB * NB, NB, -1.0);  // A_ik = -C_i P
    tile32_to_lds<SB32>(R0, P, NB, 1.0);
    __syncthreads();
    mma32(L1, R0, acc);
  } else {
    // T = P R_j ; A_ij += (-C_i) T        (all four operands requested up front)
    tile32_to_lds<SA32>(L0, P, NB, 1.0);
    tile32_to_lds<SB32>(R0, Rs + (int64_t)bj * NB, D, 1.0);
    tile32_to_lds<SA32>(L1, Cs + (int64_t)bi * NB * NB, NB, -1.0);
    dbl4 a_old;
    acc_foreach(a_old, [&](int row, int col, double& v) { v = Aij[(int64_t)row * D + col]; });
    __syncthreads();
    dbl4 tq = {0.0, 0.0, 0.0, 0.0};
    mma32(L0, R0, tq);
    acc_foreach(tq, [&](int row, int col, double& v) { T0[row * SB32 + col] = v; });
    __syncthreads();
    acc = a_old;
    mma32(L1, T0, acc);
  }
  acc_foreach(acc, [&](int row, int col, double& v) { Aij[(int64_t)row * D + col] = v; });
  if (k + 1 >= K) return;
  const int k1 = k + 1;
  if (bj == k1) acc_foreach(acc, [&](int row, int col, double& v) { Cn[((int64_t)bi * NB + row) * NB + col] = v; });
  if (bi == k1) acc_foreach(acc, [&](int row, int col, double& v) { Rn[(int64_t)row * D + (int64_t)bj * NB + col] = v; });
  if (bi == k1 && bj == k1) {
    const bool want_gj = st == nullptr || Pstore == nullptr || st->ckpt_pending || !st->warm_valid;
    invert_diag_tile(acc, Pn, Pstore ? Pstore + (int64_t)k1 * NB * NB : nullptr,
                     pivlog ? pivlog + (int64_t)k1 * NB : nullptr, want_gj, L0, L1, R0, T0, scratch);
  }
}

void gj_setup_attributes() {}

void launch_build_at(const double* X, int64_t ldx, bool square, double* At, int64_t D, int64_t d, double s,
                     const Params* pr, const State* st, hipStream_t stream) {
  const int K = (int)(D / 64);
  dim3 grid(K, K);
  if (square)
    hipLaunchKernelGGL(build_at_kernel<true>, grid, dim3(NTHREADS), 0, stream, X, ldx, At, D, d, s, pr, st);
  else
    hipLaunchKernelGGL(build_at_kernel<false>, grid, dim3(NTHREADS), 0, stream, X, ldx, At, D, d, s, pr, st);
  HIP_TRY(hipGetLastError());
}

void launch_gj_inverse(double* A, int64_t D, const GJWork& w, const State* st, hipStream_t stream) {
  const int K = (int)(D / NB);
  double* C0 = w.C;
  double* C1 = w.C + D * NB;
  double* R0 = w.R;
  double* R1 = w.R + NB * D;
  double* P0 = w.P;
  double* P1 = w.P + NB * NB;
  hipLaunchKernelGGL(gj_prologue_kernel, dim3(K), dim3(NTHREADS), 0, stream, A, D, C0, R0, P0, w.pivlog, w.Pstore,
                     st);
  for (int k = 0; k < K; ++k)
    hipLaunchKernelGGL(gj_step_kernel, dim3(K, K), dim3(NTHREADS), 0, stream, A, D, k, C0, C1, R0, R1, P0, P1,
                       w.pivlog, w.Pstore, st);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
