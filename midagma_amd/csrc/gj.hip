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
// Block step k (64-wide block column, K = D/64 steps):
//   panel  : P = inv(A_kk) (unpivoted GJ in registers + LDS, pivots -> log|p|),
//            R_kj = P A_kj (MFMA) for j != k, column panel C_ik = A_ik copied out
//   update : A_ij -= C_i R_j (i,j != k);  A_kj = R_j;  A_ik = -C_i P;  A_kk = P
// so every launch writes only its own tile of A (side buffers carry panels).
#include "launch.h"
#include "mfma64.h"

namespace midagma {

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

__global__ __launch_bounds__(NTHREADS) void gj_panel_kernel(const double* __restrict__ A, int64_t D, int k,
                                                            double* __restrict__ Pbuf, double* __restrict__ Rbuf,
                                                            double* __restrict__ Cbuf, double* __restrict__ pivlog,
                                                            const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Ps = smem;               // [64][SA]  P as left operand
  double* Ts = Ps + 64 * SA;       // [64][SB]  A_kj as right operand
  double* rowbuf = Ts + 64 * SB;   // [2][64]   pivot row (double-buffered by step parity)
  double* colbuf = rowbuf + 128;   // [2][64]   pivot column
  const int tid = threadIdx.x, j = blockIdx.x;
  const int r = tid >> 2, cg = tid & 3, c0 = cg * 16;
  const double* Akk = A + (int64_t)k * 64 * D + (int64_t)k * 64;

  // This thread owns A_kk[r][c0 .. c0+15] in registers.
  double a[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const double2 v = *reinterpret_cast<const double2*>(Akk + (int64_t)r * D + c0 + 2 * e);
    a[2 * e] = v.x;
    a[2 * e + 1] = v.y;
  }

  for (int pb = 0; pb < 64; pb += 16) {
#pragma unroll
    for (int pp = 0; pp < 16; ++pp) {
      const int p = pb + pp;
      const int par = p & 1;
      if (r == p) {
#pragma unroll
        for (int e = 0; e < 16; ++e) rowbuf[par * 64 + c0 + e] = a[e];
      }
      if (cg == (pb >> 4)) colbuf[par * 64 + r] = a[pp];
      __syncthreads();
      const double piv = rowbuf[par * 64 + p];
      const double inv = 1.0 / piv;
      const double arp = colbuf[par * 64 + r];
      const double neg_arp_inv = -arp * inv;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = c0 + e;
        const double rpc = rowbuf[par * 64 + c] * inv;
        if (r == p)
          a[e] = (c == p) ? inv : rpc;
        else
          a[e] = (c == p) ? neg_arp_inv : __builtin_fma(-arp, rpc, a[e]);
      }
      if (pivlog && j == 0 && tid == 0) pivlog[(int64_t)k * 64 + p] = log(fabs(piv));
    }
  }

  if (j == k) {
#pragma unroll
    for (int e = 0; e < 16; ++e) Pbuf[r * 64 + c0 + e] = a[e];
    return;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) Ps[r * SA + c0 + e] = a[e];
  tile_to_lds<SB>(Ts, A + (int64_t)k * 64 * D + (int64_t)j * 64, D, Ident());
  __syncthreads();
  Quad q;
  q.zero();
  quad_mma<false>(Ps, Ts, q);
  double* Rj = Rbuf + (int64_t)j * 64;
  quad_foreach(q, [&](int row, int col, double& v) { Rj[(int64_t)row * D + col] = v; });
  // column panel tile (j, k) -> Cbuf rows j*64.., leading dim 64
  const double* Ajk = A + (int64_t)j * 64 * D + (int64_t)k * 64;
  double* Cj = Cbuf + (int64_t)j * 64 * 64;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int item = it * NTHREADS + tid;
    const int row = item >> 5, c = (item & 31) * 2;
    *reinterpret_cast<double2*>(Cj + row * 64 + c) = *reinterpret_cast<const double2*>(Ajk + (int64_t)row * D + c);
  }
}

__global__ __launch_bounds__(NTHREADS) void gj_update_kernel(double* __restrict__ A, int64_t D, int k,
                                                             const double* __restrict__ Pbuf,
                                                             const double* __restrict__ Rbuf,
                                                             const double* __restrict__ Cbuf,
                                                             const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int bi = blockIdx.y, bj = blockIdx.x, tid = threadIdx.x;
  double* Aij = A + (int64_t)bi * 64 * D + (int64_t)bj * 64;
  if (bi == k) {
    const double* src = (bj == k) ? Pbuf : Rbuf + (int64_t)bj * 64;
    const int64_t lds = (bj == k) ? 64 : D;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int item = it * NTHREADS + tid;
      const int row = item >> 5, c = (item & 31) * 2;
      *reinterpret_cast<double2*>(Aij + (int64_t)row * D + c) =
          *reinterpret_cast<const double2*>(src + row * lds + c);
    }
    return;
  }
  double* Ls = smem;            // [64][SA]  -C_i
  double* Rs = Ls + 64 * SA;    // [64][SB]  R_j or P
  tile_to_lds<SA>(Ls, Cbuf + (int64_t)bi * 64 * 64, 64, Negate());
  Quad q;
  if (bj == k) {
    tile_to_lds<SB>(Rs, Pbuf, 64, Ident());
    q.zero();
  } else {
    tile_to_lds<SB>(Rs, Rbuf + (int64_t)bj * 64, D, Ident());
    quad_foreach(q, [&](int row, int col, double& v) { v = Aij[(int64_t)row * D + col]; });
  }
  __syncthreads();
  quad_mma<false>(Ls, Rs, q);
  quad_foreach(q, [&](int row, int col, double& v) { Aij[(int64_t)row * D + col] = v; });
}

constexpr size_t kPanelLds = (64 * SA + 64 * SB + 256) * sizeof(double);
constexpr size_t kUpdateLds = (64 * SA + 64 * SB) * sizeof(double);

void gj_setup_attributes() {
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gj_panel_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPanelLds));
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(gj_update_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kUpdateLds));
}

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
  const int K = (int)(D / 64);
  for (int k = 0; k < K; ++k) {
    hipLaunchKernelGGL(gj_panel_kernel, dim3(K), dim3(NTHREADS), kPanelLds, stream, A, D, k, w.P, w.R, w.C,
                       w.pivlog, st);
    hipLaunchKernelGGL(gj_update_kernel, dim3(K, K), dim3(NTHREADS), kUpdateLds, stream, A, D, k, w.P, w.R, w.C,
                       st);
  }
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
