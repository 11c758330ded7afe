// TCC trek regularizer on the GPU (fbleile/midagma src/notreks/notreks.py:
// trek_cycle_coupling_value_gradW as trek_value_grad calls it inside the loop, i.e. with its
// defaults: spectral penalty, version 'approx_trek_graph', Perron pairs of eig_numpy):
//
//     W2 = W o W,  A = [[W2, w S], [I, W2^T]]  (2d x 2d, nonnegative),  B = A without w S
//     rho, v, u  = Perron root, right / left Perron vectors of A (unit, positive sum)
//     value = (rho - u^T B u / (u^T u + eps)) / m
//     grad  = (2W o (G11 + G22^T) - 2W o (u1 u1^T + u2 u2^T) / (u^T u + eps)) / m,
//             G = u v^T / (u^T v + eps)
//
// The reference takes the Perron pair from two dense non-symmetric eigendecompositions.  Here
// it comes from Noda's iteration (T. Noda, Numer. Math. 17 (1971)), which needs nothing but
// the M-matrix inverse the log-det already has:
//     sigma_0 = max_i (A x)_i / x_i  (Collatz-Wielandt upper bound, x > 0),
//     (sigma_k I - A) y = x_k,  x_{k+1} = y / |y|,  sigma_{k+1} = sigma_k - min_i x_{k,i} / y_i
// sigma_k decreases to rho from above (so sigma_k I - A stays a nonsingular M-matrix and the
// unpivoted Gauss-Jordan of gj.hip applies), quadratically once close; sigma_k - max_i x/y is
// a lower bound, and the iteration stops when the two bounds agree to 1e-13 (or the upper one
// stalls: reducible A).  The iterate of the previous slot is the warm start, so a slot usually
// takes 2-3 inverses; a cold start from ones can take up to ~16 (small W).  A final inverse
// at the converged shift gives v and (its transpose) u by two inverse-iteration sweeps each;
// rho is the two-sided Rayleigh quotient u^T A v / u^T v.
//
// Every kernel obeys a gate word: gate 0 (this slot runs: every slot in 'opt' mode,
// checkpoint slots in 'log' mode), gates 1..TCC_NODA_MAX (Noda step k runs; the update kernel
// turns the later ones off on convergence), so the sequence is graph-capturable.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "launch.h"
#include "tcc_blk.h"

namespace midagma {

namespace {

constexpr int EB = NTHREADS;

__device__ __forceinline__ bool gate_on(const State* g) { return g->status == ST_RUNNING; }

// one-workgroup sum / min / max (fixed order: strided partials, then a tree)
template <class Op>
__device__ double wg_reduce(double v, double* sh, Op op) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int s = EB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = op(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}
struct Add {
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct Min {
  __device__ double operator()(double a, double b) const { return fmin(a, b); }
};
struct Max {
  __device__ double operator()(double a, double b) const { return fmax(a, b); }
};

__global__ void tcc_gate_kernel(const State* __restrict__ st, int mode, State* __restrict__ gates, int nmax,
                                const double* __restrict__ scal) {
  if (threadIdx.x != 0) return;
  const bool on = st->status == ST_RUNNING && (mode == 2 || st->ckpt_pending);
  for (int t = 0; t <= nmax; ++t) gates[t].status = on ? ST_RUNNING : ST_DONE;
  if (TCC_GATE_PRE <= nmax) gates[TCC_GATE_PRE].status = on && scal[16] != 0.0 ? ST_RUNNING : ST_DONE;
}

// A = [[W o W, w S], [I, (W o W)^T]] on the logical 2d x 2d block, zero padding (D2 x D2)
__global__ void tcc_build_kernel(const double* __restrict__ W, const double* __restrict__ S, double ws, int64_t d,
                                 int64_t D, int64_t D2, double* __restrict__ A, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int64_t n = D2 * D2;
  for (int64_t e = (int64_t)blockIdx.x * EB + threadIdx.x; e < n; e += (int64_t)gridDim.x * EB) {
    const int64_t i = e / D2, j = e - i * D2;
    double a = 0.0;
    if (i < d) {
      if (j < d) {
        const double x = W[i * D + j];
        a = x * x;
      } else if (j < 2 * d) {
        a = ws * S[i * D + (j - d)];
      }
    } else if (i < 2 * d) {
      if (j < d) {
        a = (i - d == j) ? 1.0 : 0.0;
      } else if (j < 2 * d) {
        const double x = W[(j - d) * D + (i - d)];
        a = x * x;
      }
    }
    A[e] = a;
  }
}

// x0: the previous slot's Perron vector when that solve converged and the vector is well
// inside the positive cone (a tiny entry would put the Collatz-Wielandt start far above rho),
// else ones
__global__ void tcc_init_kernel(const double* __restrict__ vprev, double* __restrict__ x, int64_t n,
                                const double* __restrict__ scal, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  double mn = INFINITY, mx = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += EB) {
    mn = fmin(mn, vprev[i]);
    mx = fmax(mx, vprev[i]);
  }
  mn = wg_reduce(mn, sh, Min());
  mx = wg_reduce(mx, sh, Max());
  // (scal[10]: the last completed slot's converged flag; scal[9] is this slot's, cleared by
  // tcc_sigma0_kernel, so a slot handed back part-way still warm-starts its re-run)
  const bool warm = scal[8] != 0.0 && scal[10] != 0.0 && mn > 1e-8 * mx && isfinite(mx);
  for (int64_t i = threadIdx.x; i < n; i += EB) x[i] = warm ? vprev[i] : 1.0;
}

// y = M x on rows < n (one wave per row, fixed-order lane tree); skip_tr: B instead of A
// (the top-right d x d block treated as zero)
// (the row block b of tcc_gemv_kernel's grid)
__device__ __forceinline__ void tcc_gemv_body(int64_t b, const double* __restrict__ M, int64_t ld, int64_t n,
                                              int64_t d, int skip_tr, const double* __restrict__ x,
                                              double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t i = b * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t jend = (skip_tr && i < d) ? d : n;
  double acc = 0.0;
  for (int64_t j = lane; j < jend; j += 64) acc += M[i * ld + j] * x[j];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) y[i] = acc;
}

__global__ void tcc_gemv_kernel(const double* __restrict__ M, int64_t ld, int64_t n, int64_t d, int skip_tr,
                                const double* __restrict__ x, double* __restrict__ y, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  tcc_gemv_body(blockIdx.x, M, ld, n, d, skip_tr, x, y);
}

// y = M^T x on columns < n: stage 1, partial sums over 64-row chunks (column block bx, chunk c)
__device__ __forceinline__ void tcc_gemv_t_partial_body(int64_t bx, int64_t c, const double* __restrict__ M,
                                                        int64_t ld, int64_t n, const double* __restrict__ x,
                                                        double* __restrict__ part) {
  const int64_t j = bx * EB + threadIdx.x;
  if (j >= n) return;
  const int64_t i1 = min(n, (c + 1) * 64);
  double acc = 0.0;
  for (int64_t i = c * 64; i < i1; ++i) acc += M[i * ld + j] * x[i];
  part[c * ld + j] = acc;
}

__global__ void tcc_gemv_t_partial_kernel(const double* __restrict__ M, int64_t ld, int64_t n,
                                          const double* __restrict__ x, double* __restrict__ part,
                                          const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  tcc_gemv_t_partial_body(blockIdx.x, blockIdx.y, M, ld, n, x, part);
}

// one sweep's two products in one launch: blocks [0, nrow) y = M x (tcc_gemv_kernel's rows), the
// rest the M^T u partials (tcc_gemv_t_partial_kernel's (column block, chunk) grid, ncb wide)
__global__ void tcc_fix_pass_kernel(const double* __restrict__ M, int64_t ld, int64_t n, int64_t d,
                                    const double* __restrict__ x, double* __restrict__ y,
                                    const double* __restrict__ u, double* __restrict__ part, int64_t nrow,
                                    int64_t ncb, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int64_t b = blockIdx.x;
  if (b < nrow)
    tcc_gemv_body(b, M, ld, n, d, 0, x, y);
  else
    tcc_gemv_t_partial_body((b - nrow) % ncb, (b - nrow) / ncb, M, ld, n, u, part);
}

__global__ void tcc_gemv_t_sum_kernel(const double* __restrict__ part, int64_t ld, int64_t n, int64_t nchunks,
                                      double* __restrict__ y, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int64_t j = (int64_t)blockIdx.x * EB + threadIdx.x;
  if (j >= n) return;
  double acc = 0.0;
  for (int64_t c = 0; c < nchunks; ++c) acc += part[c * ld + j];
  y[j] = acc;
}

// sigma_0 = max_i (A x)_i / x_i  (y = A x)
__global__ void tcc_sigma0_kernel(const double* __restrict__ x, const double* __restrict__ y, int64_t n,
                                  double* __restrict__ scal, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  double mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += EB) mx = fmax(mx, y[i] / x[i]);
  mx = wg_reduce(mx, sh, Max());
  if (threadIdx.x == 0) {
    scal[1] = mx;
    scal[2] = 0.0;  // lower bound (A >= 0)
    scal[7] = 0.0;  // breakdown flag
    scal[9] = 0.0;  // converged flag
    scal[11] = scal[12] = scal[13] = 0.0;  // the fixed-shift stage's flags
    scal[14] = mx;                         // ... its upper bound
    scal[15] = 0.0;                        // ... and its sweep count
  }
}

// Mi = sigma (1 + margin) I - A on the logical block, identity padding
__global__ void tcc_shift_kernel(const double* __restrict__ A, double* __restrict__ Mi, int64_t n, int64_t D2,
                                 const double* __restrict__ scal, double margin, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const double sig = scal[1] * (1.0 + margin);
  const int64_t tot = D2 * D2;
  for (int64_t e = (int64_t)blockIdx.x * EB + threadIdx.x; e < tot; e += (int64_t)gridDim.x * EB) {
    const int64_t i = e / D2, j = e - i * D2;
    double m;
    if (i < n && j < n)
      m = (i == j ? sig : 0.0) - A[e];
    else
      m = (i == j) ? 1.0 : 0.0;
    Mi[e] = m;
  }
}

// Noda update from y = (sigma_k I - A)^-1 x_k; turns gates k+1.. off when the bounds meet
__global__ void tcc_noda_kernel(double* __restrict__ x, const double* __restrict__ y, int64_t n,
                                double* __restrict__ scal, State* __restrict__ gates, int k, int nmax,
                                const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  double rmin = INFINITY, rmax = -INFINITY, ss = 0.0, bad = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += EB) {
    const double yi = y[i];
    if (!(yi > 0.0) || !isfinite(yi)) bad = 1.0;
    const double r = x[i] / yi;
    rmin = fmin(rmin, r);
    rmax = fmax(rmax, r);
    ss += yi * yi;
  }
  rmin = wg_reduce(rmin, sh, Min());
  rmax = wg_reduce(rmax, sh, Max());
  ss = wg_reduce(ss, sh, Add());
  bad = wg_reduce(bad, sh, Max());
  const double sig = scal[1];
  bool stop;
  if (bad != 0.0 || !(ss > 0.0) || !isfinite(ss)) {  // keep x_k, sigma_k: the final inverse uses them
    stop = true;
    if (threadIdx.x == 0) scal[7] = 1.0;
  } else {
    const double inv = 1.0 / sqrt(ss);
    for (int64_t i = threadIdx.x; i < n; i += EB) x[i] = y[i] * inv;
    const double up = sig - rmin, lo = sig - rmax;
    // bounds met, or (reducible A: the lower bound need not tighten) the upper bound stalled
    stop = !(up - lo > 1e-13 * fabs(up)) || !(sig - up > 1e-14 * fabs(up));
    if (threadIdx.x == 0) {
      scal[1] = up;
      scal[2] = lo;
      if (stop) scal[9] = 1.0;  // converged
    }
  }
  if (stop && threadIdx.x == 0)
    for (int t = k + 2; t <= nmax; ++t) gates[t].status = ST_DONE;
}

// out = y / |y|, sign such that sum(out) > 0 (notreks _make_positive_vector)
__global__ void tcc_normalize_kernel(const double* __restrict__ y, double* __restrict__ out, int64_t n,
                                     const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  double ss = 0.0, s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += EB) {
    ss += y[i] * y[i];
    s += y[i];
  }
  ss = wg_reduce(ss, sh, Add());
  s = wg_reduce(s, sh, Add());
  const double inv = (s < 0.0 ? -1.0 : 1.0) / sqrt(ss);
  for (int64_t i = threadIdx.x; i < n; i += EB) out[i] = y[i] * inv;
}

// value = (rho - u^T B u / (u^T u + eps)) / m with rho = u^T A v / u^T v; keeps the
// denominators for the gradient and the vectors for the next slot's warm start
__global__ void tcc_value_kernel(const double* __restrict__ u, const double* __restrict__ v,
                                 const double* __restrict__ Av, const double* __restrict__ Bu, int64_t n, double eps,
                                 double m, double* __restrict__ scal, double* __restrict__ vprev,
                                 double* __restrict__ uprev, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  double uav = 0.0, uv = 0.0, uu = 0.0, ubu = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += EB) {
    uav += u[i] * Av[i];
    uv += u[i] * v[i];
    uu += u[i] * u[i];
    ubu += u[i] * Bu[i];
    vprev[i] = v[i];
    uprev[i] = u[i];
  }
  uav = wg_reduce(uav, sh, Add());
  uv = wg_reduce(uv, sh, Add());
  uu = wg_reduce(uu, sh, Add());
  ubu = wg_reduce(ubu, sh, Add());
  if (threadIdx.x == 0) {
    const double rho = uav / uv;
    const double rho_lb = ubu / (uu + eps);
    const double val = (rho - rho_lb) / m;
    if (isfinite(val)) {
      scal[0] = val;
      scal[3] = rho;
      scal[4] = uv + eps;  // u^T v + eps
      scal[5] = uu + eps;  // u^T u + eps
      scal[8] = 1.0;       // warm start available
      scal[10] = scal[9];  // ... from a converged iteration
    } else {
      // no Perron gap at all (W o W and S nilpotent, e.g. W = 0 at a fit's start): the shifted
      // inverses overflow.  Value 0 and, through infinite denominators, gradient 0 -- the
      // gradient 2 W o G is 0 there anyway; no warm start is kept
      scal[0] = 0.0;
      scal[3] = 0.0;
      scal[4] = INFINITY;
      scal[5] = INFINITY;
      scal[8] = 0.0;
    }
  }
}

// Gtrek[i][j] = weight * (2W o G_W2(A) - 2W o G_W2(lb)) / m on the logical block, 0 elsewhere
__global__ void tcc_grad_kernel(const double* __restrict__ W, const double* __restrict__ u,
                                const double* __restrict__ v, const double* __restrict__ scal, int64_t d, int64_t D,
                                double m, double weight, double* __restrict__ G, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const double denA = scal[4], denB = scal[5];
  const int64_t n = D * D;
  for (int64_t e = (int64_t)blockIdx.x * EB + threadIdx.x; e < n; e += (int64_t)gridDim.x * EB) {
    const int64_t i = e / D, j = e - i * D;
    double g = 0.0;
    if (i < d && j < d) {
      const double w = W[e];
      if (w != 0.0) {
        const double gA = u[i] * v[j] / denA + u[d + j] * v[d + i] / denA;
        const double gB = (u[i] * u[j] + u[d + i] * u[d + j]) / denB;
        g = weight * (((2.0 * w) * gA - (2.0 * w) * gB) / m);
      }
    }
    G[e] = g;
  }
}

// ---- 2d <= 128: the whole TCC sequence in ONE workgroup (tcc_blk.h) --------------------------
using tccb::TccLds;
using tccb::tcc_blk_body;

template <int NB>
__global__ __launch_bounds__(NB * NB) void tcc_blk_kernel(const double* __restrict__ W, const double* __restrict__ S,
                                                            double ws, int d, int64_t D, int mode, double eps,
                                                            double m, double weight, const State* __restrict__ st,
                                                            double* __restrict__ scal, double* __restrict__ vprev,
                                                            double* __restrict__ uprev, double* __restrict__ G,
                                                            int fix) {
  if (!(st->status == ST_RUNNING && (mode == 2 || st->ckpt_pending))) return;  // tcc_gate_kernel's rule
  __shared__ TccLds<NB> L;
  tcc_blk_body<NB, 4>([&](int i, int j) { return W[(int64_t)i * D + j]; },
                   [&](int i, int j) { return S[(int64_t)i * D + j]; }, ws, d, mode, eps, m, weight, scal, vprev,
                   uprev, G, D, L, fix != 0);
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + EB - 1) / EB, 2048); }

// ---- the fixed-shift stage --------------------------------------------------------------------
// With the previous slot's Perron vectors as the warm start, sigma_0 is already close to rho, so
// inverse iteration at the FIXED shift sigma_s = sigma_0 (1 + kFixMargin) converges at the ratio
// (sigma_s - rho) / (sigma_s - lambda_2) per sweep: v from M x and u from M^T u (one pass over
// M = (sigma_s I - A)^-1 >= 0 for both), with ONE inverse per slot instead of Noda's two or three
// plus the final one.  A vector is converged when its ratios x_i / (M x)_i agree to kFixTol
// relative (its relative error); sigma_s - min_i x_i / (M x)_i >= rho is kept as the upper bound
// a Noda continuation starts from when the stage does not converge in TCC_FIX_SWEEPS sweeps (a
// cold start, a small Perron gap) or breaks down (no Perron gap: overflow) -- the Noda steps and
// the final inverse then run as before (their gates stay on).
constexpr double kFixMargin = 1e-14;
constexpr double kFixTol = 1e-13;

// the stage's outcome (thread 0): converged -> Noda and the final inverse gated off
__device__ void tcc_fix_finish(double* __restrict__ scal, State* __restrict__ gates, int easy, int hold) {
  const bool ok = scal[11] != 0.0 && scal[12] != 0.0 && scal[13] == 0.0;
  // the next fast slots' Noda step: on for `hold` slots after a hard stage (without the hold, an
  // easy stage right after a hard one turned it off and the next slot handed back)
  scal[16] = ok && scal[15] <= (double)easy ? fmax(scal[16] - 1.0, 0.0) : (double)hold;
  if (ok) {
    scal[9] = 1.0;
    for (int t = 1; t <= TCC_GATE_FINAL; ++t) gates[t].status = ST_DONE;
  } else if (scal[13] == 0.0) {
    scal[1] = fmin(scal[1], scal[14]);
  }
}

// 2d <= 256 (D2 <= 256): every sweep in one workgroup of 1024 threads (16 waves, row i on wave
// i % 16; the u products' column partials per wave summed in wave order)
__global__ __launch_bounds__(1024) void tcc_fix_small_kernel(const double* __restrict__ Mi, int64_t ld, int n,
                                                             double* __restrict__ x, double* __restrict__ u,
                                                             double* __restrict__ scal, State* __restrict__ gates,
                                                             int hold, int easy, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double xs[256], us[256], ys[256], zp[16][256], red[9][16], gsh[9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < 256) {
    xs[tid] = tid < n ? x[tid] : 0.0;
    us[tid] = tid < n ? u[tid] : 0.0;
  }
  __syncthreads();
  const double sig = scal[1] * (1.0 + kFixMargin);
  bool vok = false, uok = false, bad = false;
  double ub = scal[1];
  int sweeps = 0;
  for (int k = 0; k < TCC_FIX_SWEEPS_SMALL && !(vok && uok); ++k) {
    ++sweeps;
    // this wave's 16 rows (wv + 16 t) in batches of 4, each batch's loads issued before its
    // reduction
    double z[4] = {0.0, 0.0, 0.0, 0.0}, xv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xv[q] = xs[lane + 64 * q];  // (0 past n)
#pragma unroll 1
    for (int bt = 0; bt < 4; ++bt) {
      double acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = wv + 16 * (4 * bt + t);
        const bool rin = i < n;
        const double ui = rin ? us[i] : 0.0;
        const double* __restrict__ row = Mi + (int64_t)(rin ? i : 0) * ld;
        double a = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          const double mij = (rin && j < n) ? row[j] : 0.0;
          a += mij * xv[q];
          z[q] += mij * ui;
        }
        acc[t] = a;
      }
      // the 4 row sums over the wave's lanes, halving the values per lane at each exchange (fixed
      // order): lane bits 5..4 end up selecting the row, bits 3..0 the last four sums
#pragma unroll
      for (int h = 2, off = 32; h >= 1; h >>= 1, off >>= 1) {
        const bool hi = (lane & off) != 0;
#pragma unroll
        for (int t = 0; t < h; ++t) {
          const double keep = hi ? acc[t + h] : acc[t], send = hi ? acc[t] : acc[t + h];
          acc[t] = keep + __shfl_xor(send, off);
        }
      }
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) acc[0] += __shfl_xor(acc[0], off);
      if ((lane & 15) == 0) {
        const int r = ((lane >> 5) & 1) * 2 + ((lane >> 4) & 1);
        const int i = wv + 16 * (4 * bt + r);
        if (i < n) ys[i] = acc[0];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) zp[wv][lane + 64 * q] = z[q];
    __syncthreads();
    // fields: v ratio min / max, |y|^2, sum y; u ratio min / max, |z|^2, sum z; breakdown
    double f[9] = {INFINITY, -INFINITY, 0.0, 0.0, INFINITY, -INFINITY, 0.0, 0.0, 0.0};
    double yi = 0.0, zi = 0.0;
    if (tid < n) {
      yi = ys[tid];
      for (int w2 = 0; w2 < 16; ++w2) zi += zp[w2][tid];
      if (!(yi > 0.0) || !isfinite(yi) || !(zi > 0.0) || !isfinite(zi)) f[8] = 1.0;
      const double rv = xs[tid] / yi, ru = us[tid] / zi;
      f[0] = f[1] = rv;
      f[2] = yi * yi;
      f[3] = yi;
      f[4] = f[5] = ru;
      f[6] = zi * zi;
      f[7] = zi;
    }
#pragma unroll
    for (int c = 0; c < 9; ++c) {
      double a = f[c];
      for (int off = 32; off > 0; off >>= 1) {
        const double b = __shfl_xor(a, off);
        a = (c == 0 || c == 4) ? fmin(a, b) : ((c == 1 || c == 5 || c == 8) ? fmax(a, b) : a + b);
      }
      if (lane == 0) red[c][wv] = a;
    }
    __syncthreads();
    if (tid < 9) {  // field tid over the 16 waves, in wave order
      const int c = tid;
      double a = red[c][0];
      for (int w2 = 1; w2 < 16; ++w2) {
        const double b = red[c][w2];
        a = (c == 0 || c == 4) ? fmin(a, b) : ((c == 1 || c == 5 || c == 8) ? fmax(a, b) : a + b);
      }
      gsh[c] = a;
    }
    __syncthreads();
    double g[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) g[c] = gsh[c];
    if (g[8] != 0.0 || !(g[2] > 0.0) || !(g[6] > 0.0) || !isfinite(g[2]) || !isfinite(g[6])) {
      bad = true;  // (x, u keep the last good sweep's vectors)
      break;
    }
    vok = !(g[1] - g[0] > kFixTol * g[0]);
    uok = !(g[5] - g[4] > kFixTol * g[4]);
    ub = fmin(ub, sig - g[0]);
    if (tid < n) {
      xs[tid] = yi * ((g[3] < 0.0 ? -1.0 : 1.0) / sqrt(g[2]));
      us[tid] = zi * ((g[7] < 0.0 ? -1.0 : 1.0) / sqrt(g[6]));
    }
    __syncthreads();
  }
  if (tid < n) {
    x[tid] = xs[tid];
    u[tid] = us[tid];
  }
  if (tid == 0) {
    scal[11] = vok ? 1.0 : 0.0;
    scal[12] = uok ? 1.0 : 0.0;
    scal[13] = bad ? 1.0 : 0.0;
    scal[14] = ub;
    scal[15] = vok && uok ? (double)sweeps : 0.0;
    tcc_fix_finish(scal, gates, easy > 0 ? easy : TCC_FIX_EASY_SMALL, hold);
  }
}

// 2d > 256: one sweep's update after y = M x and z = M^T u (the GEMV kernels): both vectors
// renormalised, the convergence and breakdown flags, the later sweeps gated off when done
__global__ void tcc_fix_update_kernel(double* __restrict__ x, const double* __restrict__ y, double* __restrict__ u,
                                      double* __restrict__ z, const double* __restrict__ part, int64_t ld,
                                      int64_t nchunks, int64_t n, double* __restrict__ scal,
                                      State* __restrict__ gates, int k, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double sh[EB];
  // z = M^T u from the chunk partials (tcc_gemv_t_sum_kernel's order; nchunks = 0: z given)
  if (nchunks > 0) {
    for (int64_t j = threadIdx.x; j < n; j += EB) {
      double acc = 0.0;
      for (int64_t c = 0; c < nchunks; ++c) acc += part[c * ld + j];
      z[j] = acc;
    }
    __syncthreads();
  }
  double vmin = INFINITY, vmax = -INFINITY, vss = 0.0, vs = 0.0;
  double umin = INFINITY, umax = -INFINITY, uss = 0.0, us = 0.0, bad = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += EB) {
    const double yi = y[i], zi = z[i];
    if (!(yi > 0.0) || !isfinite(yi) || !(zi > 0.0) || !isfinite(zi)) bad = 1.0;
    const double rv = x[i] / yi, ru = u[i] / zi;
    vmin = fmin(vmin, rv);
    vmax = fmax(vmax, rv);
    vss += yi * yi;
    vs += yi;
    umin = fmin(umin, ru);
    umax = fmax(umax, ru);
    uss += zi * zi;
    us += zi;
  }
  vmin = wg_reduce(vmin, sh, Min());
  vmax = wg_reduce(vmax, sh, Max());
  vss = wg_reduce(vss, sh, Add());
  vs = wg_reduce(vs, sh, Add());
  umin = wg_reduce(umin, sh, Min());
  umax = wg_reduce(umax, sh, Max());
  uss = wg_reduce(uss, sh, Add());
  us = wg_reduce(us, sh, Add());
  bad = wg_reduce(bad, sh, Max());
  const bool brk = bad != 0.0 || !(vss > 0.0) || !(uss > 0.0) || !isfinite(vss) || !isfinite(uss);
  bool done = brk;
  if (!brk) {
    const double iv = (vs < 0.0 ? -1.0 : 1.0) / sqrt(vss), iu = (us < 0.0 ? -1.0 : 1.0) / sqrt(uss);
    for (int64_t i = threadIdx.x; i < n; i += EB) {
      x[i] = y[i] * iv;
      u[i] = z[i] * iu;
    }
    const bool vok = !(vmax - vmin > kFixTol * vmin), uok = !(umax - umin > kFixTol * umin);
    done = vok && uok;
    if (threadIdx.x == 0) {
      scal[11] = vok ? 1.0 : 0.0;
      scal[12] = uok ? 1.0 : 0.0;
      scal[14] = fmin(scal[14], scal[1] * (1.0 + kFixMargin) - vmin);
      if (done) scal[15] = (double)(k + 1);
    }
  } else if (threadIdx.x == 0) {
    scal[13] = 1.0;
  }
  if (done && threadIdx.x == 0)
    for (int t = k + 1; t < TCC_FIX_SWEEPS; ++t) gates[TCC_GATE_FIX0 + t].status = ST_DONE;
}

__global__ void tcc_fix_done_kernel(double* __restrict__ scal, State* __restrict__ gates, int hold, int easy,
                                    const State* __restrict__ gate) {
  if (!gate_on(gate) || threadIdx.x != 0) return;
  tcc_fix_finish(scal, gates, easy > 0 ? easy : TCC_FIX_EASY, hold);
}


// the shifted inverse: the two-level blocked one (pivoted path: 256-blocks, panels, MFMA trailing
// updates) where the solver allocated its buffers (D2 >= 2048), else the flat 32-block Gauss-Jordan
BInvWork tcc_binv(const TccWork& w) {
  BInvWork b{};
  b.Aalt = w.Aalt;
  b.Pst = w.Pst;
  b.Pst1 = w.Pst1;
  b.Y[0] = w.Y0;
  b.Y[1] = w.Y1;
  b.Q[0] = w.Q0;
  b.Q[1] = w.Q1;
  b.P = w.Pblk;
  b.part = w.part2;
  b.done = w.done;
  return b;
}
double* tcc_inv_input(const TccWork& w) { return w.Aalt ? binv_build_target(w.Mi, w.D2, tcc_binv(w)) : w.Mi; }
void tcc_inverse(const TccWork& w, const GJWork& gj, const State* gate, hipStream_t stream) {
  if (w.Aalt)
    launch_blocked_inverse(w.Mi, w.D2, tcc_binv(w), /*fast=*/false, gj, const_cast<State*>(gate), stream);
  else
    launch_gj_inverse(w.Mi, w.D2, w.D2, gj, gate, stream);
}
// the fast slot's fixed-stage inverse with the fast-block buffers (w.Y0): every outer block but the
// last by the product-form series warm-started from the last slot's block inverses (w.Pst, one
// ring slot: the gate words' slot count never advances, so Pst1 aliases Pst and no extrapolation
// runs), the last (whose Schur complement carries the near-singularity) by the pivoted
// Gauss-Jordan.  A block whose series does not converge sets the gate's status to ST_NEED_GJ: the
// rest of the stage is skipped and tcc_handback_kernel hands the slot back.
void tcc_inverse_fix(const TccWork& w, const GJWork& gj, const State* gate, bool fast, hipStream_t stream) {
  if (!(fast && w.Aalt && w.Y0)) return tcc_inverse(w, gj, gate, stream);
  const int K2 = (int)(w.D2 / binv_block(w.D2));
  launch_blocked_inverse(w.Mi, w.D2, tcc_binv(w), /*fast=*/true, gj, const_cast<State*>(gate), stream, NM_PASSES_RUN,
                         nullptr, nullptr, false, nullptr, K2 - 1);
}

// a truncated chain (launch_trek_tcc's handback form): Noda still running after `steps` steps
// (its gate for step `steps` not turned off) hands the slot back and gates off the final part
__global__ void tcc_handback_kernel(State* __restrict__ st, State* __restrict__ gates, int steps) {
  if (threadIdx.x != 0) return;
  if (gates[0].status == ST_NEED_GJ) {  // the fast-block inverse did not converge (tcc_inverse_fix)
    st->status = ST_NEED_GJ;
    gates[0].status = ST_DONE;
    gates[TCC_GATE_FINAL].status = ST_DONE;
    return;
  }
  if (gates[0].status != ST_RUNNING || gates[1 + steps].status != ST_RUNNING) return;
  st->status = ST_NEED_GJ;
  gates[0].status = ST_DONE;
  gates[TCC_GATE_FINAL].status = ST_DONE;
}

}  // namespace

void launch_trek_tcc(const double* W, int64_t d, int64_t D, const TccCfg& cfg, const TccWork& w, const State* st,
                     double* Gtrek, hipStream_t stream, State* handback, int steps) {
  const int64_t n = 2 * d, D2 = w.D2;
  static const bool chain = knob_set("MIDAGMA_EXP_TCC_CHAIN");  // experiments: the launch sequence at every d
  if (n <= 128 && !chain) {
    // one workgroup of 4 x 4 register blocks: 64 threads up to 2d = 32, 256 up to 64, 1024 up to 128
    const long nb = knob("MIDAGMA_EXP_TCC_NB", 0);  // experiments: force the block count
    auto go = [&](auto kern, int nt) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(nt), 0, stream, W, w.S, cfg.w, (int)d, D, cfg.mode, cfg.eps,
                         (double)cfg.m, cfg.weight, st, w.scal, w.vprev, w.uprev, Gtrek, w.fix);
    };
    if ((nb == 8 || (nb == 0 && n <= 32)) && n <= 32)
      go(tcc_blk_kernel<8>, 64);
    else if ((nb == 16 || (nb == 0 && n <= 64)) && n <= 64)
      go(tcc_blk_kernel<16>, 256);
    else
      go(tcc_blk_kernel<32>, 1024);
    HIP_TRY(hipGetLastError());
    return;
  }
  State* g0 = w.gates;
  const double m = (double)cfg.m;
  hipLaunchKernelGGL(tcc_gate_kernel, dim3(1), dim3(64), 0, stream, st, cfg.mode, w.gates, TCC_GATES - 1, w.scal);
  hipLaunchKernelGGL(tcc_build_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, W, w.S, cfg.w, d, D, D2, w.A,
                     g0);
  const dim3 gv((unsigned)((n + 3) / 4));
  const dim3 gt((unsigned)((n + EB - 1) / EB), (unsigned)((n + 63) / 64));
  const dim3 gts((unsigned)((n + EB - 1) / EB));
  const int64_t nchunks = (n + 63) / 64;
  GJWork gj = w.gj;
  gj.pivlog = nullptr;
  gj.Pstore = nullptr;
  // sigma_0 from the warm start
  hipLaunchKernelGGL(tcc_init_kernel, dim3(1), dim3(EB), 0, stream, w.vprev, w.x, n, w.scal, g0);
  hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.A, D2, n, d, 0, w.x, w.y, g0);
  hipLaunchKernelGGL(tcc_sigma0_kernel, dim3(1), dim3(EB), 0, stream, w.x, w.y, n, w.scal, g0);
  // one Noda step (tcc_noda_kernel's update; gate 1 + k, or gk)
  auto noda_step = [&](int k, const State* gk) {
    hipLaunchKernelGGL(tcc_shift_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, w.A, tcc_inv_input(w), n, D2,
                       w.scal, 0.0, gk);
    tcc_inverse(w, gj, gk, stream);
    hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.Mi, D2, n, d, 0, w.x, w.y, gk);
    hipLaunchKernelGGL(tcc_noda_kernel, dim3(1), dim3(EB), 0, stream, w.x, w.y, n, w.scal, w.gates, k, TCC_NODA_MAX,
                       gk);
  };
  // the fast slot's chain (handback): with the fixed-shift stage, `fix_pre` Noda steps when the last
  // stage was hard (took more than TCC_FIX_EASY sweeps or did not settle: their shift update brings
  // sigma much closer to rho than the warm start's bound), then the stage, and a slot that is still
  // not settled hands back at once (no further Noda step and no final inverse enqueued: their gated
  // launches alone cost more than the stage); without it, `steps` Noda steps
  const bool lean = handback && w.fix;
  const int pre = lean ? std::max(0, std::min(w.fix_pre, TCC_NODA_MAX - 1)) : 0;
  for (int k = 0; k < pre; ++k) noda_step(k, &w.gates[TCC_GATE_PRE]);
  // the fixed-shift stage (w.fix = 0, MIDAGMA_EXP_TCC_FIX=0: Noda from the warm start at once)
  if (w.fix) {
    hipLaunchKernelGGL(tcc_shift_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, w.A, tcc_inv_input(w), n, D2,
                       w.scal, kFixMargin, g0);
    tcc_inverse_fix(w, gj, g0, lean, stream);
    hipLaunchKernelGGL(tcc_init_kernel, dim3(1), dim3(EB), 0, stream, w.uprev, w.u, n, w.scal, g0);
    if (D2 <= 256) {
      hipLaunchKernelGGL(tcc_fix_small_kernel, dim3(1), dim3(1024), 0, stream, w.Mi, D2, (int)n, w.x, w.u, w.scal,
                         w.gates, w.fix_hold, w.fix_easy, g0);
    } else {
      // both products in one pass launch, then z's chunk sum and the update: in the update's one
      // workgroup up to 12 chunks (2d <= 768), in a launch of its own beyond (measured: at 2d = 2000
      // the one-workgroup sum of 32 chunks cost more than the launch it saves)
      const int64_t nrow = gv.x, ncb = gt.x;
      const dim3 gp((unsigned)(nrow + ncb * (int64_t)gt.y));
      const bool own_sum = nchunks > 12;
      for (int k = 0; k < TCC_FIX_SWEEPS; ++k) {
        const State* gk = &w.gates[TCC_GATE_FIX0 + k];
        hipLaunchKernelGGL(tcc_fix_pass_kernel, gp, dim3(EB), 0, stream, w.Mi, D2, n, d, w.x, w.y, w.u, w.part, nrow,
                           ncb, gk);
        if (own_sum)
          hipLaunchKernelGGL(tcc_gemv_t_sum_kernel, gts, dim3(EB), 0, stream, w.part, D2, n, nchunks, w.z, gk);
        hipLaunchKernelGGL(tcc_fix_update_kernel, dim3(1), dim3(EB), 0, stream, w.x, w.y, w.u, w.z, w.part, D2,
                           own_sum ? (int64_t)0 : nchunks, n, w.scal, w.gates, k, gk);
      }
      hipLaunchKernelGGL(tcc_fix_done_kernel, dim3(1), dim3(64), 0, stream, w.scal, w.gates, w.fix_hold, w.fix_easy,
                         g0);
    }
  }
  const int nsteps = lean ? 0 : (handback ? std::min(std::max(steps, 1), TCC_NODA_MAX - 1) : TCC_NODA_MAX);
  for (int k = 0; k < nsteps; ++k) noda_step(k, &w.gates[1 + k]);
  if (handback) hipLaunchKernelGGL(tcc_handback_kernel, dim3(1), dim3(64), 0, stream, handback, w.gates, nsteps);
  // final inverse just above the converged root: two sweeps for v, two (transposed) for u (the
  // Noda path: gated off when the fixed-shift stage converged)
  const State* gf = &w.gates[TCC_GATE_FINAL];
  if (!lean) {
    hipLaunchKernelGGL(tcc_shift_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, w.A, tcc_inv_input(w), n, D2,
                       w.scal, 1e-14, gf);
    tcc_inverse(w, gj, gf, stream);
    for (int r = 0; r < 2; ++r) {
      hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.Mi, D2, n, d, 0, w.x, w.y, gf);
      hipLaunchKernelGGL(tcc_normalize_kernel, dim3(1), dim3(EB), 0, stream, w.y, w.x, n, gf);
    }
    hipLaunchKernelGGL(tcc_init_kernel, dim3(1), dim3(EB), 0, stream, w.uprev, w.u, n, w.scal, gf);
    for (int r = 0; r < 2; ++r) {
      hipLaunchKernelGGL(tcc_gemv_t_partial_kernel, gt, dim3(EB), 0, stream, w.Mi, D2, n, w.u, w.part, gf);
      hipLaunchKernelGGL(tcc_gemv_t_sum_kernel, gts, dim3(EB), 0, stream, w.part, D2, n, nchunks, w.y, gf);
      hipLaunchKernelGGL(tcc_normalize_kernel, dim3(1), dim3(EB), 0, stream, w.y, w.u, n, gf);
    }
  }
  // rho (Rayleigh), the lower bound through B, value; then the gradient
  hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.A, D2, n, d, 0, w.x, w.y, g0);
  hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.A, D2, n, d, 1, w.u, w.z, g0);
  hipLaunchKernelGGL(tcc_value_kernel, dim3(1), dim3(EB), 0, stream, w.u, w.x, w.y, w.z, n, cfg.eps, m, w.scal,
                     w.vprev, w.uprev, g0);
  if (cfg.mode == 2)
    hipLaunchKernelGGL(tcc_grad_kernel, dim3(grid_for(D * D)), dim3(EB), 0, stream, W, w.u, w.x, w.scal, d, D, m,
                       cfg.weight, Gtrek, g0);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
