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
#include <cmath>
#include <type_traits>

#include "launch.h"

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

__global__ void tcc_gate_kernel(const State* __restrict__ st, int mode, State* __restrict__ gates, int nmax) {
  if (threadIdx.x != 0) return;
  const bool on = st->status == ST_RUNNING && (mode == 2 || st->ckpt_pending);
  for (int t = 0; t <= nmax; ++t) gates[t].status = on ? ST_RUNNING : ST_DONE;
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
  const bool warm = scal[8] != 0.0 && scal[9] != 0.0 && mn > 1e-8 * mx && isfinite(mx);
  for (int64_t i = threadIdx.x; i < n; i += EB) x[i] = warm ? vprev[i] : 1.0;
}

// y = M x on rows < n (one wave per row, fixed-order lane tree); skip_tr: B instead of A
// (the top-right d x d block treated as zero)
__global__ void tcc_gemv_kernel(const double* __restrict__ M, int64_t ld, int64_t n, int64_t d, int skip_tr,
                                const double* __restrict__ x, double* __restrict__ y, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t jend = (skip_tr && i < d) ? d : n;
  double acc = 0.0;
  for (int64_t j = lane; j < jend; j += 64) acc += M[i * ld + j] * x[j];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) y[i] = acc;
}

// y = M^T x on columns < n: stage 1, partial sums over 64-row chunks
__global__ void tcc_gemv_t_partial_kernel(const double* __restrict__ M, int64_t ld, int64_t n,
                                          const double* __restrict__ x, double* __restrict__ part,
                                          const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int64_t j = (int64_t)blockIdx.x * EB + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (j >= n) return;
  const int64_t i1 = min(n, (c + 1) * 64);
  double acc = 0.0;
  for (int64_t i = c * 64; i < i1; ++i) acc += M[i * ld + j] * x[i];
  part[c * ld + j] = acc;
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

// ---- 2d <= 128: the whole TCC sequence in ONE workgroup of 4 x 4 register blocks --------------
// The launch-per-kernel sequence above is ~170 dependent launches per slot (24 gated Noda steps of
// shift, Gauss-Jordan prologue and steps, GEMV and update), almost all no-ops once Noda converged:
// at d = 20 that was 0.40 ms per Adam step.  Here every step of the same algorithm (the same
// Collatz-Wielandt start, Noda updates, stopping rules, breakdown handling, final sweeps, value and
// gradient, and the same scal / warm-start words) runs in one workgroup of NB x NB threads: thread
// (a, b) keeps rows 4a..4a+3 x columns 4b..4b+3 of A and of the shifted matrix / its inverse in
// registers.  The inverses are unpivoted Gauss-Jordan (sigma I - A is a nonsingular M-matrix on
// every Noda step) with ONE barrier per pivot: the owners of row and column p + 1 publish them to a
// double-buffered LDS pair as soon as pivot p's update is done.  GEMVs reduce a row block's 4 x 4
// partials over the NB lanes of the same a by butterfly (fixed order); the vector steps (Noda
// update, normalisation, value) run in wave 0 with wave reductions.  scal[6] counts the inverses of
// the call (diagnostic).
template <int NB>
struct TccBlk {
  static constexpr int NT = NB * NB;  // threads
  static constexpr int NM = 4 * NB;   // largest 2d
  static constexpr int VT = NM > 64 ? NM / 64 : 1;  // vector entries per wave-0 lane
};

// fixed-order butterfly over the 64 lanes of a wave (every lane ends with the result)
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) v = op(v, __shfl_xor(v, off));
  return v;
}

// M (holding A's block) <- sig I - A on the logical block, identity padding
__device__ __forceinline__ void blk_shift(double (&M)[4][4], int n, int a, int b, double sig) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = 4 * a + r, j = 4 * b + c;
      M[r][c] = (i < n && j < n) ? ((i == j ? sig : 0.0) - M[r][c]) : (i == j ? 1.0 : 0.0);
    }
}

// in-place unpivoted Gauss-Jordan inverse of the block-distributed matrix.  Pivot p's update is
// one rank-1 form for every entry, M'[i][j] = M~[i][j] - c[i] r[j], where the publishers of pivot p
// hand over r = row p with r[p] = 1, c = column p with c[p] = piv - 1, and replace column p of their
// blocks by e_p; with r scaled by 1 / piv this gives row p / piv, column p times -1 / piv and
// 1 / piv at the pivot (gj.hip's result, in a different rounding).  The pivot loop runs over 4-row
// blocks with the row inside the block unrolled, so every register index is static; the identity
// padding up to a multiple of 4 pivots on 1 and changes nothing.
template <int NB>
__device__ __forceinline__ void blk_gj_inverse(double (&M)[4][4], int n, int a, int b, double (*rowb)[4 * NB],
                                               double (*colb)[4 * NB], double* pivb) {
  auto publish = [&](int q, auto Rc, int buf) {
    constexpr int R = decltype(Rc)::value;
    if (a == q) {
#pragma unroll
      for (int c = 0; c < 4; ++c) rowb[buf][4 * b + c] = (b == q && c == R) ? 1.0 : M[R][c];
    }
    if (b == q) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool piv = a == q && r == R;
        colb[buf][4 * a + r] = piv ? M[r][R] - 1.0 : M[r][R];
        if (piv) pivb[buf] = M[r][R];
        M[r][R] = piv ? 1.0 : 0.0;
      }
    }
  };
  auto step = [&](int q, auto Rc, int nq) {
    constexpr int R = decltype(Rc)::value;
    constexpr int buf = R & 1;  // the parity of p = 4 q + R
    __syncthreads();
    const double inv = 1.0 / pivb[buf];
    double rp[4], cp[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) rp[c] = rowb[buf][4 * b + c] * inv;
#pragma unroll
    for (int r = 0; r < 4; ++r) cp[r] = colb[buf][4 * a + r];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) M[r][c] = M[r][c] - cp[r] * rp[c];
    if constexpr (R < 3)
      publish(q, std::integral_constant<int, R + 1>(), buf ^ 1);
    else if (q + 1 < nq)
      publish(q + 1, std::integral_constant<int, 0>(), buf ^ 1);
  };
  const int nq = (n + 3) >> 2;
  publish(0, std::integral_constant<int, 0>(), 0);
  for (int q = 0; q < nq; ++q) {
    step(q, std::integral_constant<int, 0>(), nq);
    step(q, std::integral_constant<int, 1>(), nq);
    step(q, std::integral_constant<int, 2>(), nq);
    step(q, std::integral_constant<int, 3>(), nq);
  }
}

// y = M x (x, y in LDS, NM entries): each thread's 4 row partials over its 4 columns, summed over
// the NB threads of its row block (consecutive lanes) by butterfly
template <int NB>
__device__ __forceinline__ void blk_gemv(const double (&M)[4][4], int a, int b, bool skip_tr, int d,
                                         const double* x, double* y) {
  double xv[4], s[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) xv[c] = x[4 * b + c];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool zero = skip_tr && 4 * a + r < d && 4 * b + c >= d;  // B: top-right block 0
      acc += zero ? 0.0 : M[r][c] * xv[c];
    }
    s[r] = acc;
  }
#pragma unroll
  for (int off = 1; off < NB; off <<= 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] += __shfl_xor(s[r], off);
  if (b == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) y[4 * a + r] = s[r];
  }
  __syncthreads();
}

// y = M^T u: column partials per thread, summed over the row blocks of a wave by butterfly, then
// over the waves through LDS (fixed order)
template <int NB>
__device__ __forceinline__ void blk_gemv_t(const double (&M)[4][4], int a, int b, const double* u,
                                           double (*part)[4 * NB], double* y) {
  constexpr int NW = NB * NB / 64;  // waves
  double uv[4], t[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) uv[r] = u[4 * a + r];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc += M[r][c] * uv[r];
    t[c] = acc;
  }
#pragma unroll
  for (int off = NB; off < 64; off <<= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] += __shfl_xor(t[c], off);
  if ((threadIdx.x & 63) < NB) {
#pragma unroll
    for (int c = 0; c < 4; ++c) part[threadIdx.x >> 6][4 * b + c] = t[c];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 4 * NB; j += NB * NB) {
    double acc = 0.0;
    for (int w = 0; w < NW; ++w) acc += part[w][j];
    y[j] = acc;
  }
  __syncthreads();
}

// wave 0: warm start (tcc_init_kernel) into out: prev when the last solve converged and is inside
// the cone, else ones (0 on the padding)
template <int NB>
__device__ __forceinline__ void w0_init(const double* __restrict__ prev, int n, bool conv, bool warm_ok,
                                        double* out) {
  const int lane = threadIdx.x;
  double pv[TccBlk<NB>::VT], mn = INFINITY, mx = 0.0;
#pragma unroll
  for (int t = 0; t < TccBlk<NB>::VT; ++t) {
    const int e = lane + 64 * t;
    pv[t] = e < n ? prev[e] : 0.0;
    if (e < n) {
      mn = fmin(mn, pv[t]);
      mx = fmax(mx, pv[t]);
    }
  }
  mn = wave_reduce(mn, Min());
  mx = wave_reduce(mx, Max());
  const bool warm = warm_ok && conv && mn > 1e-8 * mx && isfinite(mx);
#pragma unroll
  for (int t = 0; t < TccBlk<NB>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < TccBlk<NB>::NM) out[e] = e < n ? (warm ? pv[t] : 1.0) : 0.0;
  }
}

// wave 0: out = y / |y| with sum(out) > 0 (tcc_normalize_kernel), 0 on the padding
template <int NB>
__device__ __forceinline__ void w0_normalize(const double* y, int n, double* out) {
  const int lane = threadIdx.x;
  double ss = 0.0, sm = 0.0;
#pragma unroll
  for (int t = 0; t < TccBlk<NB>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < n) {
      ss += y[e] * y[e];
      sm += y[e];
    }
  }
  ss = wave_reduce(ss, Add());
  sm = wave_reduce(sm, Add());
  const double inv = (sm < 0.0 ? -1.0 : 1.0) / sqrt(ss);
#pragma unroll
  for (int t = 0; t < TccBlk<NB>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < n) out[e] = y[e] * inv;
  }
}

template <int NB>
__global__ __launch_bounds__(NB * NB) void tcc_blk_kernel(const double* __restrict__ W, const double* __restrict__ S,
                                                            double ws, int d, int64_t D, int mode, double eps,
                                                            double m, double weight, const State* __restrict__ st,
                                                            double* __restrict__ scal, double* __restrict__ vprev,
                                                            double* __restrict__ uprev, double* __restrict__ G) {
  if (!(st->status == ST_RUNNING && (mode == 2 || st->ckpt_pending))) return;  // tcc_gate_kernel's rule
  constexpr int NM = TccBlk<NB>::NM, VT = TccBlk<NB>::VT;
  __shared__ double rowb[2][NM], colb[2][NM], part[NB * NB / 64][NM];
  __shared__ double xs[NM], ys[NM], us[NM], zs[NM], scs[16], pivb[2];
  const int tid = threadIdx.x, a = tid / NB, b = tid % NB, lane = tid & 63;
  const bool w0 = tid < 64;
  const int n = 2 * d;
  // A (the logical 2d x 2d block, zero padding) in LDS; registers hold the working matrix only
  constexpr int LA = NM + 2;
  __shared__ double al[NM * LA];
  for (int e = tid; e < NM * NM; e += TccBlk<NB>::NT) {  // tcc_build_kernel
    const int i = e / NM, j = e - i * NM;
    double v = 0.0;
    if (i < d) {
      if (j < d) {
        const double w = W[(int64_t)i * D + j];
        v = w * w;
      } else if (j < n) {
        v = ws * S[(int64_t)i * D + (j - d)];
      }
    } else if (i < n) {
      if (j < d) {
        v = (i - d == j) ? 1.0 : 0.0;
      } else if (j < n) {
        const double w = W[(int64_t)(j - d) * D + (i - d)];
        v = w * w;
      }
    }
    al[i * LA + j] = v;
  }
  __syncthreads();
  double M[4][4];
  auto load_a = [&](double (&T)[4][4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) T[r][c] = al[(4 * a + r) * LA + 4 * b + c];
  };
  load_a(M);
  double sc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) sc[t] = scal[t];
  if (w0) w0_init<NB>(vprev, n, sc[9] != 0.0, sc[8] != 0.0, xs);
  __syncthreads();
  blk_gemv<NB>(M, a, b, false, d, xs, ys);
  if (w0) {  // tcc_sigma0_kernel
    double mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int e = lane + 64 * t;
      if (e < n) mx = fmax(mx, ys[e] / xs[e]);
    }
    mx = wave_reduce(mx, Max());
    if (lane == 0) scs[1] = mx;
  }
  __syncthreads();
  sc[1] = scs[1];
  sc[2] = 0.0;
  sc[7] = 0.0;
  sc[9] = 0.0;
  int ninv = 0;
  for (int k = 0; k < TCC_NODA_MAX; ++k) {  // tcc_noda_kernel, until the stop rule
    ++ninv;
    load_a(M);
    blk_shift(M, n, a, b, sc[1]);
    blk_gj_inverse<NB>(M, n, a, b, rowb, colb, pivb);
    blk_gemv<NB>(M, a, b, false, d, xs, ys);
    if (w0) {
      double rmin = INFINITY, rmax = -INFINITY, ss = 0.0, bad = 0.0;
#pragma unroll
      for (int t = 0; t < VT; ++t) {
        const int e = lane + 64 * t;
        if (e < n) {
          const double yi = ys[e];
          if (!(yi > 0.0) || !isfinite(yi)) bad = 1.0;
          const double r = xs[e] / yi;
          rmin = fmin(rmin, r);
          rmax = fmax(rmax, r);
          ss += yi * yi;
        }
      }
      rmin = wave_reduce(rmin, Min());
      rmax = wave_reduce(rmax, Max());
      ss = wave_reduce(ss, Add());
      bad = wave_reduce(bad, Max());
      const double sig = sc[1];
      double up = sig, lo = sc[2], brk = 0.0, stop = 1.0;
      if (bad != 0.0 || !(ss > 0.0) || !isfinite(ss)) {  // keep x_k, sigma_k: the final inverse uses them
        brk = 1.0;
      } else {
        const double inv = 1.0 / sqrt(ss);
#pragma unroll
        for (int t = 0; t < VT; ++t) {
          const int e = lane + 64 * t;
          if (e < n) xs[e] = ys[e] * inv;
        }
        up = sig - rmin;
        lo = sig - rmax;
        // bounds met, or (reducible A: the lower bound need not tighten) the upper bound stalled
        stop = (!(up - lo > 1e-13 * fabs(up)) || !(sig - up > 1e-14 * fabs(up))) ? 1.0 : 0.0;
      }
      if (lane == 0) {
        scs[1] = up;
        scs[2] = lo;
        scs[7] = brk;
        scs[9] = (brk == 0.0 && stop != 0.0) ? 1.0 : 0.0;
        scs[10] = stop;
      }
    }
    __syncthreads();
    sc[1] = scs[1];
    sc[2] = scs[2];
    sc[7] = scs[7];
    sc[9] = scs[9];
    if (scs[10] != 0.0) break;
  }
  // the final inverse just above the root: two sweeps for v (x), two transposed for u
  load_a(M);
  blk_shift(M, n, a, b, sc[1] * (1.0 + 1e-14));
  blk_gj_inverse<NB>(M, n, a, b, rowb, colb, pivb);
  ++ninv;
  for (int t = 0; t < 2; ++t) {
    blk_gemv<NB>(M, a, b, false, d, xs, ys);
    if (w0) w0_normalize<NB>(ys, n, xs);
    __syncthreads();
  }
  if (w0) w0_init<NB>(uprev, n, sc[9] != 0.0, sc[8] != 0.0, us);
  __syncthreads();
  for (int t = 0; t < 2; ++t) {
    blk_gemv_t<NB>(M, a, b, us, part, ys);
    if (w0) w0_normalize<NB>(ys, n, us);
    __syncthreads();
  }
  load_a(M);  // the inverse is no longer needed
  blk_gemv<NB>(M, a, b, false, d, xs, ys);  // A v
  blk_gemv<NB>(M, a, b, true, d, us, zs);   // B u
  if (w0) {  // tcc_value_kernel
    double uav = 0.0, uv = 0.0, uu = 0.0, ubu = 0.0;
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int e = lane + 64 * t;
      if (e < n) {
        const double u = us[e], v = xs[e];
        uav += u * ys[e];
        uv += u * v;
        uu += u * u;
        ubu += u * zs[e];
        vprev[e] = v;
        uprev[e] = u;
      }
    }
    uav = wave_reduce(uav, Add());
    uv = wave_reduce(uv, Add());
    uu = wave_reduce(uu, Add());
    ubu = wave_reduce(ubu, Add());
    const double rho = uav / uv;
    const double val = (rho - ubu / (uu + eps)) / m;
    if (isfinite(val)) {
      sc[0] = val;
      sc[3] = rho;
      sc[4] = uv + eps;
      sc[5] = uu + eps;
      sc[8] = 1.0;
    } else {
      // no Perron gap (W o W and S nilpotent, e.g. W = 0): value 0, gradient 0 through the
      // infinite denominators, no warm start kept (tcc_value_kernel)
      sc[0] = 0.0;
      sc[3] = 0.0;
      sc[4] = INFINITY;
      sc[5] = INFINITY;
      sc[8] = 0.0;
    }
    sc[6] = (double)ninv;
    if (lane == 0) {
#pragma unroll
      for (int t = 0; t < 10; ++t) scal[t] = sc[t];
      scs[4] = sc[4];
      scs[5] = sc[5];
    }
  }
  if (mode == 2) {  // tcc_grad_kernel on the logical d x d block (the padding stays 0)
    __syncthreads();
    const double denA = scs[4], denB = scs[5];
    for (int e = tid; e < d * d; e += TccBlk<NB>::NT) {
      const int i = e / d, j = e - i * d;
      const double w = W[(int64_t)i * D + j];
      double g = 0.0;
      if (w != 0.0) {
        const double gA = us[i] * xs[j] / denA + us[d + j] * xs[d + i] / denA;
        const double gB = (us[i] * us[j] + us[d + i] * us[d + j]) / denB;
        g = weight * (((2.0 * w) * gA - (2.0 * w) * gB) / m);
      }
      G[(int64_t)i * D + j] = g;
    }
  }
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + EB - 1) / EB, 2048); }

}  // namespace

void launch_trek_tcc(const double* W, int64_t d, int64_t D, const TccCfg& cfg, const TccWork& w, const State* st,
                     double* Gtrek, hipStream_t stream) {
  const int64_t n = 2 * d, D2 = w.D2;
  static const bool chain = knob_set("MIDAGMA_EXP_TCC_CHAIN");  // experiments: the launch sequence at every d
  if (n <= 128 && !chain) {
    // one workgroup of 4 x 4 register blocks: 64 threads up to 2d = 32, 256 up to 64, 1024 up to 128
    const long nb = knob("MIDAGMA_EXP_TCC_NB", 0);  // experiments: force the block count
    auto go = [&](auto kern, int nt) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(nt), 0, stream, W, w.S, cfg.w, (int)d, D, cfg.mode, cfg.eps,
                         (double)cfg.m, cfg.weight, st, w.scal, w.vprev, w.uprev, Gtrek);
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
  hipLaunchKernelGGL(tcc_gate_kernel, dim3(1), dim3(64), 0, stream, st, cfg.mode, w.gates, TCC_NODA_MAX);
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
  for (int k = 0; k < TCC_NODA_MAX; ++k) {
    const State* gk = &w.gates[1 + k];
    hipLaunchKernelGGL(tcc_shift_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, w.A, w.Mi, n, D2, w.scal, 0.0,
                       gk);
    launch_gj_inverse(w.Mi, D2, D2, gj, gk, stream);
    hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.Mi, D2, n, d, 0, w.x, w.y, gk);
    hipLaunchKernelGGL(tcc_noda_kernel, dim3(1), dim3(EB), 0, stream, w.x, w.y, n, w.scal, w.gates, k, TCC_NODA_MAX,
                       gk);
  }
  // final inverse just above the converged root: two sweeps for v, two (transposed) for u
  hipLaunchKernelGGL(tcc_shift_kernel, dim3(grid_for(D2 * D2)), dim3(EB), 0, stream, w.A, w.Mi, n, D2, w.scal, 1e-14,
                     g0);
  launch_gj_inverse(w.Mi, D2, D2, gj, g0, stream);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(tcc_gemv_kernel, gv, dim3(EB), 0, stream, w.Mi, D2, n, d, 0, w.x, w.y, g0);
    hipLaunchKernelGGL(tcc_normalize_kernel, dim3(1), dim3(EB), 0, stream, w.y, w.x, n, g0);
  }
  hipLaunchKernelGGL(tcc_init_kernel, dim3(1), dim3(EB), 0, stream, w.uprev, w.u, n, w.scal, g0);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(tcc_gemv_t_partial_kernel, gt, dim3(EB), 0, stream, w.Mi, D2, n, w.u, w.part, g0);
    hipLaunchKernelGGL(tcc_gemv_t_sum_kernel, gts, dim3(EB), 0, stream, w.part, D2, n, nchunks, w.y, g0);
    hipLaunchKernelGGL(tcc_normalize_kernel, dim3(1), dim3(EB), 0, stream, w.y, w.u, n, g0);
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
