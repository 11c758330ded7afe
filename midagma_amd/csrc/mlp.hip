// The DagmaMLP tail for BASELINE config 5 (dims [d, m1, 1]), fused: from the fc1 output
// Z (n x d*m1, nonlinear.py:99-100) through sigmoid, the width-1 LocallyConnected layer and
// its bias (locally_connected.py:55-85, nonlinear.py:101-104) to the squared residual sum the
// log-MSE score takes (nonlinear.py:139-159):
//     S = sigmoid(Z),  Xhat[r, j] = sum_m S[r, j, m] w2[j, m] + b2[j],  ssq = sum (Xhat - X)^2
// and its backward for d(ssq) = g:
//     dXhat = 2 g (Xhat - X),  dZ = dXhat w2 S (1 - S),  dw2[j, m] = sum_r dXhat S,  db2 = sum_r dXhat.
// Four launches replace the ~20 elementwise/reduction kernels PyTorch runs for the same
// forward and backward.  Every Z access is coalesced (consecutive threads on consecutive
// columns c = j m1 + m); sums over rows run in a fixed order (deterministic).
#include <algorithm>

#include "launch.h"

namespace midagma {
namespace {

constexpr int TAIL_ROWS = 32;  // rows per workgroup of the backward (partials per row chunk)

__device__ __forceinline__ double sigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

__device__ __forceinline__ double block_sum256(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// workgroup per row: S w2 staged in LDS (coalesced over the row's d m1 columns), then thread
// j < d sums its m1 terms: R[row, j] = Xhat - X, part[row] = sum_j R^2
__global__ __launch_bounds__(NTHREADS) void mlp_tail_fwd_kernel(const double* __restrict__ Z,
                                                                const double* __restrict__ b1,
                                                                const double* __restrict__ w2,
                                                                const double* __restrict__ b2,
                                                                const double* __restrict__ X, int64_t d, int m1,
                                                                double* __restrict__ R, double* __restrict__ part) {
  extern __shared__ double sw[];  // d m1 products, then the reduction scratch
  const int64_t row = blockIdx.x, dm = d * m1;
  const double* z = Z + row * dm;
  for (int64_t c = threadIdx.x; c < dm; c += NTHREADS) sw[c] = sigmoid(b1 ? z[c] + b1[c] : z[c]) * w2[c];
  __syncthreads();
  double r2 = 0.0;
  for (int64_t j = threadIdx.x; j < d; j += NTHREADS) {
    double acc = 0.0;
    for (int m = 0; m < m1; ++m) acc += sw[j * m1 + m];
    const double r = (acc + b2[j]) - X[row * d + j];
    R[row * d + j] = r;
    r2 += r * r;
  }
  const double t = block_sum256(r2, sw + dm);
  if (threadIdx.x == 0) part[row] = t;
}

// one workgroup: out[0] = sum of the np partials (fixed order)
__global__ __launch_bounds__(NTHREADS) void mlp_sum_kernel(const double* __restrict__ part, int64_t np,
                                                           double* __restrict__ out) {
  __shared__ double red[NTHREADS];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += NTHREADS) a += part[i];
  const double t = block_sum256(a, red);
  if (threadIdx.x == 0) out[0] = t;
}

// grid (column tiles of 256, row chunks of TAIL_ROWS): thread per column c = j m1 + m over
// the chunk's rows: dZ, and the chunk's partials of dw2 (pw[chunk][c]) and db2 (pb[chunk][j])
// The objective's backward for d obj = gobj (mlp_objective_bwd's arithmetic): d obj / d ssq, with
// ssq the fixed-order sum of the forward's row partials (mlp_sum's order), computed by the
// consumer itself instead of a launch of its own.
struct ObjGrad {
  const double* part;  // the forward's row partials (null: g already is d obj / d ssq)
  int64_t np;
  const double* gobj;
  double mu, half_d, inv_n;
};

__device__ __forceinline__ double ssq_from_parts(const double* __restrict__ part, int64_t np, double* red) {
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += NTHREADS) a += part[i];
  return block_sum256(a, red);
}

__device__ __forceinline__ double gssq_of(double gv, double ssq, const ObjGrad& o) {
  const double inner = gv * o.mu;
  return ((inner * o.half_d) / (o.inv_n * ssq)) * o.inv_n;
}

__global__ __launch_bounds__(NTHREADS) void mlp_tail_bwd_kernel(const double* __restrict__ Z,
                                                                const double* __restrict__ b1,
                                                                const double* __restrict__ w2,
                                                                const double* __restrict__ R,
                                                                const double* __restrict__ g, int64_t n, int64_t d,
                                                                int m1, double* __restrict__ dZ,
                                                                double* __restrict__ pw, double* __restrict__ pb,
                                                                double* __restrict__ pz, ObjGrad og) {
  const int64_t dm = d * m1;
  double gs;
  if (og.part) {  // every workgroup reduces the partials (before any thread leaves)
    __shared__ double red[NTHREADS];
    gs = gssq_of(og.gobj[0], ssq_from_parts(og.part, og.np, red), og);
  } else {
    gs = g[0];
  }
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (c >= dm) return;
  const int64_t j = c / m1;
  const int m = (int)(c % m1);
  const double w = w2[c], g2 = 2.0 * gs, bias = b1 ? b1[c] : 0.0;
  const int64_t r0 = (int64_t)blockIdx.y * TAIL_ROWS, r1 = r0 + TAIL_ROWS < n ? r0 + TAIL_ROWS : n;
  double aw = 0.0, ab = 0.0, az = 0.0;
  // rows in groups of 8 with every load of the group issued first (the loop was one dependent
  // load round trip per row); the partial sums keep the row order
  constexpr int U = 8;
  int64_t row = r0;
  for (; row + U <= r1; row += U) {
    double rv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rv[u] = R[(row + u) * d + j];
      zv[u] = Z[(row + u) * dm + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double dxh = g2 * rv[u];
      const double s = sigmoid(b1 ? zv[u] + bias : zv[u]);
      const double dz = dxh * w * (s * (1.0 - s));
      dZ[(row + u) * dm + c] = dz;
      aw += dxh * s;
      ab += dxh;
      az += dz;
    }
  }
  for (; row < r1; ++row) {
    const double dxh = g2 * R[row * d + j];
    const double s = sigmoid(b1 ? Z[row * dm + c] + bias : Z[row * dm + c]);
    const double dz = dxh * w * (s * (1.0 - s));
    dZ[row * dm + c] = dz;
    aw += dxh * s;
    ab += dxh;
    az += dz;
  }
  pw[(int64_t)blockIdx.y * dm + c] = aw;
  if (m == 0) pb[(int64_t)blockIdx.y * d + j] = ab;
  if (pz) pz[(int64_t)blockIdx.y * dm + c] = az;
}

// dw2[c] = sum over chunks of pw[.][c], db2[j] likewise (fixed order)
__global__ __launch_bounds__(NTHREADS) void mlp_tail_dw_kernel(const double* __restrict__ pw,
                                                               const double* __restrict__ pb,
                                                               const double* __restrict__ pz, int64_t nchunk,
                                                               int64_t d, int m1, double* __restrict__ dw2,
                                                               double* __restrict__ db2, double* __restrict__ db1) {
  const int64_t dm = d * m1;
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  // four independent chains (loads in flight), combined in a fixed order
  const double* src;
  int64_t stride;
  double* dst;
  if (c < dm) {
    src = pw + c, stride = dm, dst = dw2 + c;
  } else if (c < dm + d) {
    src = pb + (c - dm), stride = d, dst = db2 + (c - dm);
  } else if (db1 && c < 2 * dm + d) {
    src = pz + (c - dm - d), stride = dm, dst = db1 + (c - dm - d);
  } else {
    return;
  }
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t k = 0;
  for (; k + 4 <= nchunk; k += 4) {
    a0 += src[k * stride];
    a1 += src[(k + 1) * stride];
    a2 += src[(k + 2) * stride];
    a3 += src[(k + 3) * stride];
  }
  for (; k < nchunk; ++k) a0 += src[k * stride];
  *dst = (a0 + a1) + (a2 + a3);
}

}  // namespace

int64_t mlp_tail_scratch(int64_t n, int64_t d, int64_t m1) {
  const int64_t chunks = (n + TAIL_ROWS - 1) / TAIL_ROWS;
  return std::max<int64_t>(n, chunks * (2 * d * m1 + d));
}

void launch_mlp_tail_fwd(const double* Z, const double* b1, const double* w2, const double* b2, const double* X,
                         int64_t n, int64_t d, int m1, double* R, double* part, double* ssq, hipStream_t stream) {
  if (d * m1 > MLP_TAIL_MAX_DM) throw std::invalid_argument("mlp tail: d * m1 above the LDS row stage");
  const size_t lds = (size_t)(d * m1 + NTHREADS) * sizeof(double);
  hipLaunchKernelGGL(mlp_tail_fwd_kernel, dim3((unsigned)n), dim3(NTHREADS), lds, stream, Z, b1, w2, b2, X, d, m1, R,
                     part);
  if (ssq) hipLaunchKernelGGL(mlp_sum_kernel, dim3(1), dim3(NTHREADS), 0, stream, part, n, ssq);
  HIP_TRY(hipGetLastError());
}

void launch_mlp_tail_bwd(const double* Z, const double* b1, const double* w2, const double* R, const double* g,
                         int64_t n, int64_t d, int m1, double* dZ, double* dw2, double* db2, double* db1,
                         double* scratch, hipStream_t stream, const double* part, const double* gobj, double mu,
                         double half_d, double inv_n) {
  const int64_t dm = d * m1, chunks = (n + TAIL_ROWS - 1) / TAIL_ROWS;
  double* pw = scratch;
  double* pb = scratch + chunks * dm;
  double* pz = db1 ? pb + chunks * d : nullptr;
  hipLaunchKernelGGL(mlp_tail_bwd_kernel, dim3((unsigned)((dm + NTHREADS - 1) / NTHREADS), (unsigned)chunks),
                     dim3(NTHREADS), 0, stream, Z, b1, w2, R, g, n, d, m1, dZ, pw, pb, pz,
                     ObjGrad{part, n, gobj, mu, half_d, inv_n});
  const int64_t cols = dm + d + (db1 ? dm : 0);
  hipLaunchKernelGGL(mlp_tail_dw_kernel, dim3((unsigned)((cols + NTHREADS - 1) / NTHREADS)), dim3(NTHREADS), 0,
                     stream, pw, pb, pz, chunks, d, m1, dw2, db2, db1);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma

// ---- the fc1 terms and the scalar objective (nonlinear.py:68-86, 139-159, 198-206) ------
namespace midagma {
namespace {

// thread per (j, i): A[i, j] = sum_m W1[j m1 + m, i]^2 (the reference's sum of fc1_weight**2
// over m, transposed, nonlinear.py:83-84); the workgroup's sum of |W1| -> l1part[wg]
__global__ __launch_bounds__(NTHREADS) void fc1_terms_kernel(const double* __restrict__ W1, int64_t d, int m1,
                                                             double* __restrict__ A, double* __restrict__ l1part) {
  __shared__ double red[NTHREADS];
  const int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  double al = 0.0;
  if (t < d * d) {
    const int64_t j = t / d, i = t % d;
    double acc = 0.0;
    for (int m = 0; m < m1; ++m) {
      const double w = W1[(j * m1 + m) * d + i];
      acc += w * w;
      al += fabs(w);
    }
    A[i * d + j] = acc;
  }
  red[threadIdx.x] = al;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) l1part[blockIdx.x] = red[0];
}

// dW1[j m1 + m, i] = 2 W1 gA[i, j] + gl1[wg(j, i)] sign(W1);  gA = (*gscale) gA when gscale is
// given (the log-det's backward, grad_out * (sI - A)^-T, folded in)
__global__ __launch_bounds__(NTHREADS) void fc1_terms_bwd_kernel(const double* __restrict__ W1, int64_t d, int m1,
                                                                 const double* __restrict__ gA,
                                                                 const double* __restrict__ gscale,
                                                                 const double* __restrict__ gl1,
                                                                 const double* __restrict__ lin, int nlin,
                                                                 double* __restrict__ dW1, const double* gobj,
                                                                 double mu, double lambda1) {
  const int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (t >= d * d) return;
  const int64_t j = t / d, i = t % d, dd = d * m1 * d;
  // gobj (nullable): d obj = gobj, so d h = gobj and d l1part = (gobj mu) lambda1 (mlp_objective_bwd)
  const double ga = gobj ? gobj[0] * gA[i * d + j] : (gscale ? gscale[0] * gA[i * d + j] : gA[i * d + j]);
  const double gl = gobj ? (gobj[0] * mu) * lambda1 : gl1[blockIdx.x];
  for (int m = 0; m < m1; ++m) {
    const int64_t e = (j * m1 + m) * d + i;
    const double w = W1[e];
    const double sg = w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : 0.0);
    double v = ga * (2.0 * w) + gl * sg;
    if (nlin > 0) {  // + the linear layer's weight gradient, summed over its split-K chunks
      double a = lin[e];
      for (int c = 1; c < nlin; ++c) a += lin[c * dd + e];
      v = a + v;
    }
    dW1[e] = v;
  }
}

// the log-det's epilogue in one launch: Mt (d x d, ldm) from the D x D workspace, and
// workgroup 0: h = -(sum of the pivot logs) + d log s (the reference's h_func, nonlinear.py:85-86)
__global__ __launch_bounds__(NTHREADS) void logdet_post_kernel(const double* __restrict__ piv, int64_t d, double dls,
                                                               double* __restrict__ h,
                                                               const double* __restrict__ Ws, int64_t D,
                                                               double* __restrict__ Mt, int64_t ldm) {
  const int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (Mt && t < d * d) {
    const int64_t i = t / d, j = t % d;
    Mt[i * ldm + j] = Ws[i * D + j];
  }
  if (blockIdx.x != 0) return;
  __shared__ double red[NTHREADS];
  double acc = 0.0;
  for (int64_t k = threadIdx.x; k < d; k += NTHREADS) acc += piv[k];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) h[0] = -red[0] + dls;
}

// one workgroup: obj = mu (0.5 d log(1/n ssq) + lambda1 sum(l1part)) + h, the reference's
// association (nonlinear.py:158, 203-204)
__global__ __launch_bounds__(NTHREADS) void mlp_objective_kernel(const double* __restrict__ ssq,
                                                                 const double* __restrict__ l1part, int64_t np,
                                                                 const double* __restrict__ h, double mu,
                                                                 double lambda1, double half_d, double inv_n,
                                                                 double* __restrict__ out,
                                                                 const double* __restrict__ part, int64_t npart,
                                                                 int64_t* __restrict__ counter) {
  __shared__ double red[NTHREADS];
  // part (nullable): ssq as the fixed-order sum of the tail's row partials (mlp_sum's order)
  const double ssq_v = part ? ssq_from_parts(part, npart, red) : ssq[0];
  if (counter && threadIdx.x == 0) *counter += 1;  // the Adam step table's index (one per step)
  double a = 0.0;
  for (int64_t k = threadIdx.x; k < np; k += NTHREADS) a += l1part[k];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double score = half_d * log(inv_n * ssq_v);
    out[0] = mu * (score + lambda1 * red[0]) + h[0];
  }
}

// g = d L / d obj -> d/d ssq, d/d l1part (every entry), d/d h, in autograd's order
__global__ __launch_bounds__(NTHREADS) void mlp_objective_bwd_kernel(const double* __restrict__ g,
                                                                     const double* __restrict__ ssq, int64_t np,
                                                                     double mu, double lambda1, double half_d,
                                                                     double inv_n, double* __restrict__ gssq,
                                                                     double* __restrict__ gl1part,
                                                                     double* __restrict__ gh) {
  const double gv = g[0], inner = gv * mu;
  const double gl1 = inner * lambda1;
  for (int64_t k = threadIdx.x; k < np; k += NTHREADS) gl1part[k] = gl1;
  if (threadIdx.x == 0) {
    gh[0] = gv;
    gssq[0] = ((inner * half_d) / (inv_n * ssq[0])) * inv_n;
  }
}

}  // namespace

int64_t fc1_terms_parts(int64_t d) { return (d * d + NTHREADS - 1) / NTHREADS; }

void launch_fc1_terms(const double* W1, int64_t d, int m1, double* A, double* l1part, hipStream_t stream) {
  hipLaunchKernelGGL(fc1_terms_kernel, dim3((unsigned)fc1_terms_parts(d)), dim3(NTHREADS), 0, stream, W1, d, m1, A,
                     l1part);
  HIP_TRY(hipGetLastError());
}

void launch_fc1_terms_bwd(const double* W1, int64_t d, int m1, const double* gA, const double* gscale,
                          const double* gl1part, const double* lin, int nlin, double* dW1, hipStream_t stream,
                          const double* gobj, double mu, double lambda1) {
  hipLaunchKernelGGL(fc1_terms_bwd_kernel, dim3((unsigned)fc1_terms_parts(d)), dim3(NTHREADS), 0, stream, W1, d, m1,
                     gA, gscale, gl1part, lin, nlin, dW1, gobj, mu, lambda1);
  HIP_TRY(hipGetLastError());
}

void launch_logdet_post(const double* piv, int64_t d, double dls, double* h, const double* Ws, int64_t D, double* Mt,
                        int64_t ldm, hipStream_t stream) {
  const int64_t blocks = std::max<int64_t>(1, (d * d + NTHREADS - 1) / NTHREADS);
  hipLaunchKernelGGL(logdet_post_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, piv, d, dls, h, Ws, D, Mt,
                     ldm);
  HIP_TRY(hipGetLastError());
}

void launch_mlp_objective(const double* ssq, const double* l1part, int64_t np, const double* h, double mu,
                          double lambda1, double half_d, double inv_n, double* out, hipStream_t stream,
                          const double* part, int64_t npart, int64_t* counter) {
  hipLaunchKernelGGL(mlp_objective_kernel, dim3(1), dim3(NTHREADS), 0, stream, ssq, l1part, np, h, mu, lambda1, half_d,
                     inv_n, out, part, npart, counter);
  HIP_TRY(hipGetLastError());
}

void launch_mlp_objective_bwd(const double* g, const double* ssq, int64_t np, double mu, double lambda1, double half_d,
                              double inv_n, double* gssq, double* gl1part, double* gh, hipStream_t stream) {
  hipLaunchKernelGGL(mlp_objective_bwd_kernel, dim3(1), dim3(NTHREADS), 0, stream, g, ssq, np, mu, lambda1, half_d,
                     inv_n, gssq, gl1part, gh);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma

// ---- the h log-det's warm-started fast path (DagmaNonlinear.minimize, BASELINE config 5) -------
// Between two Adam steps fc1 moves by ~lr, so (sI - A)^-T of the last two steps is a warm start
// for this one: the product-form series of the blocked inverse (launch_series, blockinv.hip) on
// the B x B identity-padded (sI - A)^T replaces the 32-block Gauss-Jordan's prologue and block
// steps.  The log-det itself is needed only where the caller reads it (the checkpoint steps,
// nonlinear.py:214-217 via the objective) and for the h < 0 exit (nonlinear.py:206-208): an
// entrywise nonnegative inverse of the Z-matrix sI - A (A = sum fc1^2 >= 0) proves it a nonsingular
// M-matrix, where h = sum_k tr((A/s)^k)/k >= 0 and the exit cannot fire, so such a step keeps the
// last exactly computed h.  Every other step -- no convergence, a negative or non-finite entry,
// no warm start yet (the first step of a call) -- runs the Gauss-Jordan chain, gated on the
// device, and takes its pivots' h, as do the caller's exact (checkpoint) steps.
namespace midagma {
namespace {

// (sI - A)^T into the B x B S (identity padding); one workgroup also opens the step: the
// step index (the warm-start ring's parity) and the Gauss-Jordan gate reset to "skip".
__global__ __launch_bounds__(NTHREADS) void ldfast_begin_kernel(const double* __restrict__ A, int64_t lda, int64_t d,
                                                                double s, double* __restrict__ S, int B,
                                                                State* __restrict__ st, State* __restrict__ gjst,
                                                                int build) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->slots += 1;
    gjst->status = ST_DONE;
  }
  if (!build) return;
  const int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (e >= (int64_t)B * B) return;
  const int64_t r = e / B, c = e % B;  // S[r][c] = (sI - A)^T[r][c] = s delta - A[c][r]
  double v;
  if (r < d && c < d)
    v = (r == c ? s : 0.0) - A[c * lda + r];
  else
    v = (r == c) ? 1.0 : 0.0;
  S[e] = v;
}

// The series' inverse P (B x B, converged: *done != 0) is (sI - A)^-T: Mt (d x d) from it, and
// the Gauss-Jordan gate opened (gjst->status = ST_RUNNING) when it did not converge or is not
// entrywise >= 0 and finite on the d x d block.
__global__ __launch_bounds__(NTHREADS) void ldfast_certify_kernel(const double* __restrict__ P, int B, int64_t d,
                                                                  double* __restrict__ Mt, int64_t ldm,
                                                                  const State* __restrict__ st,
                                                                  const int* __restrict__ done,
                                                                  State* __restrict__ gjst) {
  const int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  int bad = 0;
  if (e < d * d) {
    const int64_t i = e / d, j = e % d;
    const double v = P[i * B + j];
    Mt[i * ldm + j] = v;
    bad = !(v >= 0.0) || !isfinite(v);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (st->status != ST_RUNNING || *done == 0)) bad = 1;
  if (__syncthreads_or(bad) && threadIdx.x == 0)
    __hip_atomic_store(&gjst->status, (int32_t)ST_RUNNING, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The step's end: if the Gauss-Jordan chain ran (exact step, or the gate opened), h from its
// pivots (logdet_post's sum, bit for bit) and Mt from its workspace, else h = the last exact h;
// the step's inverse into the warm-start ring (slot parity of st->slots); one workgroup then
// advances the ring's state for the next step.
__global__ __launch_bounds__(NTHREADS) void ldfast_post_kernel(const double* __restrict__ piv, int64_t d, double dls,
                                                               double* __restrict__ h, const double* __restrict__ Wgj,
                                                               int64_t Dgj, double* __restrict__ Mt, int64_t ldm,
                                                               const double* __restrict__ P, int B,
                                                               double* __restrict__ ring0, double* __restrict__ ring1,
                                                               State* __restrict__ st, const State* __restrict__ gjst,
                                                               double* __restrict__ hlast, int exact) {
  const bool ran = exact || gjst->status == ST_RUNNING;
  const int64_t slot = st->slots;
  double* dst = (slot & 1) ? ring1 : ring0;
  const int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  if (e < (int64_t)B * B) {  // the ring (B = 0: no fast path, no ring)
    const int64_t i = e / B, j = e % B;
    dst[e] = ran ? ((i < Dgj && j < Dgj) ? Wgj[i * Dgj + j] : (i == j ? 1.0 : 0.0)) : P[e];
  }
  if (ran && e < d * d) {
    const int64_t i = e / d, j = e % d;
    Mt[i * ldm + j] = Wgj[i * Dgj + j];
  }
  if (blockIdx.x != 0) return;
  __shared__ double red[NTHREADS];
  double acc = 0.0;
  if (ran)
    for (int64_t k = threadIdx.x; k < d; k += NTHREADS) acc += piv[k];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s2 = NTHREADS / 2; s2 > 0; s2 >>= 1) {
    if ((int)threadIdx.x < s2) red[threadIdx.x] += red[threadIdx.x + s2];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double hv = ran ? -red[0] + dls : hlast[0];
    h[0] = hv;
    if (ran) hlast[0] = hv;
    st->warm_run = st->warm_run < 2 ? st->warm_run + 1 : 2;
    st->ckpt_pending = 0;
    st->status = ST_RUNNING;
    st->iter += 1;                // diagnostics (midagma_ldfast_stats): steps,
    if (ran) st->halvings += 1;   // and those that ran the Gauss-Jordan chain
  }
}

}  // namespace

void launch_ldfast_begin(const double* A, int64_t lda, int64_t d, double s, double* S, int B, State* st, State* gjst,
                         bool build, hipStream_t stream) {
  const unsigned blocks = build ? (unsigned)(((int64_t)B * B + NTHREADS - 1) / NTHREADS) : 1u;
  hipLaunchKernelGGL(ldfast_begin_kernel, dim3(blocks), dim3(NTHREADS), 0, stream, A, lda, d, s, S, B, st, gjst,
                     build ? 1 : 0);
  HIP_TRY(hipGetLastError());
}

void launch_ldfast_certify(const double* P, int B, int64_t d, double* Mt, int64_t ldm, const State* st,
                           const int* done, State* gjst, hipStream_t stream) {
  const int64_t blocks = std::max<int64_t>(1, (d * d + NTHREADS - 1) / NTHREADS);
  hipLaunchKernelGGL(ldfast_certify_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, P, B, d, Mt, ldm, st,
                     done, gjst);
  HIP_TRY(hipGetLastError());
}

void launch_ldfast_post(const double* piv, int64_t d, double dls, double* h, const double* Wgj, int64_t Dgj, double* Mt,
                        int64_t ldm, const double* P, int B, double* ring0, double* ring1, State* st,
                        const State* gjst, double* hlast, bool exact, hipStream_t stream) {
  const unsigned blocks = (unsigned)((std::max<int64_t>((int64_t)B * B, d * d) + NTHREADS - 1) / NTHREADS);
  hipLaunchKernelGGL(ldfast_post_kernel, dim3(blocks), dim3(NTHREADS), 0, stream, piv, d, dls, h, Wgj, Dgj, Mt, ldm,
                     P, B, ring0, ring1, st, gjst, hlast, exact ? 1 : 0);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
