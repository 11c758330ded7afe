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
#include <stdexcept>
#include <utility>

#include "launch.h"
#include "mfma64.h"

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
  // (thread j < d: its b2 and X entries loaded ahead of the staging, not after its barrier)
  const int64_t j0 = threadIdx.x;
  const double b2j = j0 < d ? b2[j0] : 0.0, xj = j0 < d ? X[row * d + j0] : 0.0;
  // the row's operands in groups of SU per thread, every load of a group issued before its
  // arithmetic (a loop of load-then-use waited out one memory round trip per column)
  constexpr int SU = 8;
  for (int64_t c0 = threadIdx.x; c0 < dm; c0 += SU * NTHREADS) {
    double zv[SU], bv[SU], wv[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int64_t c = c0 + u * NTHREADS;
      const bool ok = c < dm;
      zv[u] = ok ? z[c] : 0.0;
      bv[u] = ok && b1 ? b1[c] : 0.0;
      wv[u] = ok ? w2[c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int64_t c = c0 + u * NTHREADS;
      if (c < dm) sw[c] = sigmoid(b1 ? zv[u] + bv[u] : zv[u]) * wv[u];
    }
  }
  __syncthreads();
  double r2 = 0.0;
  for (int64_t j = threadIdx.x; j < d; j += NTHREADS) {
    double acc = 0.0;
    for (int m = 0; m < m1; ++m) acc += sw[j * m1 + m];
    const double r = (acc + (j == j0 ? b2j : b2[j])) - (j == j0 ? xj : X[row * d + j]);
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
  const int64_t c = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  const bool live = c < dm;
  const int64_t j = live ? c / m1 : 0;
  const int m = live ? (int)(c % m1) : 0;
  const int64_t r0 = (int64_t)blockIdx.y * TAIL_ROWS, r1 = r0 + TAIL_ROWS < n ? r0 + TAIL_ROWS : n;
  // a whole chunk's R and Z loads are issued first, ahead of the objective's reduction below and
  // of any arithmetic (in groups of 8 rows the loop waited out four memory round trips)
  const bool full = r1 - r0 == TAIL_ROWS;
  double rv[TAIL_ROWS], zv[TAIL_ROWS];
  double w = 0.0, bias = 0.0;
  if (live) {
    w = w2[c];
    bias = b1 ? b1[c] : 0.0;
    if (full)
#pragma unroll
      for (int u = 0; u < TAIL_ROWS; ++u) {
        rv[u] = R[(r0 + u) * d + j];
        zv[u] = Z[(r0 + u) * dm + c];
      }
  }
  double gs;
  if (og.part) {  // every workgroup reduces the partials (before any thread leaves)
    __shared__ double red[NTHREADS];
    gs = gssq_of(og.gobj[0], ssq_from_parts(og.part, og.np, red), og);
  } else {
    gs = g[0];
  }
  if (!live) return;
  const double g2 = 2.0 * gs;
  double aw = 0.0, ab = 0.0, az = 0.0;
  if (full) {  // (the partial sums keep the row order)
#pragma unroll
    for (int u = 0; u < TAIL_ROWS; ++u) {
      const double dxh = g2 * rv[u];
      const double s = sigmoid(b1 ? zv[u] + bias : zv[u]);
      const double dz = dxh * w * (s * (1.0 - s));
      dZ[(r0 + u) * dm + c] = dz;
      aw += dxh * s;
      ab += dxh;
      az += dz;
    }
  } else {
    for (int64_t row = r0; row < r1; ++row) {
      const double dxh = g2 * R[row * d + j];
      const double s = sigmoid(b1 ? Z[row * dm + c] + bias : Z[row * dm + c]);
      const double dz = dxh * w * (s * (1.0 - s));
      dZ[row * dm + c] = dz;
      aw += dxh * s;
      ab += dxh;
      az += dz;
    }
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
                         double half_d, double inv_n, bool sums) {
  const int64_t dm = d * m1, chunks = (n + TAIL_ROWS - 1) / TAIL_ROWS;
  double* pw = scratch;
  double* pb = scratch + chunks * dm;
  // (sums == false: the partials only, b1's too, for launch_mlp_step to sum)
  double* pz = db1 || (!sums && b1) ? pb + chunks * d : nullptr;
  hipLaunchKernelGGL(mlp_tail_bwd_kernel, dim3((unsigned)((dm + NTHREADS - 1) / NTHREADS), (unsigned)chunks),
                     dim3(NTHREADS), 0, stream, Z, b1, w2, R, g, n, d, m1, dZ, pw, pb, pz,
                     ObjGrad{part, n, gobj, mu, half_d, inv_n});
  if (!sums) {
    HIP_TRY(hipGetLastError());
    return;
  }
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

// fc1_terms_bwd_kernel's arithmetic with a thread per element of dW1 (c = j m1 + m, i): the
// linear layer's nlin split-K slices are read in parallel by d m1 d threads instead of in a loop
// over m by d d threads (config 5: 8 slices of 3.2 MB, 25 -> ~7 us)
__global__ __launch_bounds__(NTHREADS) void fc1_terms_bwd_elem_kernel(const double* __restrict__ W1, int64_t d, int m1,
                                                                      const double* __restrict__ gA,
                                                                      const double* __restrict__ gscale,
                                                                      const double* __restrict__ gl1,
                                                                      const double* __restrict__ lin, int nlin,
                                                                      double* __restrict__ dW1, const double* gobj,
                                                                      double mu, double lambda1) {
  const int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x, dd = d * m1 * d;
  if (e >= dd) return;
  const int64_t c = e / d, i = e % d, j = c / m1;
  const double ga = gobj ? gobj[0] * gA[i * d + j] : (gscale ? gscale[0] * gA[i * d + j] : gA[i * d + j]);
  const double gl = gobj ? (gobj[0] * mu) * lambda1 : gl1[(j * d + i) / NTHREADS];
  const double w = W1[e];
  const double sg = w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : 0.0);
  double v = ga * (2.0 * w) + gl * sg;
  if (nlin > 0) {
    double a = lin[e];
    for (int q = 1; q < nlin; ++q) a += lin[q * dd + e];
    v = a + v;
  }
  dW1[e] = v;
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
    if (ssq != nullptr && gssq != nullptr) gssq[0] = ((inner * half_d) / (inv_n * ssq[0])) * inv_n;
  }
}

// One torch-Adam step of a [d, m1, 1] DagmaMLP's four parameters in one launch, closing the step
// (DagmaNonlinear.minimize, nonlinear.py:198-236; BASELINE config 5).  It does the work of four
// launches with their arithmetic unchanged:
//   - mlp_tail_dw: the gradients of fc2's weight and bias and fc1's bias from the tail backward's
//     chunk partials;
//   - fc1_terms_bwd_elem: fc1's weight gradient;
//   - adam_gated_table_multi: the Adam update of all four tensors;
//   - the next step's fc1_terms: A = sum_m fc1^2 and the |fc1| partials of the updated weights.
// Workgroups [0, nA) hold the (j, i) pairs of fc1_terms' grid (so the l1 partials are the same sums
// in the same order); each thread walks its m1 weights.  The rest hold b1, w2 and b2 elementwise.
// Gated off (*gate < 0) nothing moves, and A and l1part come from the weights as they are.
struct MlpStepArgs {
  double *W1, *b1, *w2, *b2;
  double *mW1, *vW1, *mb1, *vb1, *mw2, *vw2, *mb2, *vb2;
  int64_t d, m1, nchunk;
  const double *gA, *gobj;
  double mu, lambda1;
  const double* lin;
  int nlin, nA;
  const double *pw, *pb, *pz;
  const double* table;
  const int64_t* counter;
  double w1, beta2, c2, eps, wd;
  const double* gate;
  double *A, *l1part;
};

// adam_gated_table_multi_kernel's element update
__device__ __forceinline__ double adam_elem(double pi, double& m, double& v, double gi, const MlpStepArgs& a,
                                            double step_size, double bc2_sqrt) {
  if (a.wd != 0.0) gi = gi + a.wd * pi;
  const double mi = m + a.w1 * (gi - m);
  const double vi = v * a.beta2 + a.c2 * gi * gi;
  const double denom = sqrt(vi) / bc2_sqrt + a.eps;
  m = mi;
  v = vi;
  return pi + (-step_size) * mi / denom;
}

// mlp_tail_dw_kernel's fixed-order sum of the chunk partials of one column (up to 32 chunks: every
// load first, then the same four chains)
__device__ __forceinline__ double chunk_sum(const double* __restrict__ src, int64_t stride, int64_t nchunk) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  constexpr int KU = 32;
  if (nchunk <= KU) {
    double x[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) x[u] = u < nchunk ? src[u * stride] : 0.0;
#pragma unroll
    for (int u = 0; u + 4 <= KU; u += 4)
      if (u + 4 <= nchunk) {
        a0 += x[u];
        a1 += x[u + 1];
        a2 += x[u + 2];
        a3 += x[u + 3];
      }
#pragma unroll
    for (int u = 0; u < KU; ++u)
      if (u >= nchunk / 4 * 4 && u < nchunk) a0 += x[u];
    return (a0 + a1) + (a2 + a3);
  }
  int64_t k = 0;
  for (; k + 4 <= nchunk; k += 4) {
    a0 += src[k * stride];
    a1 += src[(k + 1) * stride];
    a2 += src[(k + 2) * stride];
    a3 += src[(k + 3) * stride];
  }
  for (; k < nchunk; ++k) a0 += src[k * stride];
  return (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(NTHREADS) void mlp_step_kernel(MlpStepArgs a) {
  __shared__ double red[NTHREADS];
  const bool go = !(a.gate && !(*a.gate >= 0.0));
  double step_size = 0.0, bc2_sqrt = 1.0;
  if (go) {
    const int64_t t = *a.counter;
    step_size = a.table[2 * t];
    bc2_sqrt = a.table[2 * t + 1];
  }
  const int64_t d = a.d, m1 = a.m1, dm = d * m1;
  if ((int)blockIdx.x < a.nA) {
    const int64_t tt = (int64_t)blockIdx.x * NTHREADS + threadIdx.x, dd = dm * d;
    double al = 0.0;
    if (tt < d * d) {
      const int64_t j = tt / d, i = tt % d;
      const double g0 = a.gobj[0];
      const double ga = g0 * a.gA[i * d + j];
      const double gl = (g0 * a.mu) * a.lambda1;
      double acc = 0.0;
      constexpr int MU = 16, LU = 4;
      if (m1 <= MU && a.nlin <= LU) {
        // (every load of the thread's m1 weights first: a loop of load, update, store waited out
        // one memory round trip per weight)
        double wv[MU], mv[MU], vv[MU], lv[LU][MU];
#pragma unroll
        for (int m = 0; m < MU; ++m) {
          const int64_t e = (j * m1 + m) * d + i;
          const bool ok = m < m1;
          wv[m] = ok ? a.W1[e] : 0.0;
          mv[m] = ok && go ? a.mW1[e] : 0.0;
          vv[m] = ok && go ? a.vW1[e] : 0.0;
#pragma unroll
          for (int q = 0; q < LU; ++q) lv[q][m] = ok && go && q < a.nlin ? a.lin[q * dd + e] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < MU; ++m) {
          if (m >= m1) break;
          const int64_t e = (j * m1 + m) * d + i;
          const double w = wv[m];
          double pn = w;
          if (go) {
            const double sg = w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : 0.0);
            double g = ga * (2.0 * w) + gl * sg;
            if (a.nlin > 0) {
              double s = lv[0][m];
#pragma unroll
              for (int q = 1; q < LU; ++q)
                if (q < a.nlin) s += lv[q][m];
              g = s + g;
            }
            double mm = mv[m], vq = vv[m];
            pn = adam_elem(w, mm, vq, g, a, step_size, bc2_sqrt);
            a.mW1[e] = mm;
            a.vW1[e] = vq;
            a.W1[e] = pn;
          }
          acc += pn * pn;
          al += fabs(pn);
        }
      } else {
        for (int64_t m = 0; m < m1; ++m) {
          const int64_t e = (j * m1 + m) * d + i;
          const double w = a.W1[e];
          double pn = w;
          if (go) {
            const double sg = w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : 0.0);
            double g = ga * (2.0 * w) + gl * sg;
            if (a.nlin > 0) {
              double s = a.lin[e];
              for (int q = 1; q < a.nlin; ++q) s += a.lin[q * dd + e];
              g = s + g;
            }
            double mm = a.mW1[e], vq = a.vW1[e];
            pn = adam_elem(w, mm, vq, g, a, step_size, bc2_sqrt);
            a.mW1[e] = mm;
            a.vW1[e] = vq;
            a.W1[e] = pn;
          }
          acc += pn * pn;
          al += fabs(pn);
        }
      }
      a.A[i * d + j] = acc;
    }
    red[threadIdx.x] = al;
    __syncthreads();
    for (int s = NTHREADS / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) a.l1part[blockIdx.x] = red[0];
    return;
  }
  if (!go) return;
  // b1 (the partials pz), w2 (pw), b2 (pb): mlp_tail_dw's sums, then the Adam update
  const int64_t c = (int64_t)(blockIdx.x - a.nA) * NTHREADS + threadIdx.x;
  double *p, *m, *v;
  double g;
  int64_t k;
  if (c < dm) {
    k = c, p = a.b1, m = a.mb1, v = a.vb1;
    g = chunk_sum(a.pz + k, dm, a.nchunk);
  } else if (c < 2 * dm) {
    k = c - dm, p = a.w2, m = a.mw2, v = a.vw2;
    g = chunk_sum(a.pw + k, dm, a.nchunk);
  } else if (c < 2 * dm + d) {
    k = c - 2 * dm, p = a.b2, m = a.mb2, v = a.vb2;
    g = chunk_sum(a.pb + k, d, a.nchunk);
  } else {
    return;
  }
  double mm = m[k], vv = v[k];
  p[k] = adam_elem(p[k], mm, vv, g, a, step_size, bc2_sqrt);
  m[k] = mm;
  v[k] = vv;
}

}  // namespace

int64_t fc1_terms_parts(int64_t d) { return (d * d + NTHREADS - 1) / NTHREADS; }

void launch_fc1_terms(const double* W1, int64_t d, int m1, double* A, double* l1part, hipStream_t stream) {
  hipLaunchKernelGGL(fc1_terms_kernel, dim3((unsigned)fc1_terms_parts(d)), dim3(NTHREADS), 0, stream, W1, d, m1, A,
                     l1part);
  HIP_TRY(hipGetLastError());
}

void launch_mlp_step(const MlpStepPtrs& p, int64_t n, int64_t d, int m1, const double* gA, const double* gobj,
                     double mu, double lambda1, const double* lin, int nlin, const double* scratch,
                     const double* table, const int64_t* counter, double w1, double beta2, double c2, double eps,
                     double wd, const double* gate, double* A, double* l1part, hipStream_t stream) {
  const int64_t dm = d * m1, nchunk = (n + TAIL_ROWS - 1) / TAIL_ROWS;
  MlpStepArgs a{};
  a.W1 = p.W1, a.b1 = p.b1, a.w2 = p.w2, a.b2 = p.b2;
  a.mW1 = p.mW1, a.vW1 = p.vW1, a.mb1 = p.mb1, a.vb1 = p.vb1, a.mw2 = p.mw2, a.vw2 = p.vw2, a.mb2 = p.mb2,
  a.vb2 = p.vb2;
  a.d = d, a.m1 = m1, a.nchunk = nchunk;
  a.gA = gA, a.gobj = gobj, a.mu = mu, a.lambda1 = lambda1, a.lin = lin, a.nlin = nlin;
  a.nA = (int)fc1_terms_parts(d);
  // the tail backward's partials (launch_mlp_tail_bwd's layout: pw, pb, pz)
  a.pw = scratch, a.pb = scratch + nchunk * dm, a.pz = a.pb + nchunk * d;
  a.table = table, a.counter = counter, a.w1 = w1, a.beta2 = beta2, a.c2 = c2, a.eps = eps, a.wd = wd;
  a.gate = gate, a.A = A, a.l1part = l1part;
  const int64_t nsmall = (2 * dm + d + NTHREADS - 1) / NTHREADS;
  hipLaunchKernelGGL(mlp_step_kernel, dim3((unsigned)(a.nA + nsmall)), dim3(NTHREADS), 0, stream, a);
  HIP_TRY(hipGetLastError());
}

void launch_fc1_terms_bwd(const double* W1, int64_t d, int m1, const double* gA, const double* gscale,
                          const double* gl1part, const double* lin, int nlin, double* dW1, hipStream_t stream,
                          const double* gobj, double mu, double lambda1) {
  if (nlin > 1) {
    const int64_t dd = d * m1 * d;
    hipLaunchKernelGGL(fc1_terms_bwd_elem_kernel, dim3((unsigned)((dd + NTHREADS - 1) / NTHREADS)), dim3(NTHREADS), 0,
                       stream, W1, d, m1, gA, gscale, gl1part, lin, nlin, dW1, gobj, mu, lambda1);
  } else {
    hipLaunchKernelGGL(fc1_terms_bwd_kernel, dim3((unsigned)fc1_terms_parts(d)), dim3(NTHREADS), 0, stream, W1, d, m1,
                       gA, gscale, gl1part, lin, nlin, dW1, gobj, mu, lambda1);
  }
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

// An exact step's opening: the step index (the warm-start ring's parity) and the Gauss-Jordan
// gate reset to "skip".  (A fast step opens in its residual launch, ldfast_resid_kernel, and
// counts the step at its end.)
__global__ __launch_bounds__(64) void ldfast_begin_kernel(State* __restrict__ st, State* __restrict__ gjst) {
  if (threadIdx.x == 0) {
    st->slots += 1;
    gjst->status = ST_DONE;
  }
}

// The series' inverse P (B x B, converged: *done != 0) is (sI - A)^-T: Mt (d x d) and the step's
// warm-start ring slot (parity of st->slots + 1: the end launch counts the step) from it, and the
// Gauss-Jordan gate opened (gjst->status = ST_RUNNING) when it did not converge or is not
// entrywise >= 0 and finite on the d x d block (the gated chain's end then overwrites Mt and the
// slot).  The slot's old contents, slot k-2's inverse, were last read by this step's residual.
__global__ __launch_bounds__(NTHREADS) void ldfast_certify_kernel(const double* __restrict__ P, int B, int64_t d,
                                                                  double* __restrict__ Mt, int64_t ldm,
                                                                  const State* __restrict__ st,
                                                                  const int* __restrict__ done,
                                                                  State* __restrict__ gjst, double* __restrict__ ring0,
                                                                  double* __restrict__ ring1) {
  const int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  double* dst = ((st->slots + 1) & 1) ? ring1 : ring0;
  int bad = 0;
  if (e < (int64_t)B * B) {
    const int64_t i = e / B, j = e % B;
    const double v = P[e];
    dst[e] = v;
    if (i < d && j < d) {
      Mt[i * ldm + j] = v;
      bad = !(v >= 0.0) || !isfinite(v);
    }
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

void launch_ldfast_begin(State* st, State* gjst, hipStream_t stream) {
  hipLaunchKernelGGL(ldfast_begin_kernel, dim3(1), dim3(64), 0, stream, st, gjst);
  HIP_TRY(hipGetLastError());
}

void launch_ldfast_certify(const double* P, int B, int64_t d, double* Mt, int64_t ldm, const State* st,
                           const int* done, State* gjst, double* ring0, double* ring1, hipStream_t stream) {
  if (d > B) throw std::invalid_argument("ldfast_certify: d exceeds the series block");
  const int64_t blocks = std::max<int64_t>(1, ((int64_t)B * B + NTHREADS - 1) / NTHREADS);
  hipLaunchKernelGGL(ldfast_certify_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, P, B, d, Mt, ldm, st,
                     done, gjst, ring0, ring1);
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

#ifdef MIDAGMA_EXPERIMENTS
// ---- fc1 and the tail fused on the f64 MFMA (experiments build; BASELINE config 5) -----------
// Forward: Z = X W1^T (nonlinear.py:99-100, fc1 without its bias) in 64 x TC tiles, TC = 16 NCB a
// multiple of m1 so that no node's m1 hidden units straddle two tiles; the epilogue stores Z (the
// backward's operand) and runs the tail forward on the tile (mlp_tail_fwd_kernel's arithmetic):
// S w2 = sigmoid(Z + b1) w2 summed over each node's m1 units, R = (that + b2) - X, and one partial
// of sum R^2 per workgroup.  It replaces rocBLAS's Z GEMM, the Z round trip through HBM and the
// tail forward launch.
// Measured at config 5 and rejected: 136.8 vs 139.7 us a step with the
// log-det in sequence, but 145 vs 123 us with the log-det on its side stream, whose kernels these
// launches' LDS / VGPR footprint keeps off the CUs.
// Backward: lin_z = dZ^T X over the z-th 128-row split, with dZ = 2 gs R w2 S (1 - S)
// (mlp_tail_bwd_kernel's arithmetic) formed while the operand chunk is staged in LDS, never
// stored; the staging threads also keep the dw2 / db2 / db1 partials of their column.  It
// replaces the tail backward, the dZ round trip and the split-K bmm.
namespace midagma {
namespace {

// development probe only (tools/micro/mlp_micro.hip): bit 0 skips the forward's MFMAs, bit 1 its
// epilogue; bit 2 the backward's MFMAs; bit 4 the forward's S stores, bit 5 its node sums
#ifndef MLP_FUSED_PROBE
#define MLP_FUSED_PROBE 0
#endif
constexpr int FK = 32;      // k depth of one LDS chunk
constexpr int FS = FK + 2;  // image row stride: 34 = 2 mod 32, conflict-free ds_read_b64 fragments
constexpr int FBR = 128;    // rows per split of the fused backward
constexpr int FFK = 40;     // the forward's k chunk (d = 200: five, no zero steps)
constexpr int FFS = 66;     // its image stride (2 mod 32)

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NCB>
__global__ __launch_bounds__(NTHREADS, 2) void mlp_fc1_tail_fwd_kernel(
    const double* __restrict__ X, const double* __restrict__ W1, const double* __restrict__ b1,
    const double* __restrict__ w2, const double* __restrict__ b2, int64_t n, int64_t d, int m1,
    double* __restrict__ S, double* __restrict__ R, double* __restrict__ part) {
  constexpr int TC = 16 * NCB;
  constexpr int NOPS = (64 + TC) * FFS, NSTG = 4 * 16 * (TC + 1);
  // at least 56 KB: at most two workgroups per CU (three would share a SIMD's matrix pipe
  // three ways on some CUs while others idle)
  constexpr int NL = NOPS > NSTG ? NOPS : NSTG, NCAP = 7 * 1024;
  __shared__ __attribute__((aligned(16))) double lds[NL > NCAP ? NL : NCAP];
  __shared__ double red[4];
  double* As = lds;             // [64 rows][FFS]: X
  double* Bs = lds + 64 * FFS;  // [TC columns][FFS]: W1 (op(B) = W1^T read [n][k])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int64_t dm = d * m1, row0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * TC;
  constexpr int XA = (64 * FFK + NTHREADS - 1) / NTHREADS, XB = (TC * FFK + NTHREADS - 1) / NTHREADS;
  double xa[XA], xb[XB];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int it = 0; it < XA; ++it) {  // consecutive threads on consecutive k: 256-B row runs
      const int e = it * NTHREADS + tid, rr = e / FFK, kk = e % FFK;
      const int64_t gr = row0 + rr, gk = k0 + kk;
      xa[it] = (rr < 64 && gr < n && gk < d) ? X[gr * d + gk] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < XB; ++it) {
      const int e = it * NTHREADS + tid, cc = e / FFK, kk = e % FFK;
      const int64_t gc = c0 + cc, gk = k0 + kk;
      xb[it] = (cc < TC && gc < dm && gk < d) ? W1[gc * d + gk] : 0.0;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int it = 0; it < XA; ++it) {
      const int e = it * NTHREADS + tid;
      if (e < 64 * FFK) As[(e / FFK) * FFS + e % FFK] = xa[it];
    }
#pragma unroll
    for (int it = 0; it < XB; ++it) {
      const int e = it * NTHREADS + tid;
      if (e < TC * FFK) Bs[(e / FFK) * FFS + e % FFK] = xb[it];
    }
  };
  dbl4 acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = dbl4{0.0, 0.0, 0.0, 0.0};
  // the epilogue's per-column operands, loaded up front (a load per element there left every
  // sigmoid waiting on its own round trip)
  double eb[NCB], ew[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int64_t gc = c0 + 16 * cb + (lane & 15);
    eb[cb] = (gc < dm && b1) ? b1[gc] : 0.0;
    ew[cb] = gc < dm ? w2[gc] : 0.0;
  }
  load(0);
  for (int64_t k0 = 0; k0 < d; k0 += FFK) {
    stage();
    __syncthreads();
    if (k0 + FFK < d) load(k0 + FFK);  // the next chunk's loads fly under this chunk's MFMAs
    // k steps of this chunk that hold any k < d (d = 200: five full chunks of 40)
    const int steps = (int)((d - k0 < FFK ? d - k0 : FFK) + 3) / 4;
#pragma unroll 2
    for (int s = 0; s < ((MLP_FUSED_PROBE & 1) ? 0 : steps); ++s) {
      const double a = As[(16 * w + r) * FFS + 4 * s + kq];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const double b = Bs[(16 * cb + r) * FFS + 4 * s + kq];
        acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[cb], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (MLP_FUSED_PROBE & 2) {
    double a = 0.0;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) a += (acc[cb][0] + acc[cb][1]) + (acc[cb][2] + acc[cb][3]);
    if (a == 12345.0) part[0] = a;
    return;
  }
  // epilogue: S, then S w2 per wave through LDS (the operand images are dead)
  double* sg = lds + w * 16 * (TC + 1);
  const int64_t rw = row0 + 16 * w;
  // every sigmoid first (independent chains the scheduler interleaves: two waves per SIMD do not
  // hide one chain's latency), then the stores
  double sv[NCB][4];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int t = 0; t < 4; ++t) sv[cb][t] = sigmoid(b1 ? acc[cb][t] + eb[cb] : acc[cb][t]);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int rl = acc_row(lane, t), cl = 16 * cb + acc_col(lane);
      const int64_t gr = rw + rl, gc = c0 + cl;
      if (!(MLP_FUSED_PROBE & 16) && gr < n && gc < dm) S[gr * dm + gc] = sv[cb][t];
      sg[rl * (TC + 1) + cl] = gc < dm ? sv[cb][t] * ew[cb] : 0.0;
    }
  __syncthreads();
  if (MLP_FUSED_PROBE & 32) {
    if (tid == 0) part[0] = sg[lane];
    return;
  }
  const int nn = TC / m1;
  const int64_t j0 = c0 / m1;
  double r2 = 0.0;
  for (int e = lane; e < 16 * nn; e += 64) {
    const int rl = e / nn, q = e % nn;
    const int64_t gr = rw + rl, j = j0 + q;
    if (gr < n && j < d) {
      double acc1 = 0.0;
      for (int m = 0; m < m1; ++m) acc1 += sg[rl * (TC + 1) + q * m1 + m];
      const double rv = (acc1 + b2[j]) - X[gr * d + j];
      R[gr * d + j] = rv;
      r2 += rv * rv;
    }
  }
  r2 = wave_sum64(r2);
  if (lane == 0) red[w] = r2;
  __syncthreads();
  if (tid == 0) part[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// grid (ceil(dm / 64), ceil(n / FBR)), 512 threads: wave w owns columns c0 + 16 (w & 3) + [0, 16)
// of dZ^T and half (w >> 2) of X's NIB 16-wide column blocks (d <= 16 NIB): two waves per SIMD,
// so one wave's LDS reads and staging overlap the other's MFMAs
constexpr int BT = 512;
template <int NIB>
__global__ __launch_bounds__(BT, 1) void mlp_tail_bwd_lin_kernel(
    const double* __restrict__ S, const double* __restrict__ w2,
    const double* __restrict__ R, const double* __restrict__ X, int64_t n, int64_t d, int m1, ObjGrad og,
    double* __restrict__ lin, double* __restrict__ pw, double* __restrict__ pb, double* __restrict__ pz) {
  constexpr int NI = 16 * NIB, H0 = (NIB + 1) / 2;  // blocks of half 0; half 1 has NIB - H0
  __shared__ __attribute__((aligned(16))) double As[64 * FS];  // [c][r]: dZ^T of the chunk
  __shared__ __attribute__((aligned(16))) double Bs[NI * FS];  // [i][r]: X^T of the chunk
  __shared__ double red[BT];
  double g2;
  {
    double a = 0.0;
    for (int64_t q = threadIdx.x; q < og.np; q += BT) a += og.part[q];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int s2 = BT / 2; s2 > 0; s2 >>= 1) {
      if ((int)threadIdx.x < s2) red[threadIdx.x] += red[threadIdx.x + s2];
      __syncthreads();
    }
    g2 = 2.0 * gssq_of(og.gobj[0], red[0], og);
    __syncthreads();
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int cb = w & 3, half = w >> 2, ib0 = half ? H0 : 0, nib = half ? NIB - H0 : H0;
  const int64_t dm = d * m1, c0 = (int64_t)blockIdx.x * 64, rs0 = (int64_t)blockIdx.y * FBR;
  const int64_t rs1 = rs0 + FBR < n ? rs0 + FBR : n;
  // the staging thread's column (fixed) and rows tid / 64 + 8 q of each chunk
  const int cc = tid & 63;
  const int64_t gc = c0 + cc;
  const bool cv = gc < dm;
  const int64_t j = cv ? gc / m1 : 0;
  const bool mz = cv && gc % m1 == 0;
  const double wv = cv ? w2[gc] : 0.0;
  double aw = 0.0, ab = 0.0, az = 0.0;
  constexpr int XB = FK * NI / BT;  // X values per thread per chunk (NI / 16)
  double rv[4], zv[4], xb[XB];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t gr = k0 + (tid >> 6) + 8 * q;
      const bool ok = cv && gr < rs1;
      rv[q] = ok ? R[gr * d + j] : 0.0;
      zv[q] = ok ? S[gr * dm + gc] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < XB; ++it) {
      const int e = it * BT + tid, rr = e / NI, i = e % NI;
      const int64_t gr = k0 + rr;
      xb[it] = (gr < rs1 && i < d) ? X[gr * d + i] : 0.0;
    }
  };
  dbl4 acc[H0];
#pragma unroll
  for (int ib = 0; ib < H0; ++ib) acc[ib] = dbl4{0.0, 0.0, 0.0, 0.0};
  load(rs0);
  for (int64_t k0 = rs0; k0 < rs1; k0 += FK) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = (tid >> 6) + 8 * q;
      double dz = 0.0;
      if (cv && k0 + rr < rs1) {
        const double dxh = g2 * rv[q];
        const double sv = zv[q];
        dz = dxh * wv * (sv * (1.0 - sv));
        aw += dxh * sv;
        ab += dxh;
        az += dz;
      }
      As[cc * FS + rr] = dz;
    }
#pragma unroll
    for (int it = 0; it < XB; ++it) {
      const int e = it * BT + tid;
      Bs[(e % NI) * FS + e / NI] = xb[it];
    }
    __syncthreads();
    if (k0 + FK < rs1) load(k0 + FK);
#pragma unroll
    for (int s = 0; s < ((MLP_FUSED_PROBE & 4) ? 0 : FK / 4); ++s) {
      const double a = As[(16 * cb + r) * FS + 4 * s + kq];
#pragma unroll
      for (int ib = 0; ib < H0; ++ib) {
        if (ib < nib) {
          const double b = Bs[(16 * (ib0 + ib) + r) * FS + 4 * s + kq];
          acc[ib] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[ib], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  double* out = lin + (int64_t)blockIdx.y * dm * d;
#pragma unroll
  for (int ib = 0; ib < H0; ++ib)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t c = c0 + 16 * cb + acc_row(lane, t), i = 16 * (ib0 + ib) + acc_col(lane);
      if (ib < nib && c < dm && i < d) out[c * d + i] = acc[ib][t];
    }
  // the column partials of this split: the eight threads of a column in a fixed order
  const int64_t zs = blockIdx.y;
  double vals[3] = {aw, ab, az};
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    red[tid] = vals[f];
    __syncthreads();
    if (tid < 64 && cv) {
      const double v = ((red[tid] + red[tid + 64]) + (red[tid + 128] + red[tid + 192])) +
                       ((red[tid + 256] + red[tid + 320]) + (red[tid + 384] + red[tid + 448]));
      if (f == 0) pw[zs * dm + gc] = v;
      if (f == 1 && mz) pb[zs * d + j] = v;
      if (f == 2 && pz) pz[zs * dm + gc] = v;
    }
    __syncthreads();
  }
}

template <int NCB>
void launch_fwd_ncb(const double* X, const double* W1, const double* b1, const double* w2, const double* b2,
                    int64_t n, int64_t d, int m1, double* S, double* R, double* part, hipStream_t stream) {
  const int64_t dm = d * m1;
  hipLaunchKernelGGL(mlp_fc1_tail_fwd_kernel<NCB>, dim3((unsigned)((n + 63) / 64), (unsigned)((dm + 16 * NCB - 1) / (16 * NCB))),
                     dim3(NTHREADS), 0, stream, X, W1, b1, w2, b2, n, d, m1, S, R, part);
}

template <int NIB>
void launch_bwd_nib(const double* S, const double* w2, const double* R, const double* X, int64_t n, int64_t d, int m1,
                    const ObjGrad& og, double* lin, double* pw, double* pb, double* pz, hipStream_t stream) {
  const int64_t dm = d * m1;
  hipLaunchKernelGGL(mlp_tail_bwd_lin_kernel<NIB>, dim3((unsigned)((dm + 63) / 64), (unsigned)((n + FBR - 1) / FBR)),
                     dim3(BT), 0, stream, S, w2, R, X, n, d, m1, og, lin, pw, pb, pz);
}

template <int... I>
void dispatch_nib(std::integer_sequence<int, I...>, int nib, const double* S, const double* w2, const double* R,
                  const double* X, int64_t n, int64_t d, int m1, const ObjGrad& og, double* lin, double* pw,
                  double* pb, double* pz, hipStream_t stream) {
  ((nib == I + 1 ? (launch_bwd_nib<I + 1>(S, w2, R, X, n, d, m1, og, lin, pw, pb, pz, stream), 0) : 0), ...);
}

}  // namespace

// the 16-column blocks of a forward tile for m1 hidden units: the largest NCB <= 8 with 16 NCB a
// multiple of m1 (0: the fused path does not take this m1)
int mlp_fused_ncb(int64_t m1) {
  for (int ncb = 8; ncb >= 1; --ncb)
    if ((16 * ncb) % m1 == 0) return ncb;
  return 0;
}

int64_t mlp_fused_parts(int64_t n, int64_t d, int64_t m1) {
  const int ncb = (n >= 1 && d >= 1 && d <= 16 * MLP_FUSED_MAX_NIB && m1 >= 1) ? mlp_fused_ncb(m1) : 0;
  if (ncb == 0) return 0;
  return ((n + 63) / 64) * ((d * m1 + 16 * ncb - 1) / (16 * ncb));
}

int64_t mlp_fused_splits(int64_t n) { return (n + FBR - 1) / FBR; }

void launch_mlp_fc1_tail_fwd(const double* X, const double* W1, const double* b1, const double* w2, const double* b2,
                             int64_t n, int64_t d, int m1, double* S, double* R, double* part, hipStream_t stream) {
  switch (mlp_fused_ncb(m1)) {
    case 1: launch_fwd_ncb<1>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 2: launch_fwd_ncb<2>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 3: launch_fwd_ncb<3>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 4: launch_fwd_ncb<4>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 5: launch_fwd_ncb<5>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 6: launch_fwd_ncb<6>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 7: launch_fwd_ncb<7>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    case 8: launch_fwd_ncb<8>(X, W1, b1, w2, b2, n, d, m1, S, R, part, stream); break;
    default: throw std::invalid_argument("mlp_fc1_tail_fwd: m1 not supported by the fused path");
  }
  HIP_TRY(hipGetLastError());
}

void launch_mlp_tail_bwd_lin(const double* S, const double* w2, const double* R, const double* X,
                             const double* part, int64_t npart, const double* gobj, double mu, double half_d,
                             double inv_n, int64_t n, int64_t d, int m1, double* lin, double* dw2, double* db2,
                             double* db1, double* scratch, hipStream_t stream) {
  const int64_t dm = d * m1, ns = mlp_fused_splits(n);
  const int nib = (int)((d + 15) / 16);
  if (nib < 1 || nib > MLP_FUSED_MAX_NIB) throw std::invalid_argument("mlp_tail_bwd_lin: d above the fused path");
  double* pw = scratch;
  double* pb = scratch + ns * dm;
  double* pz = db1 ? pb + ns * d : nullptr;
  dispatch_nib(std::make_integer_sequence<int, MLP_FUSED_MAX_NIB>{}, nib, S, w2, R, X, n, d, m1,
               ObjGrad{part, npart, gobj, mu, half_d, inv_n}, lin, pw, pb, pz, stream);
  const int64_t cols = dm + d + (db1 ? dm : 0);
  hipLaunchKernelGGL(mlp_tail_dw_kernel, dim3((unsigned)((cols + NTHREADS - 1) / NTHREADS)), dim3(NTHREADS), 0,
                     stream, pw, pb, pz, ns, d, m1, dw2, db2, db1);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma

#endif  // MIDAGMA_EXPERIMENTS
