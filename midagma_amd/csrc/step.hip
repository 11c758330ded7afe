// Per-step control and the fused elementwise update (linear.py:224-331).
//
// reduce_check : domain test any(inv + 1e-16 < 0) (linear.py:226-230) and, on
//                checkpoint slots, the score / L1 partial sums (linear.py:85-87, 129)
// control      : one workgroup; deterministic sums, checkpoint objective and
//                tolerance test (linear.py:279-331), the out-of-domain branch
//                with lr halving (linear.py:230-241), Adam bias terms
// fused_update : G_obj (linear.py:248) -> Adam (138-163) -> W -= lr g; W *= mask
//                (275-276), or the line-search W += lr g; W -= (lr/2) g.
// Elementwise arithmetic keeps numpy's operation order; the library is built
// with -ffp-contract=off so no multiply-add is fused behind our back.
#include "launch.h"
#include "control.h"
#include "np_sum.h"

namespace midagma {

__device__ __forceinline__ double block_sum_min(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = NTHREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
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

__global__ __launch_bounds__(NTHREADS) void reduce_check_kernel(const double* __restrict__ Mt,
                                                                const double* __restrict__ W,
                                                                const double* __restrict__ Z,
                                                                const Params* __restrict__ pr,
                                                                State* __restrict__ st,
                                                                double* __restrict__ partials, int64_t d,
                                                                int64_t D) {
  if (st->status != ST_RUNNING) return;
  const bool w32 = pr->w32 != 0;
  __shared__ double red[NTHREADS];
  __shared__ int flag_sh;
  if (threadIdx.x == 0) flag_sh = 0;
  const bool ck = st->ckpt_pending != 0;
  int flag = 0;
  double sd = 0.0, l1 = 0.0;
  for (int64_t i = blockIdx.x; i < d; i += gridDim.x) {
    for (int64_t j = threadIdx.x; j < d; j += NTHREADS) {
      const int64_t idx = i * D + j;
      const double m = Mt[idx];
      if (m_entry(m, w32) < 0.0) flag |= 1;
      if (!isfinite(m)) flag |= 2;
      if (ck) {
        const double w = W[idx];
        sd += one_minus(i == j, w, w32) * Z[idx];
        l1 += fabs(w);
      }
    }
  }
  __syncthreads();
  if (flag) atomicOr(&flag_sh, flag);
  const double s_sd = block_sum(sd, red);
  const double s_l1 = block_sum(l1, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = s_sd;
    partials[2 * blockIdx.x + 1] = s_l1;
    if (flag_sh) atomicOr(&st->flags, flag_sh);
  }
}

// |W| flattened, numpy's order: 32-bit index arithmetic while d * d fits (the 64-bit division
// was most of a serial chunk's time)
struct AbsW32u {
  const double* W;
  uint32_t d;
  int64_t D;
  __device__ float operator()(int64_t f) const {
    const uint32_t u = (uint32_t)f;
    return fabsf((float)W[(int64_t)(u / d) * D + u % d]);
  }
};

// np.abs(W).sum() of a float32 W as numpy computes it (np_sum.h), on checkpoint slots of a
// float32 fit: a thread per 8192-element chunk (numpy's pairwise sum inside it), then the
// chunks' running float32 total in order.  One workgroup: ~1 ms per checkpoint at d = 1000,
// checkpoint slots only.
__global__ __launch_bounds__(1024) void np_l1_kernel(const double* __restrict__ W, int64_t d, int64_t D,
                                                     const State* __restrict__ st, float* __restrict__ chunk_sums,
                                                     double* __restrict__ out) {
  if (st->status != ST_RUNNING || !st->ckpt_pending) return;
  const int64_t n = d * d, nc = (n + NP_SUM_CHUNK - 1) / NP_SUM_CHUNK;
  for (int64_t c = threadIdx.x; c < nc; c += blockDim.x) {
    const int64_t off = c * NP_SUM_CHUNK, len = n - off < NP_SUM_CHUNK ? n - off : NP_SUM_CHUNK;
    chunk_sums[c] = n < (int64_t(1) << 32) ? np_pairwise(AbsW32u{W, (uint32_t)d, D}, off, len)
                                           : np_pairwise(AbsW32{W, d, D}, off, len);
  }
  __threadfence_block();
  __syncthreads();
  if (threadIdx.x == 0) {
    float total = 0.f;
    for (int64_t c = 0; c < nc; ++c) total += chunk_sums[c];
    out[0] = (double)total;
  }
}

__global__ __launch_bounds__(NTHREADS) void control_kernel(const Params* __restrict__ pr, State* __restrict__ st,
                                                           const double* __restrict__ partials,
                                                           const double* __restrict__ pivlog,
                                                           const double* __restrict__ loss_total,
                                                           const double* __restrict__ bc_table,
                                                           CkptRec* __restrict__ ckpt, int64_t ckpt_cap,
                                                           const double* __restrict__ npart, int64_t nnpart,
                                                           const double* __restrict__ trek_val,
                                                           const double* __restrict__ l1_32) {
  if (st->status != ST_RUNNING) {
    if (threadIdx.x == 0) st->action = ACT_NOOP;
    return;
  }
  __shared__ double red[NTHREADS];
  const bool ck = st->ckpt_pending != 0;
  double sd = 0.0, l1 = 0.0, ld = 0.0;
  double nf[NORM_FIELDS];
  if (ck) {
    for (int i = threadIdx.x; i < NRED; i += NTHREADS) {
      sd += partials[2 * i];
      l1 += partials[2 * i + 1];
    }
    for (int64_t i = threadIdx.x; i < pr->d; i += NTHREADS) ld += pivlog[i];
    sd = block_sum(sd, red);
    l1 = block_sum(l1, red);
    ld = block_sum(ld, red);
    // the checkpoint step's norms (fused_update partials of the previous slot)
    for (int f = 0; f < NORM_FIELDS; ++f) nf[f] = f == NF_WMIN ? INFINITY : 0.0;
    for (int64_t b = threadIdx.x; b < nnpart; b += NTHREADS) {
      const double* q = npart + b * NORM_FIELDS;
      for (int f = 0; f < NF_WMAX; ++f) nf[f] += q[f];
      nf[NF_WMAX] = fmax(nf[NF_WMAX], q[NF_WMAX]);
      nf[NF_WMIN] = fmin(nf[NF_WMIN], q[NF_WMIN]);
    }
    for (int f = 0; f < NF_WMAX; ++f) nf[f] = block_sum(nf[f], red);
    nf[NF_WMAX] = -block_sum_min(-nf[NF_WMAX], red);
    nf[NF_WMIN] = block_sum_min(nf[NF_WMIN], red);
  }
  if (threadIdx.x != 0) return;
  control_open(st);
  const int flags = st->flags;
  st->flags = 0;
  if (ck) {
    st->ckpt_pending = 0;
    const double score = pr->logistic ? loss_total[0] * pr->logit_scale : pr->score_scale * sd;
    double h, l1term;
    if (l1_32) {
      // float32 W (linear.py:113-114, 127): np.abs(W).sum() is numpy's float32 sum (np_l1_kernel),
      // lambda1 * it a float32 product (a Python float times a float32 scalar), slogdet's log|det|
      // a float32 (modelled as the float64 one rounded); score and h come out float64
      l1 = l1_32[0];
      l1term = f32r(f32r(pr->lambda1) * l1);
      h = -f32r(ld) + pr->d_log_s;
    } else {
      l1term = pr->lambda1 * l1;
      h = -ld + pr->d_log_s;
    }
    double obj = pr->mu * (score + l1term) + h;
    const double tv = trek_val ? trek_val[0] : 0.0;
    if (pr->trek_mode == 2) obj = obj + pr->trek_weight * tv;  // linear.py:131-133
    if (st->n_ckpt < ckpt_cap) {
      CkptRec& r = ckpt[st->n_ckpt];
      r.iter = st->iter;
      r.obj = obj;
      r.score = score;
      r.h = h;
      r.lr = st->lr;
      r.l1 = l1;
      r.w_norm = sqrt(nf[NF_W2]);
      r.max_abs_w = nf[NF_WMAX];
      r.min_abs_w_nonzero = isfinite(nf[NF_WMIN]) ? nf[NF_WMIN] : 0.0;  // linear.py:311: 0 if W == 0
      r.grad_raw_norm = sqrt(nf[NF_GOBJ]);
      r.grad_step_norm = sqrt(nf[NF_GSTEP]);
      r.grad_score_norm = sqrt(nf[NF_GSCORE]);
      r.grad_dag_norm = sqrt(nf[NF_GDAG]);
      r.grad_l1_norm = sqrt(nf[NF_GL1]);
      r.grad_inc_norm = sqrt(nf[NF_GINC]);
      r.elapsed = (double)(__builtin_amdgcn_s_memrealtime() - st->t0) * 1e-8;
      r.reg_trek_value = tv;
      r.grad_trek_norm = sqrt(nf[NF_GTREK]);
    }
    st->n_ckpt += 1;
    st->obj_last = obj;
    st->score_last = score;
    st->h_last = h;
    st->l1_last = l1;
    if (fabs((st->obj_prev - obj) / st->obj_prev) <= pr->tol) {
      st->status = ST_DONE;
      st->early_stop = 1;
      st->action = ACT_NOOP;
      return;
    }
    st->obj_prev = obj;
    if (st->iter >= pr->max_iter) {
      st->status = ST_DONE;
      st->action = ACT_NOOP;
      return;
    }
  }
  control_decide(pr, st, flags, bc_table);
}

__device__ __forceinline__ double sign_of(double w) { return w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : w); }

// the score partial at idx: one buffer, or split-K slices summed as sum_slices_kernel does
// (up to 4 slices, the cov score GEMM's split at every size: the loads issue together; a loop
// over a run-time count waited for each before the next)
__device__ __forceinline__ double z_at(const double* __restrict__ Z, int zsplit, int64_t zstride, int64_t idx) {
  if (zsplit <= 4) {
    const double z0 = Z[idx];
    const double z1 = zsplit > 1 ? Z[zstride + idx] : 0.0;
    const double z2 = zsplit > 2 ? Z[2 * zstride + idx] : 0.0;
    const double z3 = zsplit > 3 ? Z[3 * zstride + idx] : 0.0;
    double acc = z0;
    if (zsplit > 1) acc += z1;
    if (zsplit > 2) acc += z2;
    if (zsplit > 3) acc += z3;
    return acc;
  }
  double acc = Z[idx];
  for (int z = 1; z < zsplit; ++z) acc += Z[z * zstride + idx];
  return acc;
}

// One entry of a checkpoint iteration's STEP: the update of update_entry (the same arithmetic)
// and the entry's terms of the record's norms in q (linear.py:262-273, 307-311); m, v stored,
// the new W entry returned
__device__ __forceinline__ double step_entry_norms(const Params* __restrict__ pr, const State* __restrict__ st,
                                                   const double* __restrict__ W, double* __restrict__ m,
                                                   double* __restrict__ v, const double* __restrict__ Mt,
                                                   const double* __restrict__ Z, int zsplit, int64_t zstride,
                                                   const double* __restrict__ cov, const double* __restrict__ minc,
                                                   const double* __restrict__ mexc, const double* __restrict__ trek,
                                                   int64_t idx, double (&q)[NORM_FIELDS]) {
  const double w = W[idx];
  const bool w32 = pr->w32 != 0;
  const double mt = m_entry(Mt[idx], w32);
  double gs = pr->zscale * z_at(Z, zsplit, zstride, idx);
  if (pr->logistic) gs = gs + pr->cscale * cov[idx];
  const double sg = sign_of(w);
  const double gl1 = pr->mu_l1 * sg;
  const double gh = h_term(w, mt, w32);
  double gobj = gs + gl1;
  gobj = gobj + gh;
  double ginc = 0.0;
  if (pr->has_inc) {
    ginc = minc[idx] * sg;
    gobj = gobj + ginc;
  }
  double gtr = 0.0;
  if (trek) {  // Gobj + weight * trek_grad (linear.py:257-258); trek holds weight * grad
    gtr = trek[idx];
    gobj = gobj + gtr;
  }
  const double mm = m[idx] * pr->beta1 + pr->c1 * gobj;
  const double vv = v[idx] * pr->beta2 + pr->c2 * (gobj * gobj);
  const double mh = mm / st->bc1;
  const double vh = vv / st->bc2;
  const double gd = mh / (sqrt(vh) + 1e-8);
  double wn = w - st->lr_a * gd;
  if (w32) wn = f32r(wn);  // W -= lr * grad into a float32 W (linear.py:275)
  if (pr->has_exc) wn = wn * mexc[idx];
  m[idx] = mm;
  v[idx] = vv;
  q[NF_GOBJ] = gobj * gobj;
  q[NF_GSCORE] = gs * gs;
  q[NF_GDAG] = gh * gh;
  q[NF_GL1] = gl1 * gl1;
  q[NF_GINC] = ginc * ginc;
  q[NF_GTREK] = gtr * gtr;
  q[NF_GSTEP] = gd * gd;
  q[NF_W2] = wn * wn;
  q[NF_WMAX] = fabs(wn);
  if (wn != 0.0) q[NF_WMIN] = fabs(wn);
  return wn;
}

__device__ __forceinline__ void norms_init(double (&q)[NORM_FIELDS]) {
  for (int f = 0; f < NORM_FIELDS; ++f) q[f] = f == NF_WMIN ? INFINITY : 0.0;
}

// The workgroup's NORM_FIELDS partials of a 256-column row chunk into out (lane butterflies, then
// the four waves in a fixed order); every thread of the workgroup calls it
__device__ __forceinline__ void norms_store(const double (&q)[NORM_FIELDS], double (*red)[4],
                                            double* __restrict__ out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int f = 0; f < NORM_FIELDS; ++f) {
    double x = q[f];
    for (int off = 32; off > 0; off >>= 1) {
      const double y = __shfl_xor(x, off);
      x = f == NF_WMAX ? fmax(x, y) : (f == NF_WMIN ? fmin(x, y) : x + y);
    }
    if (lane == 0) red[f][wv] = x;
  }
  __syncthreads();
  if (threadIdx.x < NORM_FIELDS) {
    const int f = threadIdx.x;
    const double a = red[f][0], b = red[f][1], c = red[f][2], e = red[f][3];
    const double r = f == NF_WMAX ? fmax(fmax(a, b), fmax(c, e))
                                  : (f == NF_WMIN ? fmin(fmin(a, b), fmin(c, e)) : (a + b) + (c + e));
    out[f] = r;
  }
  __syncthreads();
}

// The STEP of a checkpoint iteration: the same update as fused_update_kernel plus the
// partials of the record's norms, one row of NORM_FIELDS per (row, 256-column chunk).  Only
// every `checkpoint`-th slot takes this path.
__device__ __noinline__ void fused_step_with_norms(const Params* __restrict__ pr, const State* __restrict__ st,
                                                   double* __restrict__ W, double* __restrict__ m,
                                                   double* __restrict__ v,
                                                   const double* __restrict__ Mt, const double* __restrict__ Z,
                                                   int zsplit, int64_t zstride,
                                                   const double* __restrict__ cov, const double* __restrict__ minc,
                                                   const double* __restrict__ mexc, const double* __restrict__ trek,
                                                   int64_t d, int64_t D, double* __restrict__ npart) {
  __shared__ double red[NORM_FIELDS][4];
  const int64_t j = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  const int64_t i = blockIdx.y;
  double q[NORM_FIELDS];
  norms_init(q);
  if (j < d) {
    const int64_t idx = i * D + j;
    W[idx] = step_entry_norms(pr, st, W, m, v, Mt, Z, zsplit, zstride, cov, minc, mexc, trek, idx, q);
  }
  norms_store(q, red, npart + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * NORM_FIELDS);
}

// One entry's update (act STEP, HALVE or REVERT; no checkpoint norms): m, v stored on a STEP,
// the new W entry returned (fused_update_kernel and the tiled fused_update_at_kernel)
__device__ __forceinline__ double update_entry(
    const Params* __restrict__ pr, const State* __restrict__ st, int act, const double* __restrict__ W,
    double* __restrict__ m, double* __restrict__ v, const double* __restrict__ Mt, const double* __restrict__ Z,
    int zsplit, int64_t zstride, const double* __restrict__ cov, const double* __restrict__ minc,
    const double* __restrict__ mexc, const double* __restrict__ trek, int64_t idx) {
  if (act == ACT_STEP) {
    // every operand load first (the optional ones behind uniform selects), then the arithmetic:
    // with the loads among the branches the compiler waited for each before the next
    const bool logistic = pr->logistic != 0, has_inc = pr->has_inc != 0, has_exc = pr->has_exc != 0;
    const double w = W[idx], mtr = Mt[idx], mo = m[idx], vo = v[idx];
    const double zs = z_at(Z, zsplit, zstride, idx);
    const double cv = logistic ? cov[idx] : 0.0;
    const double ci = has_inc ? minc[idx] : 0.0;
    const double tk = trek ? trek[idx] : 0.0;
    const double ce = has_exc ? mexc[idx] : 1.0;
    const bool w32 = pr->w32 != 0;
    const double mt = m_entry(mtr, w32);
    double gs = pr->zscale * zs;
    if (logistic) gs = gs + pr->cscale * cv;
    const double sg = sign_of(w);
    double gobj = gs + pr->mu_l1 * sg;
    gobj = gobj + h_term(w, mt, w32);
    if (has_inc) gobj = gobj + ci * sg;
    if (trek) gobj = gobj + tk;
    const double mm = mo * pr->beta1 + pr->c1 * gobj;
    const double vv = vo * pr->beta2 + pr->c2 * (gobj * gobj);
    const double mh = mm / st->bc1;
    const double vh = vv / st->bc2;
    const double gd = mh / (sqrt(vh) + 1e-8);
    double wn = w - st->lr_a * gd;
    if (w32) wn = f32r(wn);  // W -= lr * grad into a float32 W (linear.py:275)
    if (has_exc) wn = wn * ce;
    m[idx] = mm;
    v[idx] = vv;
    return wn;
  }
  // the last STEP's Adam direction, recomputed from its m, v and bias terms (unchanged
  // since: bit-identical to the value that step applied, so no d x d store per step)
  const double gd = (m[idx] / st->bc1) / (sqrt(v[idx] / st->bc2) + 1e-8);
  // (float32 W: each in-place update rounds, linear.py:235, 239)
  const bool w32 = pr->w32 != 0;
  if (act == ACT_HALVE) {
    double wn = W[idx] + st->lr_a * gd;
    if (w32) wn = f32r(wn);
    wn = wn - st->lr_b * gd;
    return w32 ? f32r(wn) : wn;
  }
  const double wn = W[idx] + st->lr_a * gd;  // ACT_REVERT
  return w32 ? f32r(wn) : wn;
}

__global__ __launch_bounds__(NTHREADS) void fused_update_kernel(
    const Params* __restrict__ pr, const State* __restrict__ st, double* __restrict__ W, double* __restrict__ m,
    double* __restrict__ v, const double* __restrict__ Mt, const double* __restrict__ Z,
    int zsplit, int64_t zstride, const double* __restrict__ cov, const double* __restrict__ minc,
    const double* __restrict__ mexc, const double* __restrict__ trek, int64_t d, int64_t D,
    double* __restrict__ npart) {
  const int act = st->action;
  if (act == ACT_NOOP) return;
  const int64_t j = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (act == ACT_STEP && st->ckpt_pending) {  // checkpoint step: also the record's norms
    fused_step_with_norms(pr, st, W, m, v, Mt, Z, zsplit, zstride, cov, minc, mexc, trek, d, D, npart);
    return;
  }
  if (j >= d) return;
  const int64_t idx = i * D + j;
  W[idx] = update_entry(pr, st, act, W, m, v, Mt, Z, zsplit, zstride, cov, minc, mexc, trek, idx);
}

// fused_update on a fast slot with the next slot's build_at folded in (MIDAGMA_EXP_AT_FOLD):
// 8-row x 256-column tiles of the whole padded D x D grid, thread t on column t of the tile.
// Each entry's update is fused_update_kernel's (update_entry; on a checkpoint iteration's STEP
// step_entry_norms and the norm partials of each (row, 256-column chunk), fused_step_with_norms'
// partition and order); then I - W_new (IW, row-major; nullable) and A^T = s I - (W_new o W_new)^T
// through the LDS tile into A0, one 64-byte row segment per 8 threads (build_at_tile's values and
// padding, bit for bit).
__global__ __launch_bounds__(NTHREADS) void fused_update_at_kernel(
    const Params* __restrict__ pr, const State* __restrict__ st, double* __restrict__ W, double* __restrict__ m,
    double* __restrict__ v, const double* __restrict__ Mt, const double* __restrict__ Z, int zsplit,
    int64_t zstride, const double* __restrict__ cov, const double* __restrict__ minc,
    const double* __restrict__ mexc, const double* __restrict__ trek, int64_t d, int64_t D,
    double* __restrict__ A0, double* __restrict__ IW, double* __restrict__ npart) {
  const int act = st->action;
  if (act == ACT_NOOP) return;
  __shared__ double tile[NTHREADS][9];
  __shared__ double red[NORM_FIELDS][4];
  const bool w32 = pr->w32 != 0;
  const double s = pr->s;
  const bool norms = act == ACT_STEP && st->ckpt_pending;
  const int64_t J = (int64_t)blockIdx.x * NTHREADS + threadIdx.x, I0 = (int64_t)blockIdx.y * 8;
  const int64_t gx = (d + NTHREADS - 1) / NTHREADS;  // fused_update_kernel's column chunks
  for (int r = 0; r < 8; ++r) {
    const int64_t I = I0 + r, idx = I * D + J;
    const bool in = I < d && J < d;
    double x = 0.0;
    if (norms) {
      double q[NORM_FIELDS];
      norms_init(q);
      if (in) {
        x = step_entry_norms(pr, st, W, m, v, Mt, Z, zsplit, zstride, cov, minc, mexc, trek, idx, q);
        W[idx] = x;
      }
      if (I < d && (int64_t)blockIdx.x < gx) norms_store(q, red, npart + (I * gx + blockIdx.x) * NORM_FIELDS);
    } else if (in) {
      x = update_entry(pr, st, act, W, m, v, Mt, Z, zsplit, zstride, cov, minc, mexc, trek, idx);
      W[idx] = x;
    }
    if (J < D && IW) IW[idx] = one_minus(I == J, x, w32);
    tile[threadIdx.x][r] = in ? sw_entry(I == J, s, x, w32) : ((I == J) ? 1.0 : 0.0);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = it * NTHREADS + threadIdx.x, jj = e >> 3, ii = e & 7;
    const int64_t Jw = (int64_t)blockIdx.x * NTHREADS + jj;
    if (Jw < D) A0[Jw * D + I0 + ii] = tile[jj][ii];
  }
}

__global__ void scale_kernel(const double* __restrict__ x, double a, double* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTHREADS)
    y[i] = a * x[i];
}

__global__ void h_grad_kernel(const double* __restrict__ W, const double* __restrict__ Mt, double* __restrict__ G,
                              int64_t d, int64_t D) {
  const int64_t j = (int64_t)blockIdx.x * NTHREADS + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= d) return;
  G[i * d + j] = (2.0 * W[i * D + j]) * Mt[i * D + j];
}

__global__ __launch_bounds__(NTHREADS) void trace_l1_kernel(const double* __restrict__ W,
                                                            const double* __restrict__ Z,
                                                            double* __restrict__ partials, int64_t d,
                                                            int64_t D) {
  __shared__ double red[NTHREADS];
  double sd = 0.0, l1 = 0.0;
  for (int64_t i = blockIdx.x; i < d; i += gridDim.x)
    for (int64_t j = threadIdx.x; j < d; j += NTHREADS) {
      const int64_t idx = i * D + j;
      const double w = W[idx];
      sd += (((i == j) ? 1.0 : 0.0) - w) * Z[idx];
      l1 += fabs(w);
    }
  sd = block_sum(sd, red);
  l1 = block_sum(l1, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = sd;
    partials[2 * blockIdx.x + 1] = l1;
  }
}

__global__ void any_nonfinite_kernel(const double* __restrict__ x, int64_t n, int* __restrict__ flag) {
  int f = 0;
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTHREADS)
    f |= isfinite(x[i]) ? 0 : 1;
  if (__any(f) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void launch_any_nonfinite(const double* x, int64_t n, int* flag, hipStream_t stream) {
  HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), stream));
  int64_t blocks = (n + NTHREADS - 1) / NTHREADS;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(any_nonfinite_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, x, n, flag);
  HIP_TRY(hipGetLastError());
}

void launch_reduce_check(const double* Mt, const double* W, const double* Z, const Params* pr, State* st,
                         double* partials, int64_t d, int64_t D, hipStream_t stream) {
  hipLaunchKernelGGL(reduce_check_kernel, dim3(NRED), dim3(NTHREADS), 0, stream, Mt, W, Z, pr, st, partials, d, D);
  HIP_TRY(hipGetLastError());
}

void launch_control(const Params* pr, State* st, const double* partials, const double* pivlog,
                    const double* loss_total, const double* bc_table, CkptRec* ckpt, int64_t ckpt_cap,
                    const double* npart, int64_t d, const double* trek_val, hipStream_t stream,
                    const double* l1_32) {
  const int64_t nnpart = ((d + NTHREADS - 1) / NTHREADS) * d;  // fused_update workgroups
  hipLaunchKernelGGL(control_kernel, dim3(1), dim3(NTHREADS), 0, stream, pr, st, partials, pivlog, loss_total,
                     bc_table, ckpt, ckpt_cap, npart, nnpart, trek_val, l1_32);
  HIP_TRY(hipGetLastError());
}

int64_t np_l1_chunks(int64_t d) { return (d * d + NP_SUM_CHUNK - 1) / NP_SUM_CHUNK; }

void launch_np_l1(const double* W, int64_t d, int64_t D, const State* st, float* chunk_sums, double* out,
                  hipStream_t stream) {
  hipLaunchKernelGGL(np_l1_kernel, dim3(1), dim3(1024), 0, stream, W, d, D, st, chunk_sums, out);
  HIP_TRY(hipGetLastError());
}

void launch_fused_update(const Params* pr, const State* st, double* W, double* m, double* v, const double* Mt, const double* Z, int zsplit, int64_t zstride, const double* cov,
                         const double* minc, const double* mexc, const double* trek, int64_t d, int64_t D,
                         double* npart, hipStream_t stream) {
  dim3 grid((unsigned)((d + NTHREADS - 1) / NTHREADS), (unsigned)d);
  hipLaunchKernelGGL(fused_update_kernel, grid, dim3(NTHREADS), 0, stream, pr, st, W, m, v, Mt, Z, zsplit,
                     zstride, cov, minc, mexc, trek, d, D, npart);
  HIP_TRY(hipGetLastError());
}

void launch_fused_update_at(const Params* pr, const State* st, double* W, double* m, double* v, const double* Mt,
                            const double* Z, int zsplit, int64_t zstride, const double* cov, const double* minc,
                            const double* mexc, const double* trek, int64_t d, int64_t D, double* A0, double* IW,
                            double* npart, hipStream_t stream) {
  if (D % 8 || !A0 || !npart) throw std::invalid_argument("fused_update_at: needs D % 8 == 0, A0 and npart");
  const dim3 grid((unsigned)((D + NTHREADS - 1) / NTHREADS), (unsigned)(D / 8));
  hipLaunchKernelGGL(fused_update_at_kernel, grid, dim3(NTHREADS), 0, stream, pr, st, W, m, v, Mt, Z, zsplit, zstride,
                     cov, minc, mexc, trek, d, D, A0, IW, npart);
  HIP_TRY(hipGetLastError());
}

void launch_scale(const double* x, double a, double* y, int64_t n, hipStream_t stream) {
  int64_t blocks = (n + NTHREADS - 1) / NTHREADS;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(scale_kernel, dim3((unsigned)blocks), dim3(NTHREADS), 0, stream, x, a, y, n);
  HIP_TRY(hipGetLastError());
}

void launch_h_grad(const double* W, const double* Mt, double* G, int64_t d, int64_t D, hipStream_t stream) {
  dim3 grid((unsigned)((d + NTHREADS - 1) / NTHREADS), (unsigned)d);
  hipLaunchKernelGGL(h_grad_kernel, grid, dim3(NTHREADS), 0, stream, W, Mt, G, d, D);
  HIP_TRY(hipGetLastError());
}

void launch_trace_l1(const double* W, const double* Z, double* partials, int64_t d, int64_t D,
                     hipStream_t stream) {
  hipLaunchKernelGGL(trace_l1_kernel, dim3(NRED), dim3(NTHREADS), 0, stream, W, Z, partials, d, D);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
