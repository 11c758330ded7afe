// Small-d cov-mode inner loop in ONE persistent workgroup (d <= 64, l2; the TCC trek regularizer
// at d <= 32, tcc_blk.h; no PST).
//
// At d = 20 a graph-replayed slot is 8 dependent launches of a 64 x 64 padded problem, each
// 4-6 us (profiles/r01_rocprof_cov_small_kernel_stats.csv): the GPU ran the reference's loop
// only 1.7x faster than its CPU.  Here the whole per-mu state lives in one CU for as many
// Adam steps as the host asks for:
//   registers : this lane's elements of W, m, v, the inverse and the score gradient, and the
//               last two slots' inverses (the warm start)
//   LDS       : (-mu) cov (the score GEMM's A operand, loaded once per launch), W and
//               I - W images (the transposed build and the MFMA B operand), the product
//               form's operand images, the Gauss-Jordan pivot row / column (double-buffered),
//               pivots, reduction slots, the State and the controller's decision
// One slot is exactly the reference's loop body (linear.py:224-331), in its order:
//   build (sI - W o W)^T -> its inverse: the warm-started product form on
//   v_mfma_f64_16x16x4f64 (3-4 dependent 32^3 products), or the unpivoted Gauss-Jordan
//   (d steps, one barrier each; sI - W o W is an M-matrix in the domain) on
//   checkpoint slots, which need the pivots for log|det| -> rhs = ((-mu) cov)(I - W) on the
//   matrix cores -> domain test any(inv + 1e-16 < 0) / non-finite ->
//   control (checkpoint objective + tolerance, line search, lr halving: the decisions of
//   step.hip's control_kernel, by thread 0 on a State kept in LDS, broadcast through LDS) ->
//   G_obj, Adam, W -= lr g, W *= mask (or the line-search revert / halving).
// Element ownership follows the f64 16x16x4 MFMA accumulator map, so every product's output
// lands in the registers of the lane that owns the element: wave w owns the 16 x 16 tile
// (w / (DS/16), w % (DS/16)); lane l owns column 16 tc + (l & 15), rows 16 tr + (l >> 4) + 4 t
// for t = 0..3.  DS = 16, 32, 64 -> 1, 4, 16 waves.
// Arithmetic per element is step.hip's, in the same order (built with -ffp-contract=off).
#include <type_traits>

#include "launch.h"
#include "np_sum.h"
#include "mfma64.h"
#include "tcc_blk.h"

namespace midagma {

// Phase stamps of the persistent slot loop (diagnostic build only: `make kstamps`, -DMIDAGMA_KSTAMPS;
// tools/small_stamps.py): thread 0 reads the shader clock at the slot's phase points and sums each
// phase over the launch's slots; without MIDAGMA_KSTAMPS the macros are empty.
#ifdef MIDAGMA_KSTAMPS
__device__ unsigned long long g_small_stamps[16];  // [0..11] phase sums, [12] slots, [13] real time
#define SS_DECL                                                     \
  unsigned long long ss_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long ss_t = __builtin_amdgcn_s_memtime();            \
  const unsigned long long ss_rt0 = __builtin_amdgcn_s_memrealtime(); \
  unsigned long long ss_n = 0
#define SS_MARK(p)                                                  \
  {                                                                 \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    ss_acc[p] += t_ - ss_t;                                         \
    ss_t = t_;                                                      \
  }
#define SS_COUNT(p, c) ss_acc[p] += (c)
#define SS_SLOT() ++ss_n
#define SS_END()                                                                                 \
  if (threadIdx.x == 0) {                                                                        \
    for (int p_ = 0; p_ < 12; ++p_) atomicAdd(&g_small_stamps[p_], ss_acc[p_]);                  \
    atomicAdd(&g_small_stamps[12], ss_n);                                                        \
    atomicAdd(&g_small_stamps[13], __builtin_amdgcn_s_memrealtime() - ss_rt0);                  \
  }
#else
#define SS_DECL \
  do {          \
  } while (0)
#define SS_MARK(p)
#define SS_COUNT(p, c)
#define SS_SLOT()
#define SS_END()
#endif
namespace {

__device__ __forceinline__ double sgn(double w) { return w > 0.0 ? 1.0 : (w < 0.0 ? -1.0 : w); }

__device__ __forceinline__ double wave_sum(double x) {
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}
__device__ __forceinline__ double wave_max(double x) {
  for (int off = 32; off > 0; off >>= 1) x = fmax(x, __shfl_xor(x, off));
  return x;
}
__device__ __forceinline__ double wave_min(double x) {
  for (int off = 32; off > 0; off >>= 1) x = fmin(x, __shfl_xor(x, off));
  return x;
}

// colb position of row i: the 4 rows a lane owns (16 tr + q + 4 t) are 4 consecutive slots
__device__ __forceinline__ int cpos(int i) { return (i & ~15) + 4 * (i & 3) + ((i & 15) >> 2); }

// acc += A[row0 .. row0+15][0 .. kd) * B[0 .. kd)[col0 .. col0+15] on the f64 16x16x4 MFMA;
// A from an [m][k] image (stride SA_), B from a [k][n] image (stride SB_).  Terms with
// k >= d are exact zeros in every product of this file (zero off-diagonal padding).
template <int DS, int SA_, int SB_>
__device__ __forceinline__ dbl4 tile_mma(const double* __restrict__ A, const double* __restrict__ B, int row0,
                                         int col0, int q, int c, int kd, dbl4 acc) {
  if (DS >= 64) {  // (a full unroll keeps 32 operands in flight: the 1024-thread kernel's registers spill)
#pragma unroll 4
    for (int kk = 0; 4 * kk < kd; ++kk)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(row0 + c) * SA_ + 4 * kk + q], B[(4 * kk + q) * SB_ + col0 + c],
                                                 acc, 0, 0, 0);
    return acc;
  }
  // DS <= 32: all DS / 4 k-steps, unguarded (the k >= d terms are the exact zeros above): the
  // operand reads of a branch-free unrolled chain issue together, where a guard per k-step
  // serialised read, wait and MFMA (d = 20: 5 guarded steps cost more than 8 pipelined ones)
  (void)kd;
#pragma unroll
  for (int kk = 0; kk < DS / 4; ++kk)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(row0 + c) * SA_ + 4 * kk + q], B[(4 * kk + q) * SB_ + col0 + c],
                                               acc, 0, 0, 0);
  return acc;
}

struct SmallCtl {
  int32_t act, norms, run, pad_;
  double lr_a, lr_b, bc1, bc2;
};

// The Params fields the controller reads, copied once per launch into LDS (read through the
// out-of-line controller's pointer argument, Params were vector-memory loads on every slot; passed
// by value, the struct went through the stack).  next_ck: the next multiple of `checkpoint` above
// the iteration (the controller advances it), in place of a 64-bit remainder per slot.
struct SmallCtlParams {
  double d_log_s, score_scale, mu, lambda1, trek_weight, tol, s;
  int64_t max_iter, checkpoint;
  int32_t trek_mode, w32;  // w32: float32 W, the objective's float32 terms (step.hip control_kernel)
};

// The controller: step.hip's control_kernel decisions (linear.py:230-241, 279-331) on the
// State in LDS, run by thread 0 once per slot.  Kept out of line: inlined into the slot loop,
// its code raised the kernel to 230+ VGPRs (DS = 64 spilled inside the Gauss-Jordan loop).
template <int NW>
__device__ __noinline__ void small_control(const SmallCtlParams& pr_, State& S, SmallCtl& ctl,
                                           const double (*red)[NW], const double (*nred)[NW], const int* flw,
                                           CkptRec* __restrict__ ckpt, int64_t ckpt_cap, double bc1n,
                                           double bc2n, const double* trek_val, int64_t& next_ck) {
    const SmallCtlParams* const pr = &pr_;
    int flags = 0;
#pragma unroll 1
    for (int x = 0; x < NW; ++x) flags |= flw[x];
    if (S.slots == 0) S.t0 = __builtin_amdgcn_s_memrealtime();
    S.slots += 1;
    S.warm_valid = 1;
    S.warm_run = S.warm_run < 2 ? S.warm_run + 1 : 2;
    S.flags = 0;
    int act = ACT_NOOP;
    bool running = true;
    if (S.ckpt_pending) {
      double sd = 0.0, l1 = 0.0, ld = 0.0;
      double nf[NORM_FIELDS];
#pragma unroll 1
      for (int x = 0; x < NW; ++x) {
        sd += red[0][x];
        l1 += red[1][x];
        ld += red[2][x];
      }
      for (int f = 0; f < NORM_FIELDS; ++f) {
        double x = f == NF_WMIN ? INFINITY : 0.0;
#pragma unroll 1
        for (int y = 0; y < NW; ++y)
          x = f == NF_WMAX ? fmax(x, nred[f][y]) : (f == NF_WMIN ? fmin(x, nred[f][y]) : x + nred[f][y]);
        nf[f] = x;
      }
      S.ckpt_pending = 0;
      // float32 W: l1 arrives as numpy's float32 sum, lambda1 * l1 and log|det| in float32
      // (step.hip control_kernel, linear.py:113-114, 127)
      const double h = pr->w32 ? -f32r(ld) + pr->d_log_s : -ld + pr->d_log_s;
      const double score = pr->score_scale * sd;
      const double l1term = pr->w32 ? f32r(f32r(pr->lambda1) * l1) : pr->lambda1 * l1;
      double obj = pr->mu * (score + l1term) + h;
      const double tv = trek_val ? trek_val[0] : 0.0;
      if (trek_val && pr->trek_mode == 2) obj = obj + pr->trek_weight * tv;  // linear.py:131-133
      if (S.n_ckpt < ckpt_cap) {
        CkptRec& r = ckpt[S.n_ckpt];
        r.iter = S.iter;
        r.obj = obj;
        r.score = score;
        r.h = h;
        r.lr = S.lr;
        r.l1 = l1;
        r.w_norm = sqrt(nf[NF_W2]);
        r.max_abs_w = nf[NF_WMAX];
        r.min_abs_w_nonzero = isfinite(nf[NF_WMIN]) ? nf[NF_WMIN] : 0.0;  // linear.py:311
        r.grad_raw_norm = sqrt(nf[NF_GOBJ]);
        r.grad_step_norm = sqrt(nf[NF_GSTEP]);
        r.grad_score_norm = sqrt(nf[NF_GSCORE]);
        r.grad_dag_norm = sqrt(nf[NF_GDAG]);
        r.grad_l1_norm = sqrt(nf[NF_GL1]);
        r.grad_inc_norm = sqrt(nf[NF_GINC]);
        r.elapsed = (double)(__builtin_amdgcn_s_memrealtime() - S.t0) * 1e-8;
        r.reg_trek_value = tv;
        r.grad_trek_norm = trek_val ? sqrt(nf[NF_GTREK]) : 0.0;
      }
      S.n_ckpt += 1;
      S.obj_last = obj;
      S.score_last = score;
      S.h_last = h;
      S.l1_last = l1;
      if (fabs((S.obj_prev - obj) / S.obj_prev) <= pr->tol) {
        S.status = ST_DONE;
        S.early_stop = 1;
        running = false;
      } else {
        S.obj_prev = obj;
        if (S.iter >= pr->max_iter) {
          S.status = ST_DONE;
          running = false;
        }
      }
    }
    if (running) {
      if (flags & 2) {
        S.status = ST_SINGULAR;
      } else if (flags & 1) {  // sI - W o W left the M-matrix domain (linear.py:230-241)
        if (S.iter == 0 || pr->s <= 0.9) {
          S.status = ST_FAILED;
        } else {
          S.warm_run = 1;
          const double lr_old = S.lr;
          S.lr = lr_old * .5;
          S.halvings += 1;
          S.lr_a = lr_old;
          S.lr_b = S.lr;
          if (S.lr <= 1e-16) {
            S.status = ST_LR_UNDERFLOW;
            act = ACT_REVERT;
          } else {
            act = ACT_HALVE;
          }
        }
      } else {
        const int64_t it = S.iter + 1;
        S.bc1 = bc1n;
        S.bc2 = bc2n;
        S.lr_a = S.lr;
        act = ACT_STEP;
        S.iter = it;
        const bool at_ck = it == next_ck;  // (it % checkpoint == 0)
        if (at_ck) next_ck += pr->checkpoint;
        if (at_ck || it == pr->max_iter) S.ckpt_pending = 1;
      }
    }
    S.action = act;
    ctl.act = act;
    ctl.norms = act == ACT_STEP && S.ckpt_pending;
    ctl.run = S.status == ST_RUNNING;
    ctl.lr_a = S.lr_a;
    ctl.lr_b = S.lr_b;
    ctl.bc1 = S.bc1;
    ctl.bc2 = S.bc2;
}

template <int DS, int NW, int TCC, bool W32 = false>
__global__ __launch_bounds__(64 * NW) void small_minimize_kernel(
    const Params* __restrict__ pr, State* __restrict__ stg, double* __restrict__ Wg, double* __restrict__ mg,
    double* __restrict__ vg, const double* __restrict__ covs, const double* __restrict__ minc,
    const double* __restrict__ mexc, const double* __restrict__ bc_table, CkptRec* __restrict__ ckpt,
    int64_t ckpt_cap, double* __restrict__ carry, double* __restrict__ pstore, int64_t n_slots, SmallTcc tc) {
  constexpr int NT = 64 * NW, TPR = DS / 16, TPW = TPR * TPR / NW, E = 4 * TPW;
  // TCC (0: off): tcc_blk.h's body on this workgroup.  4: NB x NB = NT threads of 4 x 4 blocks
  // (DS = 16: NB = 8, DS = 32: 16); 5: one wave of 5 x 5 blocks (NB = 8, 2d <= 40: d <= 20), the
  // other waves along without writes
  constexpr int TBS = TCC == 5 ? 5 : 4;
  constexpr int TNB = TCC == 5 ? 8 : DS / 2;
  static_assert(TCC == 0 || (TCC == 4 && TNB * TNB == NT && DS <= 32) || (TCC == 5 && DS == 32 && NT >= 64),
                "TCC in the small loop: d <= 32");
  static_assert(TPW * NW == TPR * TPR, "whole tiles per wave");
  constexpr int SW = DS + 2;                         // W, cov images: 16 rows x 4 cols per read
  constexpr int SI = ((DS + 15) / 32) * 32 + 16;     // I - W image: B operand rows, = 16 mod 32
  // DS = 64: the images are single-buffered (an extra barrier before each rewrite), R / Q serve
  // as A and B operand from one [m][k] image, and W is not imaged (its transpose is read from
  // the I - W image, whose off-diagonal entries are -W exactly, the diagonal from wdiag): 4
  // images of 64 x 66 / 64 x 80 doubles fit the CU's 160 KB of LDS
  constexpr bool ONE = DS >= 64;
  constexpr int SB = ONE ? SW : SI;                  // stride of the product form's B images
  __shared__ double Wimg[ONE ? 1 : DS * SW];
  __shared__ double wdiag[DS];
  __shared__ double Cimg[DS * SW];
  __shared__ double IWimg[DS * SI];
  __shared__ __attribute__((aligned(32))) double rowb[2][DS];
  __shared__ __attribute__((aligned(32))) double colb[2][DS];
  __shared__ double piv[DS];
  // product-form inverse operands, two sets: [m][k] images (PA: the left factor, PR: R as a
  // left factor) and [k][n] images (PB)
  __shared__ double PAbuf[(ONE ? 1 : 2) * DS * SW];
  __shared__ double PRbuf[(ONE ? 1 : 2) * DS * SW];
  __shared__ double PBbuf[ONE ? 1 : 2 * DS * SI];
  double* const PA[2] = {PAbuf, ONE ? PAbuf : PAbuf + DS * SW};
  double* const PR[2] = {PRbuf, ONE ? PRbuf : PRbuf + DS * SW};
  double* const PB[2] = {ONE ? PRbuf : PBbuf, ONE ? PRbuf : PBbuf + DS * SI};
  __shared__ int nrm[NW];                     // per wave: residual above 1e-2 (bit 0), 1e-4 (bit 1)
  __shared__ double red[3][NW];               // checkpoint objective: (I - W) o Z, |W|, log|pivot|
  __shared__ double nred[NORM_FIELDS][NW];    // the checkpoint step's norms, per wave
  __shared__ int flw[NW];
  __shared__ float l1img[W32 ? DS * DS : 1];  // float32 W: |W| in numpy's flat order (np_sum.h)
  __shared__ State S;                         // the controller's (thread 0's) state
  __shared__ SmallCtl ctl;                    // its decision for the slot, read by every thread
  // TCC: the body's LDS and the regularizer's state words (scal, v, u), loaded at entry
  __shared__ std::conditional_t<TCC != 0, tccb::TccLds<TNB, TBS>, char> TL;
  __shared__ double tsc[TCC ? 10 : 1], tvp[TCC ? TBS * TNB : 1], tup[TCC ? TBS * TNB : 1];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  int tr[TPW], cols[E], rows[E];
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    const int tile = w * TPW + u;
    tr[u] = tile / TPR;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      rows[4 * u + t] = 16 * tr[u] + q + 4 * t;
      cols[4 * u + t] = 16 * (tile % TPR) + c;
    }
  }
  const int64_t d = pr->d, D = pr->D;
  const int di = (int)d;
  const bool has_inc = pr->has_inc != 0, has_exc = pr->has_exc != 0;

  __shared__ SmallCtlParams cp;  // (thread 0's)
  __shared__ int64_t next_ck;
  if (tid == 0) {
    cp = SmallCtlParams{pr->d_log_s, pr->score_scale, pr->mu,          pr->lambda1,   pr->trek_weight,
                        pr->tol,     pr->s,           pr->max_iter,    pr->checkpoint, pr->trek_mode, W32 ? 1 : 0};
    S = *stg;
    next_ck = (S.iter / cp.checkpoint + 1) * cp.checkpoint;
    ctl.run = S.status == ST_RUNNING && n_slots > 0;
    if (S.ckpt_pending)  // the pending checkpoint step's norms, reduced by the last launch
      for (int f = 0; f < NORM_FIELDS; ++f) {
        nred[f][0] = carry[f];
        for (int y = 1; y < NW; ++y) nred[f][y] = f == NF_WMIN ? INFINITY : 0.0;
      }
  }
  bool real[E];
  double wv[E], mv[E], vv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    real[e] = rows[e] < di && cols[e] < di;
    const int64_t idx = (int64_t)rows[e] * D + cols[e];
    wv[e] = real[e] ? Wg[idx] : 0.0;
    mv[e] = real[e] ? mg[idx] : 0.0;
    vv[e] = real[e] ? vg[idx] : 0.0;
  }
  // MFMA A operand image: (-mu) cov, zero padding
  for (int e = tid; e < DS * SW; e += NT) {
    const int r = e / SW, k = e % SW;
    Cimg[e] = (r < di && k < di) ? covs[(int64_t)r * D + k] : 0.0;
  }
  if (!ONE)
    for (int e = tid; e < DS * SW; e += NT) Wimg[e] = 0.0;
  for (int e = tid; e < DS; e += NT) wdiag[e] = 0.0;
  for (int e = tid; e < DS * SI; e += NT) IWimg[e] = 0.0;
  if constexpr (TCC) {
    if (tid < 10) tsc[tid] = tc.scal[tid];
    for (int e = tid; e < 2 * (int)pr->d; e += NT) {
      tvp[e] = tc.vprev[e];
      tup[e] = tc.uprev[e];
    }
  }
  __syncthreads();
  if (!ctl.run) return;
  constexpr bool w32 = W32;  // dtype=np.float32 (common.h f32r; a template argument: the float64
                             // loop carries none of its selects, 5.5 -> 5.8 us a step at d = 20)
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (real[e]) {
      if (!ONE) Wimg[rows[e] * SW + cols[e]] = wv[e];
      if (rows[e] == cols[e]) wdiag[rows[e]] = wv[e];
      IWimg[rows[e] * SI + cols[e]] = one_minus(rows[e] == cols[e], wv[e], w32);
    }
  const double s_dom = pr->s;
  // the last two slots' inverses (warm start of the product form) and how many are valid;
  // kept across launches (pstore, carry[NORM_FIELDS]) so that results do not depend on how
  // the host batches slots
  double p1[E], p2[E];
  const int warm0 = (int)carry[NORM_FIELDS];
  int warm = warm0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    p1[e] = warm0 > 0 ? pstore[rows[e] * DS + cols[e]] : 0.0;
    p2[e] = warm0 > 1 ? pstore[DS * DS + rows[e] * DS + cols[e]] : 0.0;
  }
  __syncthreads();

  // the update's constants in registers (read through pr in the loop, they were reloaded every
  // slot: the out-of-line controller may write memory), and the lane's mask entries, fixed for
  // the launch (linear.py:217-222)
  const double c_zscale = pr->zscale, c_mu_l1 = pr->mu_l1, c_beta1 = pr->beta1, c_c1 = pr->c1,
               c_beta2 = pr->beta2, c_c2 = pr->c2;
  double incv[E], excv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t idx = (int64_t)rows[e] * D + cols[e];
    incv[e] = !ONE && has_inc && real[e] ? minc[idx] : 0.0;  // (DS = 64: read in the loop)
    excv[e] = !ONE && has_exc && real[e] ? mexc[idx] : 1.0;
  }
  // the controller's state every thread keeps (wave-uniform copies of S's fields): a plain Adam
  // step (no checkpoint due, no domain or finiteness flag) is decided by every thread from these,
  // thread 0 mirroring the State in LDS without a barrier; other slots go through small_control
  // (thread 0, then a barrier) and reload them.  Not at DS = 64, whose 16 waves have 128 VGPRs
  // each: the copies spill there (d = 48: 46.4k -> 43.0k steps/s)
  constexpr bool RC = !ONE;
  const int64_t c_ld_table = pr->ld_table, c_max_iter = cp.max_iter, c_checkpoint = cp.checkpoint;
  int64_t r_iter = S.iter, r_slots = S.slots, r_next = next_ck;
  double r_lr = S.lr;
  int r_ckpt = S.ckpt_pending, r_wrun = S.warm_run;

  SS_DECL;
  for (int64_t slot = 0; slot < n_slots; ++slot) {
    SS_SLOT();
    // the TCC regularizer of this slot's W (linear.py:251-258; tcc_gate_kernel's rule: every slot
    // in 'opt' mode, checkpoint slots in 'log' mode)
    bool tcc_ran = false;
    if constexpr (TCC) {
      if (tc.mode == 2 || (RC ? r_ckpt : S.ckpt_pending)) {
        tccb::tcc_blk_body<TNB, TBS>([&](int i, int j) { return Wimg[i * SW + j]; },
                                [&](int i, int j) { return tc.S[(int64_t)i * D + j]; }, tc.ws, di, tc.mode, tc.eps,
                                tc.m, tc.weight, tsc, tvp, tup, nullptr, D, TL, tc.fix != 0);
        tcc_ran = true;
      }
    }
    // 1 - beta^it for it = iter + 1 from the host table (read early: latency under the inverse)
    double bc1n = 1.0, bc2n = 1.0;
    if (RC ? r_iter < c_ld_table : (tid == 0 && S.iter < c_ld_table)) {
      const int64_t it0 = RC ? r_iter : S.iter;
      bc1n = bc_table[2 * it0];
      bc2n = bc_table[2 * it0 + 1];
    }

    // ---- (sI - W o W)^T, identity padding (linear.py:226, 113)
    double a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = rows[e], j = cols[e];
      // (read unconditionally, then selected: a read per element under its own exec mask
      // serialised the reads)
      const double wji = ONE ? (i == j ? wdiag[i] : -IWimg[j * SI + i]) : Wimg[j * SW + i];
      a[e] = real[e] ? sw_entry(i == j, s_dom, wji, w32) : ((i == j) ? 1.0 : 0.0);
    }
    // ---- a <- inv(A^T) = inv(A)^T.  Checkpoint slots (log|det| needs the pivots), the first
    // slot of a launch and unconverged warm starts: Gauss-Jordan.  Otherwise the product form
    // inv(S) = X0 (I + R)(I + R^2)[(I + R^4)], R = I - S X0, from the linear extrapolation
    // X0 = 2 P1 - P2 of the last two inverses (P1 alone after a halving), on the matrix cores
    // (blockinv.hip's fast path at one-workgroup scale; d ||R||max bounds ||R||inf).
    SS_MARK(0)  // TCC (when on), the table read issued, (sI - W o W)^T built
    bool gj = (RC ? r_ckpt : S.ckpt_pending) != 0 || warm == 0;
    if (!gj) {
      double x0[E], r[E];
      // ||R||: d max|R_ij| against 1e-2 (the series converges in the passes below) and 1e-4
      // (a third pass); rounding of d x is monotone, so max_ij(d |R_ij|) = d max_ij |R_ij| and
      // the two tests are lane tests, reduced by ballots (a wave max took 6 dependent shuffles)
      bool big2 = false, big4 = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = rows[e], j = cols[e];
        x0[e] = real[e] ? (warm >= 2 ? 2.0 * p1[e] - p2[e] : p1[e]) : ((i == j) ? 1.0 : 0.0);
        PA[1][i * SW + j] = a[e];
        PB[1][i * SB + j] = x0[e];
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const dbl4 t4 = tile_mma<DS, SW, SB>(PA[1], PB[1], 16 * tr[u], cols[4 * u] - c, q, c, di,
                                             dbl4{0.0, 0.0, 0.0, 0.0});
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int e = 4 * u + t;
          r[e] = real[e] ? (((rows[e] == cols[e]) ? 1.0 : 0.0) - t4[t]) : 0.0;
          const double dr = (double)di * fabs(r[e]);  // (NaN: fails both tests, as a NaN max did)
          big2 = big2 || !(dr <= 1e-2);
          big4 = big4 || !(dr <= 1e-4);
        }
      }
      if (ONE) __syncthreads();  // every wave is done reading the images it overwrites
#pragma unroll
      for (int e = 0; e < E; ++e) {
        PA[0][rows[e] * SW + cols[e]] = x0[e];
        PB[0][rows[e] * SB + cols[e]] = r[e];
        PR[0][rows[e] * SW + cols[e]] = r[e];
      }
      {
        const unsigned long long b2 = __ballot(big2), b4 = __ballot(big4);
        if (lane == 0) nrm[w] = (b2 ? 1 : 0) | (b4 ? 2 : 0);
      }
      __syncthreads();
      int nfl = 0;
#pragma unroll
      for (int x = 0; x < NW; ++x) nfl |= nrm[x];
      SS_MARK(7)  // warm start, residual R = I - S X0, its norm (ballots, barrier)
      if (!(nfl & 1)) {
        const bool three = (nfl & 2) != 0;  // ||R||^4 > 1e-16: one more factor
        double y[E], r2[E];
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
          const int row0 = 16 * tr[u], col0 = cols[4 * u] - c;
          const dbl4 yv = tile_mma<DS, SW, SB>(PA[0], PB[0], row0, col0, q, c, di,
                                               dbl4{x0[4 * u], x0[4 * u + 1], x0[4 * u + 2], x0[4 * u + 3]});
          const dbl4 rv = tile_mma<DS, SW, SB>(PR[0], PB[0], row0, col0, q, c, di, dbl4{0.0, 0.0, 0.0, 0.0});
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = 4 * u + t;
            y[e] = real[e] ? yv[t] : ((rows[e] == cols[e]) ? 1.0 : 0.0);
            r2[e] = real[e] ? rv[t] : 0.0;
          }
        }
        if (ONE) __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
          PA[1][rows[e] * SW + cols[e]] = y[e];
          PB[1][rows[e] * SB + cols[e]] = r2[e];
          if (three) PR[1][rows[e] * SW + cols[e]] = r2[e];
        }
        __syncthreads();
        SS_MARK(8)  // pass 1: Y = X0 + X0 R, R^2, images, barrier
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
          const int row0 = 16 * tr[u], col0 = cols[4 * u] - c;
          const dbl4 yv = tile_mma<DS, SW, SB>(PA[1], PB[1], row0, col0, q, c, di,
                                               dbl4{y[4 * u], y[4 * u + 1], y[4 * u + 2], y[4 * u + 3]});
          dbl4 rv = dbl4{0.0, 0.0, 0.0, 0.0};
          if (three) rv = tile_mma<DS, SW, SB>(PR[1], PB[1], row0, col0, q, c, di, rv);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = 4 * u + t;
            y[e] = real[e] ? yv[t] : ((rows[e] == cols[e]) ? 1.0 : 0.0);
            r2[e] = real[e] ? rv[t] : 0.0;
          }
        }
        SS_MARK(9)  // pass 2: Y + Y R^2 (and R^4)
        if (three) {
          if (ONE) __syncthreads();
#pragma unroll
          for (int e = 0; e < E; ++e) {
            PA[0][rows[e] * SW + cols[e]] = y[e];
            PB[0][rows[e] * SB + cols[e]] = r2[e];
          }
          __syncthreads();
#pragma unroll
          for (int u = 0; u < TPW; ++u) {
            const dbl4 yv = tile_mma<DS, SW, SB>(PA[0], PB[0], 16 * tr[u], cols[4 * u] - c, q, c, di,
                                                 dbl4{y[4 * u], y[4 * u + 1], y[4 * u + 2], y[4 * u + 3]});
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int e = 4 * u + t;
              y[e] = real[e] ? yv[t] : ((rows[e] == cols[e]) ? 1.0 : 0.0);
            }
          }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) a[e] = y[e];
      } else {
        gj = true;
      }
    }
    if (gj) {
      // in-place Gauss-Jordan, no pivoting (the pivots give log|det| on checkpoint slots)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (rows[e] == 0) rowb[0][cols[e]] = a[e];
        if (cols[e] == 0) colb[0][cpos(rows[e])] = a[e];
      }
      __syncthreads();
      for (int k = 0; k < di; ++k) {
        const int b = k & 1;
        const double p = rowb[b][k];
        const double pinv = 1.0 / p;
        if (tid == 0) piv[k] = p;
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
          const int j = cols[4 * u];
          const double rk = rowb[b][j] * pinv;
          const double4 ck = *reinterpret_cast<const double4*>(&colb[b][16 * tr[u] + 4 * q]);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = 4 * u + t;
            if (!real[e]) continue;
            const int i = rows[e];
            const double cki = t == 0 ? ck.x : (t == 1 ? ck.y : (t == 2 ? ck.z : ck.w));
            if (i == k)
              a[e] = (j == k) ? pinv : a[e] * pinv;
            else if (j == k)
              a[e] = -(a[e] * pinv);
            else
              a[e] = a[e] - cki * rk;
          }
        }
        if (k + 1 < di) {
          const int b1 = b ^ 1;
#pragma unroll
          for (int e = 0; e < E; ++e) {
            if (rows[e] == k + 1) rowb[b1][cols[e]] = a[e];
            if (cols[e] == k + 1) colb[b1][cpos(rows[e])] = a[e];
          }
        }
        __syncthreads();
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      p2[e] = p1[e];
      p1[e] = a[e];
    }
    warm = warm < 2 ? warm + 1 : 2;
    SS_MARK(1)  // the inverse (product form, or Gauss-Jordan on checkpoint / cold slots)
    SS_COUNT(6, gj ? 1 : 0);

    // ---- rhs = ((-mu) cov) @ (I - W)  (linear.py:244) on the matrix cores
    double z[E];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < DS / 4; ++kk)
        if (!ONE || 4 * kk < di)  // (DS <= 32 unguarded, as tile_mma; cov's padding is zero)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Cimg[(16 * tr[u] + c) * SW + 4 * kk + q],
                                                     IWimg[(4 * kk + q) * SI + cols[4 * u]], acc, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) z[4 * u + t] = acc[t];
    }

    SS_MARK(2)  // the score product on the matrix cores
    // ---- domain test (linear.py:226-230) and, when due, the checkpoint objective's sums
    int fl = 0;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (real[e]) {
        if (m_entry(a[e], w32) < 0.0) fl |= 1;
        if (!isfinite(a[e])) fl |= 2;
      }
    {
      const unsigned long long b1 = __ballot(fl & 1), b2 = __ballot(fl & 2);
      if (lane == 0) flw[w] = (b1 ? 1 : 0) | (b2 ? 2 : 0);
    }
    if (RC ? r_ckpt : S.ckpt_pending) {
      double sd = 0.0, l1 = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (real[e]) {
          sd += one_minus(rows[e] == cols[e], wv[e], w32) * z[e];
          l1 += fabs(wv[e]);
        }
      const double ld = tid < di ? log(fabs(piv[tid])) : 0.0;
      if constexpr (W32) {
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (real[e]) l1img[rows[e] * di + cols[e]] = fabsf((float)wv[e]);
      }
      sd = wave_sum(sd);
      l1 = wave_sum(l1);
      const double lds = wave_sum(ld);
      if (lane == 0) {
        red[0][w] = sd;
        red[1][w] = l1;
        red[2][w] = lds;
      }
    }
    __syncthreads();

    // ---- control (step.hip control_kernel; linear.py:230-241, 279-331): checkpoint slots and
    // flagged slots on thread 0 (small_control), the plain step by every thread
    SS_MARK(3)  // domain flags and checkpoint sums, barrier
    int fl_all = 0;
    if (RC)
#pragma unroll
      for (int x = 0; x < NW; ++x) fl_all |= flw[x];
    int act;
    bool norms, more;
    double lr_a, lr_b, bc1, bc2;
    if (!RC || r_ckpt || fl_all) {
      if constexpr (W32) {  // numpy's float32 np.abs(W).sum() (one chunk: d * d <= 1024)
        if (tid == 0 && (RC ? r_ckpt : S.ckpt_pending)) {
          red[1][0] = (double)np_pairwise([&](int64_t f) { return l1img[f]; }, 0, (int64_t)di * di);
          for (int x = 1; x < NW; ++x) red[1][x] = 0.0;
        }
      }
      if (tid == 0)
        small_control<NW>(cp, S, ctl, red, nred, flw, ckpt, ckpt_cap, bc1n, bc2n, TCC ? tsc : nullptr, next_ck);
      __syncthreads();
      act = ctl.act;
      norms = ctl.norms != 0;
      more = ctl.run != 0;
      lr_a = ctl.lr_a;
      lr_b = ctl.lr_b;
      bc1 = ctl.bc1;
      bc2 = ctl.bc2;
      r_iter = S.iter;
      r_slots = S.slots;
      r_lr = S.lr;
      r_ckpt = S.ckpt_pending;
      r_wrun = S.warm_run;
      r_next = next_ck;
    } else {  // small_control's ACT_STEP branch, state in registers
      const int64_t it = r_iter + 1;
      const bool at_ck = it == r_next;  // (it % checkpoint == 0)
      if (at_ck) r_next += c_checkpoint;
      r_ckpt = (at_ck || it == c_max_iter) ? 1 : 0;
      r_wrun = r_wrun < 2 ? r_wrun + 1 : 2;
      if (tid == 0) {
        if (r_slots == 0) S.t0 = __builtin_amdgcn_s_memrealtime();
        S.slots = r_slots + 1;
        S.warm_valid = 1;
        S.warm_run = r_wrun;
        S.flags = 0;
        S.bc1 = bc1n;
        S.bc2 = bc2n;
        S.lr_a = r_lr;
        S.iter = it;
        S.action = ACT_STEP;
        S.ckpt_pending = r_ckpt;
        next_ck = r_next;
      }
      r_slots += 1;
      r_iter = it;
      act = ACT_STEP;
      norms = r_ckpt != 0;
      more = true;
      lr_a = r_lr;
      lr_b = 0.0;
      bc1 = bc1n;
      bc2 = bc2n;
    }
    SS_MARK(4)  // the controller (thread 0 and a barrier on checkpoint / flagged slots)
    if (act == ACT_NOOP) break;  // terminal: nothing of this slot is applied
    if (act == ACT_HALVE) warm = 1;  // W turns back: the last two inverses do not extrapolate

    // ---- G_obj -> Adam -> update (linear.py:248, 138-163, 275-276), or the line search's
    // revert / halving with the last step's direction recomputed from m, v (step.hip)
    double qf[NORM_FIELDS];
#pragma unroll
    for (int f = 0; f < NORM_FIELDS; ++f) qf[f] = f == NF_WMIN ? INFINITY : 0.0;
    if (RC && act == ACT_STEP) {
      // straight-line over the lane's E elements (selects, no per-element branches), so that
      // the four elements' division and square-root chains interleave: one wave per SIMD has no
      // other wave to hide their latency (d = 20: 3762 -> 2839 cycles a slot in this phase)
      double gs[E], gl1[E], gh[E], gi[E], gtr[E], gob[E], mm[E], vx[E], gd[E], wn[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double wo = wv[e];
        const double mt = m_entry(a[e], w32);
        gs[e] = c_zscale * z[e];
        const double sg = sgn(wo);
        gl1[e] = c_mu_l1 * sg;
        gh[e] = h_term(wo, mt, w32);
        double g = gs[e] + gl1[e];
        g = g + gh[e];
        gi[e] = has_inc ? incv[e] * sg : 0.0;
        g = has_inc ? g + gi[e] : g;
        gtr[e] = 0.0;
        if constexpr (TCC) {  // Gobj + weight * trek_grad (linear.py:257-258), step.hip's order
          if (tc.mode == 2 && tcc_ran) {
            gtr[e] = tccb::tcc_grad_elem<TNB, TBS>(TL, di, rows[e], cols[e], wo, tc.m, tc.weight);
            g = g + gtr[e];
          }
        }
        gob[e] = g;
        mm[e] = mv[e] * c_beta1 + c_c1 * g;
        vx[e] = vv[e] * c_beta2 + c_c2 * (g * g);
      }
      double mh[E], vh[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        mh[e] = mm[e] / bc1;
        vh[e] = vx[e] / bc2;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) vh[e] = sqrt(vh[e]) + 1e-8;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        gd[e] = mh[e] / vh[e];
        double x = wv[e] - lr_a * gd[e];
        if (w32) x = f32r(x);  // W -= lr * grad into a float32 W (linear.py:275)
        wn[e] = has_exc ? x * excv[e] : x;
      }
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (real[e]) {
          mv[e] = mm[e];
          vv[e] = vx[e];
          wv[e] = wn[e];
        }
      if (norms) {
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (real[e]) {
            qf[NF_GOBJ] += gob[e] * gob[e];
            qf[NF_GSCORE] += gs[e] * gs[e];
            qf[NF_GDAG] += gh[e] * gh[e];
            qf[NF_GL1] += gl1[e] * gl1[e];
            qf[NF_GINC] += gi[e] * gi[e];
            qf[NF_GTREK] += gtr[e] * gtr[e];
            qf[NF_GSTEP] += gd[e] * gd[e];
            qf[NF_W2] += wn[e] * wn[e];
            qf[NF_WMAX] = fmax(qf[NF_WMAX], fabs(wn[e]));
            if (wn[e] != 0.0) qf[NF_WMIN] = fmin(qf[NF_WMIN], fabs(wn[e]));
          }
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!real[e]) continue;
        const double wo = wv[e];
        if (act == ACT_STEP) {  // (DS = 64: per element, the form above spills there)
          const double mt = m_entry(a[e], w32);
          const double gs = c_zscale * z[e];
          const double sg = sgn(wo);
          const double gl1 = c_mu_l1 * sg;
          const double gh = h_term(wo, mt, w32);
          double gobj = gs + gl1;
          gobj = gobj + gh;
          double gi = 0.0;
          if (has_inc) {
            gi = minc[(int64_t)rows[e] * D + cols[e]] * sg;
            gobj = gobj + gi;
          }
          const double mm = mv[e] * c_beta1 + c_c1 * gobj;
          const double vx = vv[e] * c_beta2 + c_c2 * (gobj * gobj);
          const double mh = mm / bc1;
          const double vh = vx / bc2;
          const double gd = mh / (sqrt(vh) + 1e-8);
          double wn = wo - lr_a * gd;
          if (w32) wn = f32r(wn);
          if (has_exc) wn = wn * mexc[(int64_t)rows[e] * D + cols[e]];
          mv[e] = mm;
          vv[e] = vx;
          wv[e] = wn;
          if (norms) {
            qf[NF_GOBJ] += gobj * gobj;
            qf[NF_GSCORE] += gs * gs;
            qf[NF_GDAG] += gh * gh;
            qf[NF_GL1] += gl1 * gl1;
            qf[NF_GINC] += gi * gi;
            qf[NF_GSTEP] += gd * gd;
            qf[NF_W2] += wn * wn;
            qf[NF_WMAX] = fmax(qf[NF_WMAX], fabs(wn));
            if (wn != 0.0) qf[NF_WMIN] = fmin(qf[NF_WMIN], fabs(wn));
          }
          continue;
        }
        const double gd = (mv[e] / bc1) / (sqrt(vv[e] / bc2) + 1e-8);
        if (act == ACT_HALVE) {  // (float32 W: each in-place update rounds, linear.py:235, 239)
          double wn = wo + lr_a * gd;
          if (w32) wn = f32r(wn);
          wn = wn - lr_b * gd;
          wv[e] = w32 ? f32r(wn) : wn;
        } else {
          const double wn = wo + lr_a * gd;
          wv[e] = w32 ? f32r(wn) : wn;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (real[e]) {
        if (!ONE) Wimg[rows[e] * SW + cols[e]] = wv[e];
        if (rows[e] == cols[e]) wdiag[rows[e]] = wv[e];
        IWimg[rows[e] * SI + cols[e]] = one_minus(rows[e] == cols[e], wv[e], w32);
      }
    if (norms) {
#pragma unroll
      for (int f = 0; f < NORM_FIELDS; ++f) {
        const double x = f == NF_WMAX ? wave_max(qf[f]) : (f == NF_WMIN ? wave_min(qf[f]) : wave_sum(qf[f]));
        if (lane == 0) nred[f][w] = x;
      }
    }
    __syncthreads();
    SS_MARK(5)  // G_obj, Adam, update (and the checkpoint norms), barrier
    if (!more) break;
  }
  SS_END();

  // write back: the state, this lane's elements, the pending checkpoint step's norms
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (real[e]) {
      const int64_t idx = (int64_t)rows[e] * D + cols[e];
      Wg[idx] = wv[e];
      mg[idx] = mv[e];
      vg[idx] = vv[e];
    }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    pstore[rows[e] * DS + cols[e]] = p1[e];
    pstore[DS * DS + rows[e] * DS + cols[e]] = p2[e];
  }
  if constexpr (TCC) {
    if (tid < 10) tc.scal[tid] = tsc[tid];
    for (int e = tid; e < 2 * (int)pr->d; e += NT) {
      tc.vprev[e] = tvp[e];
      tc.uprev[e] = tup[e];
    }
  }
  if (tid == 0) {
    carry[NORM_FIELDS] = (double)warm;
    if (S.ckpt_pending)
      for (int f = 0; f < NORM_FIELDS; ++f) {
        double x = f == NF_WMIN ? INFINITY : 0.0;
#pragma unroll 1
        for (int y = 0; y < NW; ++y)
          x = f == NF_WMAX ? fmax(x, nred[f][y]) : (f == NF_WMIN ? fmin(x, nred[f][y]) : x + nred[f][y]);
        carry[f] = x;
      }
    *stg = S;
  }
}

}  // namespace

#ifdef MIDAGMA_KSTAMPS
// the phase sums of the small loop since the last call (then zeroed): [0..5], [7..9] shader-clock
// cycles per phase, [6] Gauss-Jordan slots, [12] slots, [13] real-time (100 MHz) span of the launches
extern "C" int midagma_debug_small_stamps(unsigned long long* out) {
  const size_t bytes = 16 * sizeof(unsigned long long);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_small_stamps), bytes) != hipSuccess) return -1;
  static const unsigned long long zero[16] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_small_stamps), zero, bytes) != hipSuccess) return -1;
  return 0;
}
#endif

// d <= 64 (DS = 64: single-buffered images, 16 waves; MIDAGMA_EXP_SMALL64=0 keeps 32 < d <= 64 on
// the graph-replayed slots)
int small_block(int64_t d) {
  static const bool s64 = knob("MIDAGMA_EXP_SMALL64", 1) != 0;
  return d <= 16 ? 16 : (d <= 32 ? 32 : (d <= 64 && s64 ? 64 : 0));
}

void launch_small_minimize(const Params* pr, State* st, double* W, double* m, double* v, const double* covs,
                           const double* minc, const double* mexc, const double* bc_table, CkptRec* ckpt,
                           int64_t ckpt_cap, double* carry, double* pstore, int64_t d, int64_t n_slots,
                           hipStream_t stream, const SmallTcc* tcc, bool w32) {
  const int ds = small_block(d);
  if (ds == 0) throw std::invalid_argument("small_minimize: d > 64");
  if (tcc && ds > 32) throw std::invalid_argument("small_minimize: the TCC regularizer needs d <= 32");
  if (tcc && w32) throw std::invalid_argument("small_minimize: float32 W with TCC runs on the graph path");
  // d <= 20 on DS = 32: the one-wave 5 x 5 body (d=20: 10.4k -> 11.7k steps/s; experiment knob
  // MIDAGMA_EXP_TCC_BS5=0: NB = 16, 4 x 4)
  const bool bs5 = tcc && ds == 32 && d <= 20 && knob("MIDAGMA_EXP_TCC_BS5", 1) != 0;
  const SmallTcc tc = tcc ? *tcc : SmallTcc{};
#define MIDAGMA_SMALL(DS_, NW_, TCC_, W32_)                                                                \
  hipLaunchKernelGGL((small_minimize_kernel<DS_, NW_, TCC_, W32_>), dim3(1), dim3(64 * NW_), 0, stream, pr, st, W, \
                     m, v, covs, minc, mexc, bc_table, ckpt, ckpt_cap, carry, pstore, n_slots, tc)
  // one wave per 16 x 16 tile
  if (ds == 16) {
    if (tcc)
      MIDAGMA_SMALL(16, 1, 4, false);
    else if (w32)
      MIDAGMA_SMALL(16, 1, 0, true);
    else
      MIDAGMA_SMALL(16, 1, 0, false);
  } else if (ds == 32) {
    if (bs5)
      MIDAGMA_SMALL(32, 4, 5, false);
    else if (tcc)
      MIDAGMA_SMALL(32, 4, 4, false);
    else if (w32)
      MIDAGMA_SMALL(32, 4, 0, true);
    else
      MIDAGMA_SMALL(32, 4, 0, false);
  } else if (w32) {
    throw std::invalid_argument("small_minimize: a float32 W with 32 < d <= 64 runs on the graph path");
  } else {
    MIDAGMA_SMALL(64, 16, 0, false);
  }
#undef MIDAGMA_SMALL
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
