// Shared definitions for the MI355X (gfx950) DAGMA inner-solver kernels.
//
// Layout in HBM: every d x d matrix is stored row-major with leading dimension
// D = round_up(d, 64), so 64 x 64 tiles are aligned and the f64 MFMA tile
// kernels never need edge guards.  Padding is zero for W/m/v/g/cov and the
// identity for the log-det work matrix, which keeps the padded block of the
// inverse equal to I and its pivots equal to 1 (log 1 = 0).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "status.h"

namespace midagma {

constexpr int TILE = 64;          // tile edge of every blocked kernel
constexpr int NTHREADS = 256;     // 4 waves of 64 lanes
constexpr int NRED = 256;         // fixed number of partial-sum slots (deterministic reduction)

// LDS row strides (in doubles) that make the MFMA operand reads conflict-free:
// the f64 16x16x4 MFMA reads A[m0 + (lane&15)][k0 + (lane>>4)] and
// B[k0 + (lane>>4)][n0 + (lane&15)]; with ds_read_b64 a 32-lane group touches
// rows {0..15} x k {0,1}.  [m][k] images need stride = 2 mod 32, [k][n] images
// need stride = 16 mod 32.
constexpr int SA = 66;            // operand image stored [m][k]
constexpr int SB = 80;            // operand image stored [k][n] (or [k][m])

enum Action : int32_t { ACT_NOOP = 0, ACT_STEP = 1, ACT_HALVE = 2, ACT_REVERT = 3 };

// Per-minimize constants, uploaded once per call (linear.py:165-175, 217-222).
struct Params {
  double mu, s, lambda1, tol, beta1, beta2, c1, c2;  // c1 = 1 - beta1, c2 = 1 - beta2 (host)
  double mu_l1;       // mu * lambda1, host-rounded as the reference (linear.py:248)
  double zscale;      // G_score = zscale * Z + cscale * cov
  double cscale;
  double score_scale; // checkpoint score = score_scale * sum(dif * Z) (+ logistic loss term)
  double logit_scale; // 1/n for the logistic loss partial
  double d_log_s;     // d * log(s), host-rounded (linear.py:114)
  int64_t max_iter, checkpoint, d, D, ld_table;
  int32_t has_inc, has_exc, logistic;
  int32_t w32;        // dtype=np.float32: W is float32 in the reference (f32r below)
  double trek_weight;  // PST trek regularizer (linear.py:257-258, 131-133): weight,
  int32_t trek_mode;   //   0 off, 1 'log' (value at checkpoints), 2 'opt' (+ gradient every step)
  int32_t pad2_;
};

// Device-resident solver state: written only by the 1-workgroup controller
// kernel, read by every other kernel (kernel boundaries give visibility).
struct State {
  int64_t iter;          // Adam steps applied so far
  int64_t halvings;
  int64_t slots;         // slots the controller has seen (diagnostics)
  int64_t n_ckpt;
  int32_t status;
  int32_t ckpt_pending;  // objective of the current W is due this slot
  int32_t early_stop;
  int32_t action;        // decision for this slot's fused update
  double lr;             // current learning rate
  double lr_a, lr_b;     // HALVE: W += lr_a*g; W -= lr_b*g.  STEP: lr_a = lr
  double bc1, bc2;       // 1 - beta^it from the host table (bit-exact with Python)
  double obj_prev;
  double obj_last, score_last, h_last, l1_last;
  int32_t flags;         // bit0: inverse has an entry < 0 after +1e-16; bit1: non-finite
  int32_t warm_valid;    // Pstore holds the diagonal-block inverses of the previous slot
  int32_t warm_run;      // consecutive slots of this call whose outer-block inverses are stored (cap 2)
  uint64_t t0;           // device real-time clock (100 MHz) at the call's first slot
};

// One checkpoint record: the numeric fields of the reference's `minimize.checkpoint` event
// (linear.py:290-326).  W statistics are of W after the checkpoint step; the gradient norms
// are of that step (linear.py:262-273), as the reference computes them.
struct CkptRec {
  int64_t iter;
  double obj, score, h, lr, l1;
  double w_norm, max_abs_w, min_abs_w_nonzero;
  double grad_raw_norm, grad_step_norm, grad_score_norm, grad_dag_norm, grad_l1_norm, grad_inc_norm;
  double elapsed;  // seconds from the call's first slot to this record (device real-time clock)
  double reg_trek_value, grad_trek_norm;  // trek regularizer value at W, ||weight * trek grad||
};

// Per-workgroup partials the fused update leaves on a checkpoint step (sums of squares, then
// max |W| and min nonzero |W|), reduced by the next slot's controller.
constexpr int NORM_FIELDS = 10;  // sums of squares first, then the two extrema
enum NormField : int { NF_GOBJ = 0, NF_GSCORE, NF_GDAG, NF_GL1, NF_GINC, NF_GTREK, NF_GSTEP, NF_W2, NF_WMAX, NF_WMIN };

__host__ __device__ inline int64_t round_up64(int64_t x) { return (x + 63) / 64 * 64; }

// dtype=np.float32 (reference linear.py:29, 408, 429): Id and W are float32, so numpy rounds
// every array operation on them to float32 while cov and the gradients stay float64.  W is kept
// in float64 buffers holding float32 values, and each float32 operation is emulated as the
// float64 operation rounded to float32 (exact: 53 >= 2 * 24 + 2, so the double rounding of +, -,
// * is innocuous).
__host__ __device__ inline double f32r(double x) { return (double)(float)x; }
// one entry of s I - W o W as linear.py:226 forms it (float32: s * Id - W * W in float32)
__host__ __device__ inline double sw_entry(bool diag, double s, double w, bool w32) {
  if (!w32) return (diag ? s : 0.0) - w * w;
  const double ww = f32r(w * w);
  return diag ? f32r(f32r(s) - ww) : -ww;
}
// one entry of I - W (linear.py:244; float32: Id - W rounds the diagonal's 1 - w)
__host__ __device__ inline double one_minus(bool diag, double w, bool w32) {
  const double v = (diag ? 1.0 : 0.0) - w;
  return (w32 && diag) ? f32r(v) : v;
}
// the inverse's entry as linear.py:226, 248 use it: M = inv + 1e-16 (float32: the float32
// inverse, modelled as the float64 one rounded, plus 1e-16 in float32)
__host__ __device__ inline double m_entry(double inv, bool w32) {
  return w32 ? f32r(f32r(inv) + f32r(1e-16)) : inv + 1e-16;
}
// 2 W o M^T (float32: a float32 product)
__host__ __device__ inline double h_term(double w, double mt, bool w32) {
  return w32 ? f32r((2.0 * w) * mt) : (2.0 * w) * mt;
}

}  // namespace midagma

#define HIP_TRY(expr)                                                     \
  do {                                                                    \
    hipError_t _e = (expr);                                               \
    if (_e != hipSuccess) {                                               \
      throw ::midagma::HipError(_e, #expr, __FILE__, __LINE__);           \
    }                                                                     \
  } while (0)
