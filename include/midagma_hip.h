/*
 * midagma_hip.h -- C ABI of the MI355X-native DAGMA inner solver.
 *
 * The reference (fbleile/midagma) has no native code and no FFI: its hot path
 * is the Python method `DagmaLinear.minimize` (src/dagma/linear.py:165-333)
 * with helpers `_score` (70-94), `_h` (97-116), `_func` (118-135) and
 * `_adam_update` (138-163), reading object state set by `fit()`
 * (linear.py:406-429).  Each entry point below replaces one of those Python
 * call sites; the ctypes binding that makes them a drop-in lives in
 * `midagma_amd/_lib.py` and is shown in INTEGRATION.md.
 *
 * Conventions
 *   - plain C types only; host arrays are caller-owned, C-contiguous float64;
 *     device pointers (the *_dev entry points, midagma_bind_zbuf) are borrowed.
 *   - every function returns MIDAGMA_OK (0) or a negative error code; the
 *     message is available from midagma_last_error(solver) (or (NULL) for
 *     errors raised before a solver exists).  No C++ exception crosses the ABI.
 *   - a solver is not thread-safe; one host thread drives it.
 */
#ifndef MIDAGMA_HIP_H_
#define MIDAGMA_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIDAGMA_ABI_VERSION 11

/* return codes */
#define MIDAGMA_OK 0
#define MIDAGMA_E_HIP (-1)      /* HIP runtime failure            -> RuntimeError        */
#define MIDAGMA_E_SINGULAR (-2) /* non-finite inverse (scipy getrf info>0) -> LinAlgError */
#define MIDAGMA_E_ARG (-3)      /* bad argument / shape, non-finite input (scipy check_finite) -> ValueError */
#define MIDAGMA_E_STATE (-4)    /* call out of sequence            -> RuntimeError        */

/* loss_type (linear.py:52-53) and score mode */
#define MIDAGMA_LOSS_L2 0
#define MIDAGMA_LOSS_LOGISTIC 1
#define MIDAGMA_MODE_COV 0  /* cov = X^T X / n precomputed (linear.py:428); l2 only   */
#define MIDAGMA_MODE_DATA 1 /* X row shard resident; per-step X^T(...) + all-reduce */

/* minimize outcome (midagma_result.status) */
#define MIDAGMA_ST_RUNNING 0
#define MIDAGMA_ST_DONE 1         /* max_iter or tolerance      -> (W, True)  linear.py:333, 330 */
#define MIDAGMA_ST_FAILED 2       /* out of domain, iter 1 or s<=0.9 -> (W, False) linear.py:233   */
#define MIDAGMA_ST_LR_UNDERFLOW 3 /* lr <= 1e-16               -> (W, True)  linear.py:237-238   */
#define MIDAGMA_ST_SINGULAR 4

typedef struct midagma_solver midagma_solver;

typedef struct {
  int64_t iters;         /* Adam steps applied (pbar.update total, linear.py:332)   */
  int64_t halvings;      /* lr halvings in the domain line search (linear.py:236)   */
  int64_t slots;         /* device step slots consumed (diagnostics)                */
  int64_t n_checkpoints; /* objective evaluations (linear.py:279-280)               */
  int32_t status;        /* MIDAGMA_ST_*                                            */
  int32_t early_stop;    /* 1 if |dobj/obj| <= tol ended the call (linear.py:328)   */
  double lr_final;
  double obj_last, score_last, h_last, l1_last;
} midagma_result;

/* The numeric fields of the reference's `minimize.checkpoint` event (linear.py:290-326):
 * obj_total, score_datafit, reg_dag_value (h), lr, w_abs_sum (l1), W statistics after the
 * step, and the norms of the checkpoint step's gradients (linear.py:262-273). */
typedef struct {
  int64_t iter;
  double obj, score, h, lr, l1;
  double w_norm, max_abs_w, min_abs_w_nonzero;
  double grad_raw_norm, grad_step_norm, grad_score_norm, grad_dag_norm, grad_l1_norm, grad_inc_norm;
  double elapsed; /* seconds since the call's first device slot */
  double reg_trek_value, grad_trek_norm; /* PST trek regularizer (0 when none) */
} midagma_ckpt;

int midagma_abi_version(void);
int midagma_device_count(int* n);
const char* midagma_last_error(const midagma_solver* s);

/* Replaces DagmaLinear.__init__ + the data part of fit() (linear.py:25-67, 406-429).
 * d: number of nodes; device: HIP ordinal; stream: hipStream_t to run on, or NULL
 * for a solver-owned stream (required for the graph-replayed minimize loop). */
int midagma_create(midagma_solver** out, int loss, int mode, int64_t d, int device, void* stream);
void midagma_destroy(midagma_solver* s);
void* midagma_stream(midagma_solver* s);
int64_t midagma_padded_dim(const midagma_solver* s);

/* cov = X^T X / n (linear.py:428), host d x d with leading dimension ld. */
int midagma_set_cov(midagma_solver* s, const double* cov, int64_t ld);
/* mask_inc / mask_exc for the next minimize call (linear.py:217-222), host d x d or NULL. */
int midagma_set_masks(midagma_solver* s, const double* mask_inc, const double* mask_exc);
/* ABI 8: W's dtype in the reference's arithmetic (DagmaLinear(dtype=...), linear.py:29, 408, 429).
 * float32 != 0: the loop emulates numpy's float32 array operations on W and Id -- W rounded to
 * float32 after every in-place update (275, 235, 239), s*Id - W*W and Id - W in float32 (226, 244),
 * M = inv + 1e-16 and 2 W o M^T in float32 (226, 248) -- with the inverse itself in float64 (a
 * float32 getrf's bits cannot be reproduced).  Takes effect at the next minimize / begin. */
int midagma_set_w_float32(midagma_solver* s, int float32);
/* data mode: this rank's row shard of X (n_local x d, ld = d); n_global = rows over all ranks.
 * on_device != 0: X is a device pointer (copied). */
int midagma_set_data(midagma_solver* s, const double* X, int64_t n_local, int64_t n_global, int on_device);
/* data mode: zbuf <- X_k^T X_k (all-reduce it, then midagma_cov_from_zbuf(n): cov = zbuf / n). */
int midagma_data_gram(midagma_solver* s);
int midagma_cov_from_zbuf(midagma_solver* s, double n);
/* The solver's cov (d x d, ld) to the host: the `self.cov` attribute fit() keeps (linear.py:428)
 * when cov was built on the device from the ranks' shards. */
int midagma_get_cov(midagma_solver* s, double* out, int64_t ld);
/* ABI 7: fit()'s data preparation on the device (linear.py:406-428), for a device-resident or
 * row-sharded X in either score mode.  All on `stream` (a hipStream_t, NULL = default).
 * colsum_dev: out_dev[j] = sum_r X[r, j] (n x d, ldx; fixed summation order); returns after it
 *   is written.  Sharded: all-reduce it, then center with n_global.
 * center_dev: X[r, j] -= colsum_dev[j] / nrows in place (the l2 centring, linear.py:411); async.
 * gram: G_dev (d x d, ldg, device) = X^T X (linear.py:428) for X (n x d, ldx) in device memory
 *   (on_device != 0) or host memory, streamed in zero-padded row chunks through the 128 x 128
 *   FP64 MFMA GEMM, chunk sums in a fixed order; MIDAGMA_E_ARG if X holds inf/nan.  Returns
 *   after G is written.  Sharded: all-reduce G over ranks.
 * set_cov_dev: the solver's cov = G_dev / divisor (divisor = n, float(self.n) in linear.py:428),
 *   G_dev d x d (ldg) device memory complete before the call; MIDAGMA_E_ARG on inf/nan. */
int midagma_colsum_dev(const double* X, int64_t n, int64_t d, int64_t ldx, double* out_dev, void* stream);
int midagma_center_dev(double* X, int64_t n, int64_t d, int64_t ldx, const double* colsum_dev, double nrows,
                       void* stream);
int midagma_gram(const double* X, int64_t n, int64_t d, int64_t ldx, int on_device, double* G_dev, int64_t ldg,
                 void* stream);
int midagma_set_cov_dev(midagma_solver* s, const double* G_dev, int64_t ldg, double divisor);
/* ABI 7: the data-mode score all-reduce inside the library (linear.py:244-246 over row
 * shards).  comm_unique_id: RCCL's 128-byte ncclUniqueId (rank 0 makes it, the caller broadcasts
 * it, e.g. over torch.distributed).  comm_init: this solver joins an nranks communicator as `rank`;
 * from then on every captured slot sums the score partial over the ranks (in place, on the solver
 * stream, between the GEMMs and the update), so midagma_minimize / midagma_run_slots drive a
 * multi-rank minimize from replayed graphs, and every host poll all-reduces (status, iters): a
 * divergent replica makes every rank fail with MIDAGMA_E_STATE instead of hanging.  Needs a ring
 * all-reduce for bit-identical replicas (NCCL_ALGO=Ring).  RCCL is loaded at run time (the copy in
 * the process, else ROCm's): MIDAGMA_E_STATE when absent.  comm_ranks: 0 without a communicator. */
int midagma_comm_unique_id(void* out, int64_t cap); /* returns 128 (the id's size) */
int midagma_comm_init(midagma_solver* s, const void* id, int64_t id_len, int nranks, int rank);
int midagma_comm_ranks(const midagma_solver* s);
/* the score partial of midagma_score_partial (or data_gram) summed over the communicator, on the
 * solver stream: `_score` in data mode between score_partial and score_finish */
int midagma_comm_allreduce_zbuf(midagma_solver* s);
/* The d x d (+ tail) device buffer that carries the per-step score partial Z_k.
 * Bind an external buffer (e.g. a torch tensor that torch.distributed all-reduces). */
int64_t midagma_zbuf_len(const midagma_solver* s);
int midagma_bind_zbuf(midagma_solver* s, void* dev_ptr, int64_t len);

/* ABI 11: data mode on several devices from ONE process ("one host thread drives
 * all its devices ... the Python side stays single-process"), behind the reference's single-process
 * DagmaLinear.fit(X) (linear.py:335-351; the per-step score gradient 244-246 summed over row shards).
 * A group holds one data-mode solver per entry of devices[] (member k holds row shard k of X); the
 * score partial is summed over the members inside every captured slot, between the GEMMs and the
 * update:
 *   - devices all distinct: one RCCL communicator per member from ncclCommInitAll over devices[];
 *     each member's slot graphs carry its all-reduce and are replayed by a library thread of its
 *     own, with the (status, iters) agreement all-reduce at every poll (midagma_comm_init's
 *     protocol).  All members finish their setup (begin, graph capture) before any collective is
 *     issued; a member that fails before that point fails the call on every member.
 *   - flags & MIDAGMA_GROUP_EMULATE (every entry of devices[] the same device; tests on one GPU): no
 *     RCCL.  The members' slots are captured as ONE graph over their streams with a fixed-order
 *     device sum of the partials (member 0 + member 1 + ...) in place of the all-reduce, and the
 *     calling thread replays it (test strategy 4).
 * Members are ordinary data-mode solvers (midagma_group_member, owned by the group): set_cov,
 * set_masks, set_w_float32, set_trek*, h, score_partial / score_finish and checkpoints act on one
 * member; apply the loop's settings (cov, masks, dtype, trek) to every member. */
#define MIDAGMA_GROUP_EMULATE 1
typedef struct midagma_group midagma_group;
int midagma_group_create(midagma_group** out, int loss, int64_t d, const int* devices, int ndev, int flags);
void midagma_group_destroy(midagma_group* g);
const char* midagma_group_last_error(const midagma_group* g);
int midagma_group_size(const midagma_group* g);
int midagma_group_emulated(const midagma_group* g);
midagma_solver* midagma_group_member(midagma_group* g, int k);
/* host X (n x d row-major): member k gets rows [lo_k, hi_k) of the even split (the first n % ndev
 * members take one row more), with n_global = n.  MIDAGMA_E_ARG when n < ndev. */
int midagma_group_set_data(midagma_group* g, const double* X, int64_t n);
/* every member's score buffer (score_partial's or data_gram's partial) <- the sum over the members;
 * returns after it is written */
int midagma_group_allreduce_zbuf(midagma_group* g);
/* DagmaLinear.minimize over the group (arguments and result as midagma_minimize).  W: host d x d,
 * in/out, from member 0 after the members were checked to end with the same W bits, status,
 * iterations and halvings (else MIDAGMA_E_STATE: the replicas diverged). */
int midagma_group_minimize(midagma_group* g, double* W, double mu, int64_t max_iter, double s_dom, double lr,
                           double tol, double beta1, double beta2, double lambda1, int64_t checkpoint,
                           midagma_result* res);

/* Replaces DagmaLinear.minimize(W, mu, max_iter, s, lr, tol, beta_1, beta_2)
 * (linear.py:165-333) with trek_reg disabled.  W: host d x d, in/out. */
int midagma_minimize(midagma_solver* s, double* W, double mu, int64_t max_iter, double s_dom, double lr,
                     double tol, double beta1, double beta2, double lambda1, int64_t checkpoint,
                     midagma_result* res);

/* The same loop one step at a time, for an external all-reduce between the halves
 * (data mode on several ranks):  begin; { step_partial; allreduce(zbuf); step_finish }*; end. */
int midagma_begin(midagma_solver* s, const double* W, double mu, int64_t max_iter, double s_dom, double lr,
                  double tol, double beta1, double beta2, double lambda1, int64_t checkpoint);
int midagma_step_partial(midagma_solver* s);
/* enqueue n whole slots (part 1 + part 2); midagma_sync waits.  Without host polling,
 * except in cov mode with the blocked inverse (d > 64, D = 128 or a multiple of 128 from 256), where the host picks the fast or
 * the GJ path per batch (one sync per batch of <= 64 slots). */
int midagma_run_slots(midagma_solver* s, int64_t n);
int midagma_sync(midagma_solver* s);
/* Diagnostics: average device time (hipEvents on the solver stream, `reps` launches each)
 * of the slot's parts: [0] build (sI-WoW)^T, [1] GJ inverse, [2] score GEMM(s), [3] whole
 * slot (GJ path), [4] data-mode X(I-W) GEMM, [5] data-mode X^T Y GEMM, [6] cov-mode fast
 * blocked inverse, [7] whole fast slot ([6], [7]: 0 if not available, -1 if the fast path
 * handed back).  ms_out holds 8 doubles.  Advances the state by up to 3 reps + 1 slots. */
int midagma_profile_parts(midagma_solver* s, int reps, double* ms_out);
int midagma_step_finish(midagma_solver* s);
int midagma_poll(midagma_solver* s, midagma_result* res); /* synchronizes */
int midagma_end(midagma_solver* s, double* W, midagma_result* res);
int64_t midagma_checkpoints(midagma_solver* s, midagma_ckpt* out, int64_t cap);

/* The PST trek regularizer of notreks.py (pst / trek_value_grad) inside the loop
 * (linear.py:251-258, 131-133).  seq: 0 exp, 1 inv, 2 log, 3 binom; agg: 0 mean, 1 sum,
 * 2 max, 3 lse; mode: 0 off, 1 'log' (value at checkpoints only), 2 'opt' (value and
 * weight * gradient every step, weight * value in the checkpoint objective); K: log series
 * terms (binom: ignored, the exponent is d as in the reference); pairs: m (i, j) int64. */
int midagma_set_trek(midagma_solver* s, int seq, int agg, int mode, double weight, double eps_inv, int64_t K,
                     const int64_t* pairs, int64_t m);
/* The TCC trek regularizer (notreks.py:291-395 as trek_value_grad:667-706 calls it in the loop:
 * spectral penalty, 'approx_trek_graph', Perron pairs) inside the loop; mode as above; w: the
 * multiplier of the pair indicator S; eps: the reference's stabiliser (1e-12). */
int midagma_set_trek_tcc(midagma_solver* s, int mode, double weight, double w, double eps, const int64_t* pairs,
                         int64_t m);
/* trek_value_grad(W, tr) (notreks.py): value and, in 'opt' mode, the gradient (G nullable, d x d;
 * zeros in 'log' mode, as the reference returns). */
int midagma_trek(midagma_solver* s, const double* W, double* value, double* G);

/* Replaces DagmaLinear._h (linear.py:97-116): h and G_h = 2 W o inv(sI - W o W)^T (G nullable). */
int midagma_h(midagma_solver* s, const double* W, double s_dom, double* h, double* G);
/* Replaces DagmaLinear._score (linear.py:70-94) in cov mode (l2). */
int midagma_score(midagma_solver* s, const double* W, double* loss, double* G);
/* _score in data mode: partial into zbuf (all-reduce it), then finish. */
int midagma_score_partial(midagma_solver* s, const double* W);
int midagma_score_finish(midagma_solver* s, double* loss, double* G);

/* DagmaMLP.h_func kernel (nonlinear.py:68-86) on device memory:
 * Mt = (sI - A)^{-T} (ldm) and logdet_dev[0] = log|det(sI - A)| for A (d x d, lda).
 * Enqueued on `stream`, no host synchronization. */
int midagma_logdet_inv_dev(const double* A, int64_t d, int64_t lda, double s_dom, double* logdet_dev,
                           double* Mt_dev, int64_t ldm, void* stream);

/* Linear-SEM samples on the GPU (replaces utils.simulate_linear_sem, utils.py:99-172):
 * rows [row0, row0 + n_rows) of X (row-major, ld = ldx >= d, device memory) for the weighted
 * DAG W (host, d x d row-major, W[p, j] = weight of edge p -> j):
 *   x_j = sum_{p in pa(j)} W[p, j] x_p + z_j   (sem_type 0 gauss, 1 exp, 2 gumbel, 3 uniform)
 *   x_j ~ Bernoulli(sigmoid(.)) (4 logistic),  x_j ~ Poisson(exp(.)) (5 poisson).
 * Noise: Philox4x32-10 keyed by `seed`, counter (row / 2, node, draw) -- row r's values are the
 * same whatever row0 / n_rows split generated it.  noise_scale: d scales or NULL (ones).
 * MIDAGMA_E_ARG if W has a cycle.  Enqueued on `stream`; returns after the rows are written. */
int midagma_sem_linear(const double* W, int64_t d, int64_t row0, int64_t n_rows, int sem_type,
                       const double* noise_scale, uint64_t seed, double* X_dev, int64_t ldx, void* stream);

/* One torch.optim.Adam step (single-tensor algorithm, L2 weight decay wd) on n doubles of
 * device memory, enqueued on `stream`; coefficients host-rounded as torch computes them:
 * step_size = lr / (1 - b1^t), w1 = 1 - b1, c2 = 1 - b2, bc2_sqrt = sqrt(1 - b2^t).
 * Skipped when gate != NULL and *gate < 0 (device scalar: DagmaNonlinear's h, nonlinear.py:216). */
int midagma_adam_step(double* p, const double* g, double* m, double* v, int64_t n, double step_size, double w1,
                      double beta2, double c2, double bc2_sqrt, double eps, double wd, const double* gate,
                      void* stream);

/* The same step with the per-step coefficients from a device table at a device step counter:
 * step_size = table[2 t], sqrt(1 - b2^t) = table[2 t + 1], t = *counter (graph-replayable);
 * midagma_counter_advance adds 1 to *counter on `stream`. */
int midagma_adam_step_table(double* p, const double* g, double* m, double* v, int64_t n, const double* table,
                            const int64_t* counter, double w1, double beta2, double c2, double eps, double wd,
                            const double* gate, void* stream);
int midagma_counter_advance(int64_t* counter, void* stream);
/* midagma_adam_step_table over k <= 8 tensors (host arrays of their device pointers and
 * sizes) in one launch. */
int midagma_adam_step_table_multi(int64_t k, double* const* p, const double* const* g, double* const* m,
                                  double* const* v, const int64_t* n, const double* table, const int64_t* counter,
                                  double w1, double beta2, double c2, double eps, double wd, const double* gate,
                                  void* stream);

/* The DagmaMLP tail of dims [d, m1, 1] (d * m1 <= 7936), fused on torch's device memory and
 * stream (replaces sigmoid -> LocallyConnected(d, m1, 1) -> squared residual sum in
 * nonlinear.py:99-104, 139-159 and their autograd backward; dagma/locally_connected.py:55-85).
 * scratch: midagma_mlp_tail_scratch(n, d, m1) doubles of device memory.
 * fwd: Z (n x d*m1 row-major, plus b1 per column when b1 is given) -> R = Xhat - X (n x d),
 * *ssq = sum R^2 (device).
 * bwd: *g = d loss / d ssq (device) -> dZ (n x d*m1), dw2 (d x m1), db2 (d) and, when db1 is
 * given, db1 = column sums of dZ (d*m1). */
int64_t midagma_mlp_tail_scratch(int64_t n, int64_t d, int64_t m1);
int midagma_mlp_tail_fwd(const double* Z, const double* b1, const double* w2, const double* b2, const double* X,
                         int64_t n, int64_t d, int64_t m1, double* R, double* scratch, double* ssq, void* stream);
/* The rest of the [d, m1, 1] DagmaMLP objective (nonlinear.py:68-86, 139-159, 198-206):
 * fc1_terms: A[i, j] = sum_m W1[j m1 + m, i]^2 (d x d, the log-det operand) and the |W1| partial
 * sums l1part (midagma_fc1_terms_parts(d) doubles); its backward dW1 = 2 W1 gA^T + gl1 sign(W1).
 * mlp_objective: *obj = mu (half_d log(inv_n *ssq) + lambda1 sum(l1part)) + *h, and its
 * backward from *g: *gssq, gl1part[*], *gh (ssq and gssq both NULL: only gl1part and gh).
 * All device pointers, on `stream`. */
int64_t midagma_fc1_terms_parts(int64_t d);
int midagma_fc1_terms(const double* W1, int64_t d, int64_t m1, double* A, double* l1part, void* stream);
int midagma_fc1_terms_bwd(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gscale,
                          const double* gl1part, const double* lin, int64_t nlin, double* dW1, void* stream);
/* h = -log|det(sI - A)| + d log s (DagmaMLP.h_func, nonlinear.py:68-86) into *h_dev and, when
 * Mt_dev is given, (sI - A)^-T (d x d, ldm) -- its gradient -- in four launches (build, GJ,
 * epilogue; the GJ on the 32-padded problem). */
int midagma_logdet_h_dev(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev, int64_t ldm,
                         void* stream);
/* The same, enqueued in midagma_logdet_h_parts(d) parts that must be issued in order (part 0:
 * build and prologue; parts 1 .. ceil(d/32): the Gauss-Jordan block steps; the last: h and
 * (sI - A)^-T), so a caller can interleave them with other work of its step (DagmaNonlinear's
 * side-stream log-det).  The parts of one h share a per-device workspace: one h at a time. */
int64_t midagma_logdet_h_parts(int64_t d);
int midagma_logdet_h_dev_part(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev,
                              int64_t ldm, void* stream, int64_t part);
/* ABI 6: the h log-det of consecutive DagmaNonlinear.minimize steps (nonlinear.py:206-217, 85-86)
 * with a warm start.  A handle holds the warm-start ring of one minimize call's A = sum fc1^2
 * (d <= 256; larger d always runs the Gauss-Jordan chain).  A fast step (exact = 0) inverts
 * (sI - A)^T by the product-form series from the last two steps' inverses and keeps the last
 * exact h when that inverse converged and is entrywise >= 0 (then sI - A is a nonsingular
 * M-matrix and h >= 0: the reference's h < 0 exit cannot fire); otherwise it runs the
 * Gauss-Jordan chain on the device and takes its h.  An exact step (exact = 1: the steps whose
 * objective the caller reads) always runs the chain.  Both write (sI - A)^-T to Mt and feed the
 * ring.  midagma_ldfast_reset starts a call (the first step then runs the chain).  Parts as
 * midagma_logdet_h_dev_part: issued in order on one stream; one step at a time per handle. */
typedef struct midagma_ldfast midagma_ldfast;
int midagma_ldfast_create(midagma_ldfast** out, int64_t d);
void midagma_ldfast_destroy(midagma_ldfast* h);
int midagma_ldfast_reset(midagma_ldfast* h);
int64_t midagma_ldfast_parts(const midagma_ldfast* h, int exact);
/* ABI 7: d (A is d x d) must equal the handle's d, else MIDAGMA_E_ARG. */
int midagma_ldfast_enqueue(midagma_ldfast* h, const double* A, int64_t d, int64_t lda, double s, double* h_dev,
                           double* Mt_dev, int64_t ldm, void* stream, int exact, int64_t part);
/* ABI 10: fast steps enqueued from now on also add 1 to *counter (device; null: off) at their
 * end, midagma_counter_advance's work in the end's launch, for a caller that skips the scalar
 * objective on those steps.  Exact steps never touch it. */
int midagma_ldfast_set_counter(midagma_ldfast* h, int64_t* counter);
/* gate-open (Gauss-Jordan) steps and fast steps since the last reset (diagnostics; syncs) */
int midagma_ldfast_stats(midagma_ldfast* h, int64_t* steps, int64_t* exact_steps);
/* ABI 6: the [d, m1, 1] objective with the scalar objective's backward folded into its consumers
 * (no mlp_sum / mlp_objective_bwd launches; bit-identical to the ABI-5 sequence): the tail forward
 * leaves its n row partials (part), the objective sums them and, with a counter, advances the
 * Adam table's step (counter += 1, nullable), the tail backward and the fc1 terms' backward take
 * gobj = d loss / d obj and derive d obj / d ssq, d h = gobj, d l1part = (gobj mu) lambda1. */
int midagma_mlp_tail_fwd_part(const double* Z, const double* b1, const double* w2, const double* b2, const double* X,
                              int64_t n, int64_t d, int64_t m1, double* R, double* part, void* stream);
int midagma_mlp_objective_part(const double* part, int64_t npart, const double* l1part, int64_t np, const double* h,
                               double mu, double lambda1, double half_d, double inv_n, double* obj, int64_t* counter,
                               void* stream);
int midagma_mlp_tail_bwd_obj(const double* Z, const double* b1, const double* w2, const double* R, const double* part,
                             const double* gobj, double mu, double half_d, double inv_n, int64_t n, int64_t d,
                             int64_t m1, double* dZ, double* dw2, double* db2, double* db1, double* scratch,
                             void* stream);
int midagma_fc1_terms_bwd_obj(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gobj, double mu,
                              double lambda1, const double* lin, int64_t nlin, double* dW1, void* stream);
/* ABI 9: one replayed DagmaNonlinear step of a [d, m1, 1] model closed in one launch
 * (nonlinear.py:198-236): the tail's dw2 / db2 / db1 sums from the chunk partials that
 * midagma_mlp_tail_bwd_obj leaves in scratch when dw2 = db2 = db1 = NULL, fc1's weight gradient
 * (midagma_fc1_terms_bwd_obj's arithmetic), the gated table Adam step of the four parameters
 * (params / exp_avg / exp_avg_sq: fc1.weight, fc1.bias, fc2.weight, fc2.bias;
 * midagma_adam_step_table_multi's arithmetic) and the next step's fc1 terms (A, l1part as
 * midagma_fc1_terms computes them, from the updated weights).  Bit-identical to those launches. */
int midagma_mlp_step(double* const* params, double* const* exp_avg, double* const* exp_avg_sq, int64_t n, int64_t d,
                     int64_t m1, const double* gA, const double* gobj, double mu, double lambda1, const double* lin,
                     int64_t nlin, const double* scratch, const double* table, const int64_t* counter, double w1,
                     double beta2, double c2, double eps, double wd, const double* gate, double* A, double* l1part,
                     void* stream);
int midagma_mlp_objective(const double* ssq, const double* l1part, int64_t np, const double* h, double mu,
                          double lambda1, double half_d, double inv_n, double* obj, void* stream);
int midagma_mlp_objective_bwd(const double* g, const double* ssq, int64_t np, double mu, double lambda1, double half_d,
                              double inv_n, double* gssq, double* gl1part, double* gh, void* stream);
int midagma_mlp_tail_bwd(const double* Z, const double* b1, const double* w2, const double* R, const double* g,
                         int64_t n, int64_t d, int64_t m1, double* dZ, double* dw2, double* db2, double* db1,
                         double* scratch, void* stream);
#ifdef __cplusplus
}
#endif

#endif /* MIDAGMA_HIP_H_ */
