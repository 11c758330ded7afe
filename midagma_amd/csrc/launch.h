// Host-side launchers for the kernels (all enqueue on the given stream, no sync,
// no allocation: safe to capture into a hipGraph).
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "knobs.h"

namespace midagma {

struct HipError : std::runtime_error {
  hipError_t code;
  HipError(hipError_t e, const char* what, const char* file, int line)
      : std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " at " + file + ":" +
                           std::to_string(line) + " (" + what + ")"),
        code(e) {}
};

struct GJWork {
  double* P;       // >= 2 x 32 x 32  (double-buffered inverse of the diagonal block)
  double* R;       // >= 2 x 32 x D   (row panels)
  double* C;       // >= 2 x D x 32   (column panels)
  double* pivlog;  // D  (log |pivot| per row, nullable)
  double* Pstore = nullptr;  // D x 32: last inverse of every diagonal block (warm starts), nullable
};

// --- gj.hip -----------------------------------------------------------------
void gj_setup_attributes();
// At = (s*I - f(X))^T on the logical d x d block, identity padding; f = x^2 if square.
// s is read from pr->s when pr != nullptr (graph-replayed slots), else the argument.
// IW (nullable, D x D): also writes I - X (identity padding).
void launch_build_at(const double* X, int64_t ldx, bool square, double* At, int64_t D, int64_t d, double s,
                     const Params* pr, const State* st, hipStream_t stream, double* IW = nullptr);
// In place: A <- inv(A) (unpivoted blocked Gauss-Jordan) on the D x D matrix at A with
// leading dimension lda (D multiple of 32), pivot logs into w.pivlog.
void launch_gj_inverse(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, hipStream_t stream);
// the same as its parts: the prologue, then block steps k = 0 .. D/32 - 1 in order
void launch_gj_prologue(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, hipStream_t stream);
// The end of a warm-started DagmaMLP log-det step (ldfast_post's work for a fast step, in the same
// workgroup after the gated chain): if the chain ran, h from its pivots and Mt and the warm-start
// ring slot from its inverse, else h = *hlast; then the ring state advances (st->slots counts the
// step: ldfast_resid_kernel opened it without the increment).  st null: no end.
struct LdfastEnd {
  const double* piv;
  int64_t d;
  double dls;
  double* h;
  double* Mt;
  int64_t ldm;
  int B;
  double* ring0;
  double* ring1;
  State* st;
  double* hlast;
  int64_t* counter;  // nullable: the Adam table's step counter, advanced by the end (+= 1)
};
// build_at (A given, not squared) + the whole Gauss-Jordan inverse in one workgroup, gated on st
// (bit-identical to launch_build_at + launch_gj_inverse; the rare fallback of a warm-started step),
// then `end` when end.st is set
void launch_gj_inverse_1wg(const double* X, int64_t ldx, double* At, int64_t D, int64_t d, double s, const GJWork& w,
                           const State* st, hipStream_t stream, const LdfastEnd& end = LdfastEnd{});
void launch_gj_step(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, int k, hipStream_t stream);

// A GEMM launch's arguments (launch_gemm's meaning), for launches that carry one beside other work.
enum GemmB : int;
struct GemmSpec {
  int64_t M, N, K;
  const double* A;
  int64_t lda;
  bool a_trans;
  const double* B;
  int64_t ldb;
  int bmode;  // GemmB
  double* C;
  int64_t ldc;
  int split;
  int64_t slice_stride;
  // launch_gemm_trail only: the fast slot's control folded into the launch (control.h
  // control_fold_tail; null ticket: a control launch follows instead)
  const Params* ctl_pr = nullptr;
  const double* ctl_table = nullptr;
  int* ctl_ticket = nullptr;
};

// --- blockinv.hip -----------------------------------------------------------
// product-form pass slots per outer block (buffers) and the passes of the fallback fast graph
// (the default fast graph runs 2: the extrapolated warm start converges in 2 almost always;
// from a warm start one Adam step old, 3 always converged in the default d=1000 fit)
constexpr int NM_PASSES = 4;
constexpr int NM_PASSES_RUN = 3;
constexpr int PART_STRIDE = 16384;  // doubles per pass: row partials of |Q| (B2 x B2/16, B2 <= 512)
struct BInvWork {
  double* Aalt;    // second D x D buffer (outer steps ping-pong)
  double* Pst;     // D x B2: the outer diagonal blocks' inverses of the slots with even /
  double* Pst1;    //   odd st->slots (the last two slots': the warm start extrapolates them)
  double* Y[2];    // B2 x B2 product-form iterates
  double* Q[2];
  double* P;       // B2 x B2 converged inverse of the current block
  double* part;    // (D / B2) x (NM_PASSES + 1) x PART_STRIDE row partials
  int* done;       // D / B2 convergence words
  // look-ahead residual (fast path, 32-tile trailing updates): block g's launches prepare block
  // g+1's R = I - S X0 instead of a residual launch of its own (B2 x B2 each; null: off)
  double* LW;      // A(g+1, g+1) X0(g+1)      (extra tiles of block g's first pass)
  double* LZ;      // A(G, g+1) X0(g+1)        (same launch)
  double* LPZ;     // P_g LZ                   (extra tiles of block g's panel launch)
  // (D / B2) x 256 ints: block g's counters for its series run inside trailing update g - 1
  // (launch_trail128_series; null: off)
  int* sync = nullptr;
};
// Outer block width of the two-level inverse (0: not available, use launch_gj_inverse).
int binv_block(int64_t D);
// The buffer launch_build_at must fill so that the inverse ends in Mt.
double* binv_build_target(double* Mt, int64_t D, const BInvWork& bw);
// Mt <- inv(A) for A in binv_build_target(Mt): two-level blocked Gauss-Jordan, diagonal
// blocks by the warm-started product form (fast; sets ST_NEED_GJ when it cannot) or by the
// 32-block Gauss-Jordan with pivots (slow).  The fast path also ORs reduce_check's domain
// flags into st->flags from the last outer step's outputs.
// passes: product-form pass launches per outer block on the fast path (2 covers the
// extrapolated warm start's usual residual, 3 the rest; an unconverged block hands back).
// fuse (nullable; fast path): a GEMM (EPI_STORE, split-K slices) that runs in the launch of the
// last outer step's 32 x 32 trailing update (gemm.hip, launch_gemm_trail); false is returned
// when that launch is not available for this D and the caller must launch the GEMM itself.
// tla (nullable; fast path, 128-tile trailing updates): the look-ahead across two streams
// (blocked_inverse_lookahead in blockinv.hip): a high-priority side stream and 2 K2 + 2 events.
struct TrailLookAhead {
  hipStream_t side;
  hipEvent_t* ev;
};
// resid0_done (fast path, B2 = 256): outer block 0's residual already ran in launch_build_resid0.
// ain0 (nullable; fast path): outer step 0 reads A from here instead of binv_build_target (the
// A^T that the previous slot's fused_update_at wrote; only read)
// slow_from (>= 0; fast path): outer blocks from slow_from on take the pivoted Gauss-Jordan (the
// TCC's shifted inverses: only the last block's Schur complement is near-singular)
bool launch_blocked_inverse(double* Mt, int64_t D, const BInvWork& bw, bool fast, const GJWork& gw, State* st,
                            hipStream_t stream, int passes = NM_PASSES_RUN, const GemmSpec* fuse = nullptr,
                            const TrailLookAhead* tla = nullptr, bool resid0_done = false,
                            double* ain0 = nullptr, int slow_from = -1);
#ifdef MIDAGMA_EXPERIMENTS
// launch_build_at(W, ldw, square, binv_build_target(...), D, d, 0, pr, st, stream) and the fast
// blocked inverse's outer block 0 residual (S read from W) in one launch; B2 = 256 only
// (experiments build: measured slower).
void launch_build_resid0(const double* W, int64_t ldw, double* At, int64_t D, int64_t d, const Params* pr,
                         const BInvWork& bw, State* st, hipStream_t stream);
#endif

// One B2 x B2 block (B2 = 128 or 256) by the product-form series from the warm start in the
// ring Pe / Po (the slot parity and the extrapolation rule of the blocked inverse: st->slots,
// st->warm_run): nm_resid + `passes` pass launches.  On convergence the inverse is in P and
// *done holds the converging pass; otherwise *done stays 0 or st->status becomes ST_NEED_GJ
// (also at once when st->ckpt_pending).  part: (NM_PASSES + 1) x PART_STRIDE doubles.
struct SeriesWork {
  const double* Pe;
  const double* Po;
  double* Y[2];
  double* Q[2];
  double* P;
  double* part;
  int* done;
};
void launch_series(const double* S, int64_t lds, int B2, const SeriesWork& w, State* st, int passes,
                   hipStream_t stream);
// the DagmaMLP log-det's fast step: the gate gjst reset and the series' residual launch with
// S = (sI - A)^T read from A (d <= B2) and the warm start's parity of st->slots + 1
void launch_ldfast_resid(const double* A, int64_t lda, int64_t d, double s, int B2, const SeriesWork& w, State* st,
                         State* gjst, hipStream_t stream);
// pass p (1 .. NM_PASSES) of that series alone
void launch_series_pass(int B2, const SeriesWork& w, State* st, int p, hipStream_t stream);

// --- gemm.hip: the trailing update with the next block's series in the same launch ---------
// Outer step g's 128-tile trailing update (launch_trail128, B2 = 256, C0 folded in the K loop)
// whose launch also runs block g + 1's product-form series (residual and `passes` passes, the
// series launches' tile bodies: nm_series.h) on `workers` workgroups placed after the first
// round of tiles: block g + 1's diagonal S = Aout[G', G'] comes from the launch's first four
// tiles, which signal a counter; the workers hand each phase on through counters of their own
// (agent-scope release / acquire).  The counters must be 0 at launch (the panel launch of step g
// zeroes them); every wait is bounded, and a timeout hands the slot back to the pivoted path
// (ST_NEED_GJ).  sync: 8 counters of 32 ints ([0] diagonal tiles, [32 p] phase p, [224] timeouts).
struct TrailSeries {
  const double* Pe;  // block g + 1's warm-start ring (blockinv.hip's Pst / Pst1 rows)
  const double* Po;
  double* Y[2];
  double* Q[2];
  double* P;
  double* part;      // block g + 1's (NM_PASSES + 1) x PART_STRIDE row partials
  int* done;
  int* sync;
  int passes, xmap, workers;
};
void launch_trail128_series(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, State* st,
                            const TrailSeries& ts, hipStream_t stream);
// ... and block g + 1's panel too (B2 = 256): its jobs (binv_panel_job) are claimed by `workers`
// more workgroups at the end of the grid once block g + 1's band tiles and series are done; the
// panel launch of block g + 1 is skipped.  pcheck: the panel's domain flags (last block);
// Ppe / Ppo: block g + 1's warm-start stores; zsync2: block g + 2's counters (zeroed here)
struct TrailPanel {
  double* Ppe;
  double* Ppo;
  int* zsync2;
  int pcheck, pf, workers;
};
constexpr int TS_FIN = 160, TS_BAND = 192, TS_JOB = 208;  // sync words of the fused launch
void launch_trail128_panel(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, State* st,
                           const TrailSeries& ts, const TrailPanel& tp, hipStream_t stream);

// --- dfinv.hip --------------------------------------------------------------
// The fast slot's blocked inverse as one dataflow launch (tile tasks, host-planned order).
constexpr int DF_MAX_K2 = 8;  // outer blocks of 256
// D the one-launch inverse takes (D % 256 == 0, 512 <= D <= MIDAGMA_EXP_DF_MAXD, default 1536)
bool df_available(int64_t D);
// ints of the control block (zeroed once at allocation; every launch leaves it zeroed, except
// the timeout count at [2 * 32])
int64_t df_ctl_ints(int64_t D);
struct DfPlanHost {  // views into a process-wide cache
  const std::vector<int>* tasks;  // 12 ints per task, grouped by workgroup
  const std::vector<int>* woff;   // nwg + 1 offsets (in tasks)
  int nctr;
  double est_us;                  // the list scheduler's makespan under its cost model
};
DfPlanHost df_plan(int64_t D, int passes, int nwg);
struct DfWork {
  double* A[DF_MAX_K2];  // A^0 (build_at's target) .. A^{K2-1}; A^{K2} is Mt
  double* Y;             // K2 x (NM_PASSES + 1) series iterates, B2 x B2 each
  double* Q;
  double* P;             // K2 converged diagonal-block inverses
  int* ctl;
  const int* tasks[2];   // device copies of df_plan(D, 2 / 3, nwg)
  const int* woff[2];
  int nwg;
  unsigned long long* stamps = nullptr;  // diagnostics (MIDAGMA_DF_STAMPS): 3 per task of the last launch
};
void launch_df_inverse(double* Mt, int64_t D, const DfWork& w, const BInvWork& bw, int passes, State* st,
                       hipStream_t stream);

// --- small.hip --------------------------------------------------------------
// LDS/register block edge of the one-workgroup small-d inner loop (16, 32 or 64; 0: d > 64).
int small_block(int64_t d);
// Up to n_slots slots of the cov-mode l2 inner loop (linear.py:224-331) in one persistent
// workgroup: W, m, v (leading dimension pr->D) are read at entry and written back at exit,
// with the State.  Across launches: carry (NORM_FIELDS + 1 doubles) holds a pending
// checkpoint step's norms and the warm-start count, pstore (2 x 32 x 32) the last two
// inverses; zero carry before a call's first launch.  Slots after a terminal status are
// not run.
// tcc (nullable; d <= 32): the TCC trek regularizer inside every slot ('opt') or every
// checkpoint slot ('log'), tcc_blk.h's body on the workgroup, its state words read at entry and
// written back at exit (the graph-replayed slots' TccWork words, so the two paths interleave).
struct SmallTcc {
  const double* S;        // D x D pair indicator
  double ws, eps, m, weight;
  int mode;               // 1 'log', 2 'opt'
  double* scal;           // TccWork::scal, vprev, uprev
  double* vprev;
  double* uprev;
  int fix = 1;            // TccWork::fix
};
void launch_small_minimize(const Params* pr, State* st, double* W, double* m, double* v, const double* covs,
                           const double* minc, const double* mexc, const double* bc_table, CkptRec* ckpt,
                           int64_t ckpt_cap, double* carry, double* pstore, int64_t d, int64_t n_slots,
                           hipStream_t stream, const SmallTcc* tcc = nullptr, bool w32 = false);

// --- trek.hip ---------------------------------------------------------------
enum TrekSeq : int { TREK_EXP = 0, TREK_INV = 1, TREK_LOG = 2, TREK_BINOM = 3 };
enum TrekAgg : int { TREK_MEAN = 0, TREK_SUM = 1, TREK_MAX = 2, TREK_LSE = 3 };
constexpr int TREK_TAYLOR_M = 12;   // exp: Taylor degree after scaling to ||X||_1 <= 1/4
constexpr int TREK_SMAX = 12;       // exp: squaring slots (||W o W||_1 up to 2^10)
struct TrekCfg {
  int seq, agg;
  int mode;              // 1 'log' (value on checkpoint slots), 2 'opt' (value + gradient every slot)
  double weight, eps_inv;
  int K;                 // log: series terms; binom: the exponent (= d, notreks pst_mat)
  int smax;              // exp: squaring slots
  int64_t m;             // pairs
  const int32_t* pairs;  // device, (i, j) x m
};
struct TrekWork {
  GJWork gj;             // inv: the Gauss-Jordan side panels (borrowed from the solver)
  double *X, *F, *H, *S, *GT, *L, *tmp, *tmp2, *tmp3, *tmp4, *slices;  // D x D (slices: 4 D x D or null)
  double* Q[TREK_TAYLOR_M + 1 > 64 ? TREK_TAYLOR_M + 1 : 64];  // Horner / powering iterates (sized at setup)
  double* E[TREK_SMAX + 1];
  double* dQ[2];
  double* colpart;       // (D / 64) x D
  double* part;          // 4 x 256
  double* scal;          // [0] value [1] 2^-s [2] s [3] max [4] coefficient [5] ||W o W||_1
  State* gates;          // 1 + 2 smax gate words
};
// The PST penalty of W (value in w.scal[0]) and, in 'opt' mode, weight * d value / d W into
// Gtrek (D x D), gated by st (a terminated slot or, in 'log' mode, a non-checkpoint slot
// runs nothing).
void launch_trek_pst(const double* W, int64_t d, int64_t D, const TrekCfg& cfg, const TrekWork& w, const State* st,
                     double* Gtrek, hipStream_t stream);

// --- tcc.hip ----------------------------------------------------------------
constexpr int TCC_NODA_MAX = 24;     // Noda steps per slot (gated off once converged)
// the fixed-shift stage (tcc.hip): inverse iteration for v and u at the warm start's
// Collatz-Wielandt bound, at most TCC_FIX_SWEEPS sweeps; gate words after the Noda steps' ones:
// [TCC_GATE_FINAL] the Noda path's final inverse, [TCC_GATE_FIX0 + k] sweep k (2d > 256),
// [TCC_GATE_PRE] a fast slot's Noda steps before the stage (on when the last stage was hard)
constexpr int TCC_FIX_SWEEPS = 8;        // (2d > 256: two or three launches a sweep)
constexpr int TCC_FIX_SWEEPS_SMALL = 16; // (2d <= 256: one workgroup, a few microseconds a sweep)
// a stage settled within this many sweeps needs no Noda step before the next one: the whole budget,
// i.e. the Noda step only after a stage that did not settle (measured at d = 1000 after 1400 steps,
// profiles/r06_probe_tccd1000_easy.log: half the budget ran it on most slots, 2.26 ms a step,
// against 1.81 with the whole budget and 1.68 with none)
constexpr int TCC_FIX_EASY = TCC_FIX_SWEEPS, TCC_FIX_EASY_SMALL = TCC_FIX_SWEEPS_SMALL;
constexpr int TCC_GATE_FINAL = 1 + TCC_NODA_MAX;
constexpr int TCC_GATE_FIX0 = TCC_GATE_FINAL + 1;
constexpr int TCC_GATE_PRE = TCC_GATE_FIX0 + TCC_FIX_SWEEPS;
constexpr int TCC_GATES = TCC_GATE_PRE + 1;
struct TccCfg {
  int mode;              // 1 'log', 2 'opt' (as TrekCfg)
  double weight, w, eps; // regularizer weight, multiplier of S, the reference's eps
  int64_t m;             // pairs
};
struct TccWork {
  GJWork gj;             // sized for D2
  int64_t D2;            // round_up64(2 d)
  double *A, *Mi;        // D2 x D2: the block matrix, the shifted inverse
  double* S;             // D x D pair indicator
  double *x, *y, *u, *z, *vprev, *uprev;  // D2 vectors
  double* part;          // ceil(2d / 64) x D2 transposed-GEMV partials
  double* scal;          // [0] value [1] sigma [2] lower [3] rho [4] u.v+eps [5] u.u+eps [7] breakdown [8] warm
                         // [9] converged (this slot) [10] converged (the last completed slot)
                         // fixed-shift stage: [11] v converged [12] u converged [13] breakdown [14] upper bound
                         // [15] sweeps to converge (0: none did) [16] hard (kept across slots)
  State* gates;          // TCC_GATES gate words
  // the two-level blocked inverse's buffers for D2 (pivoted path: Aalt D2 x D2, Pst / Pst1 D2 x B2);
  // null: the flat Gauss-Jordan
  double* Aalt = nullptr;
  double* Pst = nullptr;
  double* Pst1 = nullptr;
  // the fixed-stage inverse on the fast path for every outer block but the last (fast slots,
  // D2 >= 2048; null Y0: off): the product-form series' buffers (BInvWork's), its warm starts in Pst
  double *Y0 = nullptr, *Y1 = nullptr, *Q0 = nullptr, *Q1 = nullptr, *Pblk = nullptr, *part2 = nullptr;
  int* done = nullptr;
  int fix = 1;  // the fixed-shift stage first (2d > 128; 0: Noda from the warm start at once)
  int fix_pre = 1;  // fast slots: Noda steps before the fixed-shift stage when the last stage was hard
  int fix_hold = 8;  // ... and for this many slots after it
  int fix_easy = 0;  // (> 0: the sweep count that still counts as easy, for both forms; 0: TCC_FIX_EASY*)
};
// The TCC penalty of W (value in w.scal[0]) and, in 'opt' mode, weight * d value / d W into
// Gtrek (D x D), gated like launch_trek_pst.
// handback (nullable; the launch-chain form, 2d > 128): only `steps` Noda steps are enqueued, and
// if Noda has not converged by then the slot hands back (handback->status = ST_NEED_GJ, the rest of
// the TCC sequence gated off): the fast cov slot's short chain, the host re-running the slot with
// all TCC_NODA_MAX steps (tcc.hip).
void launch_trek_tcc(const double* W, int64_t d, int64_t D, const TccCfg& cfg, const TccWork& w, const State* st,
                     double* Gtrek, hipStream_t stream, State* handback = nullptr, int steps = TCC_NODA_MAX);

// --- mlp.hip ----------------------------------------------------------------
constexpr int64_t MLP_TAIL_MAX_DM = 7936;  // d * m1 the fused DagmaMLP tail stages per row in LDS
#ifdef MIDAGMA_EXPERIMENTS
// fc1 and the tail fused on the MFMA (experiments build; measured slower): d <= 16 MLP_FUSED_MAX_NIB, m1 with a multiple of 16 up to
// 128 that m1 divides; mlp_fused_parts = the forward's partials of sum R^2 (0: not supported)
constexpr int MLP_FUSED_MAX_NIB = 16;
int mlp_fused_ncb(int64_t m1);
int64_t mlp_fused_parts(int64_t n, int64_t d, int64_t m1);
int64_t mlp_fused_splits(int64_t n);
void launch_mlp_fc1_tail_fwd(const double* X, const double* W1, const double* b1, const double* w2, const double* b2,
                             int64_t n, int64_t d, int m1, double* S, double* R, double* part, hipStream_t stream);
void launch_mlp_tail_bwd_lin(const double* S, const double* w2, const double* R, const double* X,
                             const double* part, int64_t npart, const double* gobj, double mu, double half_d,
                             double inv_n, int64_t n, int64_t d, int m1, double* lin, double* dw2, double* db2,
                             double* db1, double* scratch, hipStream_t stream);
#endif
// doubles of scratch the tail needs (both directions)
int64_t mlp_tail_scratch(int64_t n, int64_t d, int64_t m1);
// Z (n x d*m1) -> R = Xhat - X (n x d), *ssq = sum R^2
// (b1 nullable: Z is then the pre-activation itself, else Z + b1 per column)
void launch_mlp_tail_fwd(const double* Z, const double* b1, const double* w2, const double* b2, const double* X,
                         int64_t n, int64_t d, int m1, double* R, double* scratch, double* ssq, hipStream_t stream);
// g (device scalar) = d loss / d ssq -> dZ (n x d*m1), dw2 (d x m1), db2 (d)
// (db1 nullable: also the column sums of dZ, the fc1 bias gradient)
// (part nullable: then g = d loss / d ssq; else gobj = d loss / d obj and the backward takes ssq from
// the forward's row partials part[n] and d obj / d ssq itself, mlp_objective_bwd's arithmetic)
void launch_mlp_tail_bwd(const double* Z, const double* b1, const double* w2, const double* R, const double* g,
                         int64_t n, int64_t d, int m1, double* dZ, double* dw2, double* db2, double* db1,
                         double* scratch, hipStream_t stream, const double* part = nullptr,
                         const double* gobj = nullptr, double mu = 0.0, double half_d = 0.0, double inv_n = 0.0,
                         bool sums = true);

// fc1 terms of the [d, m1, 1] DagmaMLP: A[i, j] = sum_m W1[j m1 + m, i]^2, |W1| partial sums
// (fc1_terms_parts(d) of them); backward dW1 = 2 W1 gA^T + gl1part sign(W1)
int64_t fc1_terms_parts(int64_t d);
void launch_fc1_terms(const double* W1, int64_t d, int m1, double* A, double* l1part, hipStream_t stream);
// (lin, nlin: nlin split-K chunks of another dW1 contribution to add; nullable / 0)
// (gobj nullable: d obj; then gscale = gobj and gl1part = (gobj mu) lambda1 everywhere, the
// objective's backward folded in)
void launch_fc1_terms_bwd(const double* W1, int64_t d, int m1, const double* gA, const double* gscale,
                          const double* gl1part, const double* lin, int nlin, double* dW1, hipStream_t stream,
                          const double* gobj = nullptr, double mu = 0.0, double lambda1 = 0.0);
// Mt (d x d, ldm; nullable) from the D x D log-det workspace Ws and h = -sum(piv[0:d]) + dls
void launch_logdet_post(const double* piv, int64_t d, double dls, double* h, const double* Ws, int64_t D, double* Mt,
                        int64_t ldm, hipStream_t stream);
// The h log-det's warm-started fast path (mlp.hip, DagmaNonlinear.minimize): the step's start
// (ring parity, Gauss-Jordan gate reset; with build, (sI - A)^T into the B x B S), the series
// result's certificate (Mt from P, gate opened when P did not converge or has an entry < 0 or
// non-finite) and the step's end (h and Mt from the Gauss-Jordan chain when it ran, else h =
// *hlast; the inverse into the ring; the ring state advanced).
void launch_ldfast_begin(State* st, State* gjst, hipStream_t stream);
void launch_ldfast_certify(const double* P, int B, int64_t d, double* Mt, int64_t ldm, const State* st,
                           const int* done, State* gjst, double* ring0, double* ring1, hipStream_t stream);
void launch_ldfast_post(const double* piv, int64_t d, double dls, double* h, const double* Wgj, int64_t Dgj, double* Mt,
                        int64_t ldm, const double* P, int B, double* ring0, double* ring1, State* st,
                        const State* gjst, double* hlast, bool exact, hipStream_t stream);
// obj = mu (half_d log(inv_n ssq) + lambda1 sum(l1part)) + h and its backward
// (part nullable: ssq from the tail's npart row partials instead; counter nullable: += 1)
void launch_mlp_objective(const double* ssq, const double* l1part, int64_t np, const double* h, double mu,
                          double lambda1, double half_d, double inv_n, double* out, hipStream_t stream,
                          const double* part = nullptr, int64_t npart = 0, int64_t* counter = nullptr);
void launch_mlp_objective_bwd(const double* g, const double* ssq, int64_t np, double mu, double lambda1, double half_d,
                              double inv_n, double* gssq, double* gl1part, double* gh, hipStream_t stream);

// --- adam.hip ---------------------------------------------------------------
// the [d, m1, 1] DagmaMLP step's closing launch (mlp.hip mlp_step_kernel): the tail's dw sums, fc1's
// weight gradient, Adam over the four parameters and the next step's fc1 terms
struct MlpStepPtrs {
  double *W1, *b1, *w2, *b2;
  double *mW1, *vW1, *mb1, *vb1, *mw2, *vw2, *mb2, *vb2;
};
void launch_mlp_step(const MlpStepPtrs& p, int64_t n, int64_t d, int m1, const double* gA, const double* gobj,
                     double mu, double lambda1, const double* lin, int nlin, const double* scratch,
                     const double* table, const int64_t* counter, double w1, double beta2, double c2, double eps,
                     double wd, const double* gate, double* A, double* l1part, hipStream_t stream);
struct AdamCoef {  // host-rounded as torch.optim.Adam computes them in Python floats
  double step_size, w1, beta2, c2, bc2_sqrt, eps, wd;
};
// one torch-Adam step on n doubles, skipped when gate != nullptr and *gate < 0
void launch_adam_gated(double* p, const double* g, double* m, double* v, int64_t n, const AdamCoef& c,
                       const double* gate, hipStream_t stream);
// the same with step_size = table[2 t], sqrt(1 - b2^t) = table[2 t + 1], t = *counter
void launch_adam_gated_table(double* p, const double* g, double* m, double* v, int64_t n, const AdamCoef& c,
                             const double* table, const int64_t* counter, const double* gate, hipStream_t stream);
void launch_counter_advance(int64_t* counter, hipStream_t stream);
// the table step over k <= ADAM_MULTI tensors in one launch (off: prefix sums of the sizes)
constexpr int ADAM_MULTI = 8;
struct AdamSet {
  double* p[ADAM_MULTI];
  const double* g[ADAM_MULTI];
  double* m[ADAM_MULTI];
  double* v[ADAM_MULTI];
  int64_t off[ADAM_MULTI + 1];
  int k;
};
void launch_adam_gated_table_multi(const AdamSet& set, const AdamCoef& c, const double* table, const int64_t* counter,
                                   const double* gate, hipStream_t stream);

// --- sem.hip ----------------------------------------------------------------
// Parents (CSR over columns of W, ascending) and topological levels of a weighted DAG.
struct SemGraph {
  std::vector<int32_t> pptr, pidx, nodes, level_off;
  std::vector<double> pw;
};
struct SemDev {  // device copies of SemGraph (+ per-node noise scales)
  const int32_t *nodes, *pptr, *pidx;
  const double *pw, *scale;
};
// false if W (host, d x d row-major, W[p, j] = edge p -> j) has a cycle
bool sem_levels(const double* W, int64_t d, SemGraph& g);
// Rows [row0, row0 + rows) of the linear SEM (row0 even) into the node-major slab XT (ldt even),
// then rows [skip, rows) of it to X (row-major, ldx).  sem: 0 gauss 1 exp 2 gumbel 3 uniform
// 4 logistic 5 poisson.
void launch_sem_slab(const SemDev& g, const std::vector<int32_t>& level_off, int64_t d, int sem, uint64_t seed,
                     int64_t row0, int64_t rows, int64_t skip, double* XT, int64_t ldt, double* X, int64_t ldx,
                     hipStream_t stream);

// --- gemm.hip ---------------------------------------------------------------
enum GemmB : int { B_PLAIN = 0, B_IMINUS = 1 };
enum GemmEpi : int { EPI_STORE = 0, EPI_SIGMOID = 1, EPI_SUB_BAND = 2 /* launch_trail128 only */,
                     EPI_SUB_CROSS = 3 /* launch_trail128_split only */,
                     EPI_SUB_PRE = 4 /* EPI_SUB_BAND with C0 preloaded into the accumulators */,
                     EPI_SUB_MID = 5 /* EPI_SUB_BAND with C0 folded in during the 16 k-tiles (B2 = 256) */,
                     EPI_SUB_CROSS_MID = 6 /* EPI_SUB_CROSS with the EPI_SUB_MID fold */,
                     EPI_SIGMOID_SPLIT = 7 /* internal: launch_gemm's EPI_SIGMOID with split = 2 */ };
void gemm_setup_attributes();
// C[M x N] = op(A) * op(B); op(A) = A ([m][k], lda) or, if a_trans, A stored [k][m] (lda);
// op(B) = B or (I - B) ([k][n], ldb).  M, N, K multiples of 64.  With split > 1
// the K range is cut into `split` slices written to C + z*slice_stride.
// EPI_SIGMOID: C = expit(acc); if loss_part != nullptr and st->ckpt_pending,
// per-workgroup partials of sum(logaddexp(0,acc) - X*acc) over rows < m_valid,
// cols < n_valid go to loss_part[blockIdx.y * gridDim.x + blockIdx.x] (X = A).
// EPI_SIGMOID with split = 2 (128-tile grids with tiles % 8 == 0): the two K halves run in
// series (EPI_SIGMOID_SPLIT); C must hold the output, the first halves' partial at
// C + slice_stride (slice_stride >= M ldc) and one int flag per tile at C + 2 slice_stride, the
// flags zero before the first launch (each launch leaves them zero).
void launch_gemm(int64_t M, int64_t N, int64_t K, const double* A, int64_t lda, bool a_trans, const double* B,
                 int64_t ldb, GemmB bmode, double* C, int64_t ldc, GemmEpi epi, int split, int64_t slice_stride,
                 double* loss_part, int64_t m_valid, int64_t n_valid, const State* st, hipStream_t stream);
// Trailing update of the blocked inverse's outer step g on 128 x 128 tiles:
// Aout[i, j] = Ain[i, j] - Ain[i, G] Aout[G, j] for i, j outside G = [g B2, (g+1) B2);
// with `check`, ORs the domain flags of the outputs into st->flags.
void launch_trail128(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, bool check, const State* st,
                     hipStream_t stream);
#ifdef MIDAGMA_EXPERIMENTS
// The same update with C0 read in the epilogue at every B2 (launch_trail128 folds it in during the
// K loop at B2 = 256; experiments build, tools/micro/trail_micro.hip)
void launch_trail128_band(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, bool check,
                          const State* st, hipStream_t stream);
// The same update with the accumulators preloaded from C0 (experiments build, tools/micro/trail_micro.hip)
void launch_trail128_pre(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, bool check,
                         const State* st, hipStream_t stream);
// The B2 = 256 update (EPI_SUB_MID tiles) on `nwg` persistent workgroups: static round robin over
// the tiles (ctr == nullptr), or tiles claimed from the counter *ctr (zero before the launch)
void launch_trail128_persist(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, const State* st,
                             int nwg, int* ctr, hipStream_t stream);
// The pipelined GEMM (EPI_STORE, split-K slices as launch_gemm) on a subset of the CUs: 2 workgroups
// per CU are launched, those on a shader engine >= `ses` of their XCD exit at once, the others
// claim tiles from *ctr (zeroed by a memset node before the launch, on `stream`), so the other
// launches of the slot keep the remaining CUs to themselves (the cov score GEMM forked beside the
// inverse, MIDAGMA_EXP_COV_FORK=2 with MIDAGMA_EXP_GEMM_SES)
void launch_gemm_cupart(int64_t M, int64_t N, int64_t K, const double* A, int64_t lda, bool a_trans, const double* B,
                        int64_t ldb, GemmB bmode, double* C, int64_t ldc, int split, int64_t slice_stride,
                        const State* st, int ses, int* ctr, hipStream_t stream);
// The B2 = 256 update as data-parallel tiles plus a stream-K remainder: the first `dp` tiles (of
// xcd_remap's order) one per workgroup (EPI_SUB_MID), the other ntiles - dp tiles' 16 K-tiles each
// split evenly over `nsk` workgroups; a partial tile goes to ws (2 nsk 128 x 128 slots), the
// workgroup holding a tile's last K-tile sums its partials in K order (flags: nsk words, zero before
// the first launch; each launch leaves them zero) and writes C = C0 - sum
void launch_trail128_sk(const double* Ain, double* Aout, int64_t D, int64_t g, bool check, const State* st, int dp,
                        int nsk, double* ws, int* flags, hipStream_t stream);
#endif
// The same update in two launches: part 0 the tiles in block g + 1's row and column bands, part 1
// the rest (no domain check: the look-ahead runs on steps before the last).
void launch_trail128_split(const double* Ain, double* Aout, int64_t D, int64_t B2, int64_t g, int part,
                           const State* st, hipStream_t stream);
// The GEMM gs (EPI_STORE) and the blocked inverse's 32 x 32 trailing update of outer step g
// (n_trail tiles) in one launch.
bool gemm_trail_supported(const GemmSpec& gs);
void launch_gemm_trail(const GemmSpec& gs, const double* Ain, double* Aout, int64_t D, int B2, int g, bool check,
                       State* st, int pf, int n_trail, hipStream_t stream);
// dst[c][r] = src[r][c] (rows x cols)
void launch_transpose(const double* src, int64_t ld_src, int64_t rows, int64_t cols, double* dst, int64_t ld_dst,
                      hipStream_t stream);
// out[i] = sum_z parts[z*stride + i] (fixed order) for i < count.
void launch_sum_slices(const double* parts, int split, int64_t stride, int64_t count, double* out,
                       const State* st, hipStream_t stream);
// out[0] = sum(v[0..n)) in a fixed order (one workgroup).
void launch_sum_vector(const double* v, int64_t n, double* out, const State* st, hipStream_t stream);

// --- gram.hip (fit()'s data preparation, linear.py:406-428) ------------------
// column sums of X (n x d, ldx): colsum_parts(n) x d doubles of partials, then a fixed-order sum
int64_t colsum_parts(int64_t n);
void launch_colsum(const double* X, int64_t n, int64_t d, int64_t ldx, double* part, double* out,
                   hipStream_t stream);
// X[r, j] -= colsum[j] / nrows in place
void launch_center(double* X, int64_t n, int64_t d, int64_t ldx, const double* colsum, double nrows,
                   hipStream_t stream);
// S (rpad x D) <- rows x d of X zero-padded; *flag |= 1 on a non-finite value
void launch_stage_rows(const double* X, int64_t ldx, int64_t rows, int64_t d, double* S, int64_t D, int64_t rpad,
                       int* flag, hipStream_t stream);
void launch_nonfinite_or(const double* S, int64_t rows, int64_t cols, int64_t ld, int* flag, hipStream_t stream);
// out (d x d, ldo) = in (ldi) / divisor; *flag |= 1 on a non-finite result
void launch_div_block(const double* in, int64_t ldi, double divisor, int64_t d, double* out, int64_t ldo, int* flag,
                      hipStream_t stream);
// the chunked Gram's shape: padded D, split-K per chunk, chunk rows (a multiple of 256), chunks
struct GramPlan {
  int64_t D = 0, chunk = 0, nchunks = 0;
  int split = 1;
};
GramPlan gram_plan(int64_t n, int64_t d, int64_t chunk_rows);

// --- comm.hip (the in-library RCCL communicator of a data-mode solver) -------
// 128-byte ncclUniqueId into out (returns its size); a communicator of nranks (opaque);
// in-place all-reduce of n doubles (sum, or max) on stream (graph-capturable)
int comm_unique_id(void* out);
void* comm_create(const void* id, int nranks, int rank);
void comm_create_all(int ndev, const int* devlist, void** comms);
void comm_destroy(void* comm);
void comm_allreduce(void* comm, double* buf, size_t n, bool max, hipStream_t stream);
// out[0..4) = (status, iter, -status, -iter) of *st (one max all-reduce: max and min over ranks)
void launch_agree_pack(const State* st, double* out, hipStream_t stream);

// --- step.hip ---------------------------------------------------------------
void launch_reduce_check(const double* Mt, const double* W, const double* Z, const Params* pr, State* st,
                         double* partials, int64_t d, int64_t D, hipStream_t stream);
// npart: the checkpoint-step norm partials of fused_update (NORM_FIELDS per workgroup of its
// ceil(d/256) x d grid), reduced into the checkpoint record.
// trek_val (nullable): the trek regularizer value of this slot's W (PST, trek.hip)
void launch_control(const Params* pr, State* st, const double* partials, const double* pivlog,
                    const double* loss_total, const double* bc_table, CkptRec* ckpt, int64_t ckpt_cap,
                    const double* npart, int64_t d, const double* trek_val, hipStream_t stream,
                    const double* l1_32 = nullptr);
// float32 W (DagmaLinear(dtype=np.float32)): numpy's float32 np.abs(W).sum() (np_sum.h) into *out on
// checkpoint slots, for control's objective (linear.py:127); chunk_sums: np_l1_chunks(d) floats
int64_t np_l1_chunks(int64_t d);
void launch_np_l1(const double* W, int64_t d, int64_t D, const State* st, float* chunk_sums, double* out,
                  hipStream_t stream);
// Z: the score partial, or (zsplit > 1) split-K slices Z + z*zstride summed here in the order
// of launch_sum_slices.  trek (nullable): weight * trek gradient, added last (linear.py:258).
void launch_fused_update(const Params* pr, const State* st, double* W, double* m, double* v, const double* Mt, const double* Z, int zsplit, int64_t zstride, const double* cov,
                         const double* minc, const double* mexc, const double* trek, int64_t d, int64_t D,
                         double* npart, hipStream_t stream);
// fused_update (with the checkpoint iteration's norm partials, as launch_fused_update) plus the
// next slot's build_at from the new W: A0 = s I - (W o W)^T (outer step 0's input,
// launch_blocked_inverse ain0) and IW = I - W (nullable); D % 8 == 0
void launch_fused_update_at(const Params* pr, const State* st, double* W, double* m, double* v, const double* Mt,
                            const double* Z, int zsplit, int64_t zstride, const double* cov, const double* minc,
                            const double* mexc, const double* trek, int64_t d, int64_t D, double* A0, double* IW,
                            double* npart, hipStream_t stream);
// *flag (device int) <- 1 if any of x[0..n) is inf or nan, else 0
void launch_any_nonfinite(const double* x, int64_t n, int* flag, hipStream_t stream);
// y = a * x elementwise over n doubles
void launch_scale(const double* x, double a, double* y, int64_t n, hipStream_t stream);
// G = 2 * W * Mt on the logical block (linear.py:115)
void launch_h_grad(const double* W, const double* Mt, double* G, int64_t d, int64_t D, hipStream_t stream);
// out[0] = sum over logical block of (I - W) * Z, out[1] = sum |W|   (one pass, fixed order)
void launch_trace_l1(const double* W, const double* Z, double* partials, int64_t d, int64_t D,
                     hipStream_t stream);

}  // namespace midagma
