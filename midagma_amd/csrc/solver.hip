// Host orchestration + C ABI (include/midagma_hip.h).
//
// One "slot" = one pass of the reference's loop body (linear.py:225-331):
//   part 1  build (sI - W∘W)^T -> blocked GJ inverse (+ log|pivots|) -> score GEMM(s)
//   part 2  domain check / checkpoint partials -> control (1 WG) -> fused update
// The control decision lives in device memory, so slots are replayed from a
// hipGraph in batches with no host round trip per step; the host only polls
// the state every batch.  Slots after termination are
// no-ops (every kernel early-exits on the status word).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/midagma_hip.h"
#include "launch.h"
#include "slot_sched.h"

using namespace midagma;

namespace {
thread_local std::string g_global_error;

// scipy's check_finite (linear.py:226 -> sla.inv(..., check_finite=True)): a non-finite input
// is a ValueError, not a singular matrix
bool all_finite(const double* p, int64_t rows, int64_t cols, int64_t ld) {
  for (int64_t i = 0; i < rows; ++i)
    for (int64_t j = 0; j < cols; ++j)
      if (!std::isfinite(p[i * ld + j])) return false;
  return true;
}
constexpr const char* kNonFinite = "array must not contain infs or NaNs";

struct DevBuf {
  double* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    if (count <= n && p) return;
    release();
    HIP_TRY(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(double)));
    n = count;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};
}  // namespace

struct midagma_solver {
  int loss = 0, mode = 0, device = 0;
  int64_t d = 0, D = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // data mode: the inverse runs on a high-priority side stream beside the score GEMMs (it
  // depends on W only); fork / join are events inside the captured slot graph
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool fork_inv = !knob_set("MIDAGMA_EXP_NO_FORK");  // experiment knobs: knobs.h
  std::string err;

  DevBuf W, m, v, Mt, cov, covs, minc, mexc, P, R, C, pivlog, partials, bc_table, zown, scratch, Gtmp, Pstore;
  // ((-mu) cov)^T: the cov-mode score GEMM reads its A operand k-major (coalesced tile rows)
  DevBuf covsT;
  bool cov_at = !knob_set("MIDAGMA_EXP_COV_AMODE0");
  bool cov_iw = knob_set("MIDAGMA_EXP_COV_IW");
  DevBuf npart;  // checkpoint-step norm partials (fused_update -> control)
  // cov mode, l2, d <= 64, no trek regularizer: the one-workgroup persistent loop (small.hip)
  DevBuf scarry, sprev;  // between two small-loop launches: pending norms + warm count, last inverses
  bool use_small = !knob_set("MIDAGMA_EXP_NO_SMALL");
  bool small_tcc = knob("MIDAGMA_EXP_SMALL_TCC", 1) != 0;  // experiments: 0 keeps TCC on the graph slots
  // (the TCC regularizer runs inside it up to d = 32, tcc_blk.h; PST keeps the graph-replayed slots)
  bool small_on() const {
    return use_small && mode == MIDAGMA_MODE_COV && loss == MIDAGMA_LOSS_L2 && small_block(d) > 0 &&
           (!trek_on || (trek_tcc && small_block(d) <= 32 && small_tcc && !w32));
  }
  // PST trek regularizer (trek.hip)
  TrekCfg tcfg{};
  bool trek_on = false;
  std::vector<DevBuf> tbufs;  // every D x D work buffer of the regularizer
  DevBuf tpairs, tsmall, Gtrek, tslices;
  State* tgates = nullptr;
  State* d_state_probe = nullptr;  // RUNNING + checkpoint: gates the API-call (midagma_trek) path
  TrekWork tw{};
  // TCC trek regularizer (tcc.hip): trek_tcc selects it; mode / weight live in tcfg as for PST
  bool trek_tcc = false;
  TccCfg ccfg{};
  TccWork cw{};
  DevBuf cA, cMi, cS, cvec, cpart, cP, cR, cC;
  State* cgates = nullptr;
  // cov mode, D >= 256: two-level blocked inverse (blockinv.hip) with the warm-started fast path
  int B2 = 0;
  DevBuf Malt, Pst2, Pst2b, nmY0, nmY1, nmQ0, nmQ1, nmP, nmPart, nmDone, nmLW, nmLZ, nmLPZ, nmSync;
  // the fast slot's inverse as one dataflow launch (dfinv.hip; experiments build only,
  // MIDAGMA_EXP_DF=1: measured slower than the launch-per-phase inverse)
  bool df_on = false;
#ifdef MIDAGMA_EXPERIMENTS
  DevBuf dfA, dfY, dfQ, dfP, dfCtl, dfTasks[2], dfWoff[2], dfStamps;
  DfWork dfw{};
#endif
  bool fast_ready = false;  // Pst2 holds the previous slot's outer-block inverses
  double* zbuf = nullptr;  // d x d (+64 tail) score partial; internal or bound
  int64_t zbuf_cap = 0;
  // data mode
  DevBuf X, Y, Zparts, loss_part, cov_parts;
  int cov_split = 1;
  int64_t n_local = 0, n_pad = 0, n_global = 0;
  // X^T (D x n_pad), the xw GEMM's A operand in the m-contiguous layout (the X^T Y GEMM reads
  // X itself that way); kept when the device has the room (MIDAGMA_NO_XT disables it)
  DevBuf XT;
  DevBuf IW;  // I - W of the slot, written by build_at for the data-mode X (I - W) GEMM
  bool use_xt = false;
  const double* xw_a() const { return use_xt ? XT.p : X.p; }
  int64_t xw_lda() const { return use_xt ? n_pad : D; }
  int split = 1;
  int sig_split = 1;  // the logistic sigmoid GEMM's serial split-K (launch_gemm; 2: Y holds the partial too)
  int sig_split_force = 0;
  DevBuf cupart_ctr;  // experiments: launch_gemm_cupart's tile counter
  bool w32 = false;  // midagma_set_w_float32: the reference's float32 W arithmetic (common.h f32r)  // midagma_debug_sig_split: 0 the size rule, 1 never split, 2 split where the shape allows
  int64_t loss_part_count = 0;

  Params* d_params = nullptr;
  State* d_state = nullptr;
  CkptRec* d_ckpt = nullptr;
  int64_t ckpt_cap = 0;
  State* h_state = nullptr;  // pinned, 2 snapshots
  hipEvent_t ev[2] = {nullptr, nullptr};

  double bc_b1 = -1, bc_b2 = -1;
  int64_t bc_len = 0;
  bool has_cov = false, has_data = false, has_inc = false, has_exc = false;
  bool begun = false;
  const double* cap_minc = nullptr;  // mask pointers baked into the captured graphs
  const double* cap_mexc = nullptr;
  double mu = 1.0;
  Params hp{};

  // g_fastN: FAST_GROUP fast slots in one graph (no inter-graph dispatch gap between them)
  // g_fast2 / g_fastN2: the same with 2 product-form passes per outer block (the extrapolated
  // warm start usually converges in 2); the host falls back to 3 for a while after a hand-back
  hipGraphExec_t g_part1 = nullptr, g_part2 = nullptr, g_full = nullptr, g_fast = nullptr, g_fastN = nullptr;
  hipGraphExec_t g_fast2 = nullptr, g_fastN2 = nullptr;
  bool nm_adapt = knob("MIDAGMA_EXP_NM_ADAPT", 1) != 0;
  int64_t three_pass_left = 0;  // fast slots still to run with 3 passes (after a 2-pass hand-back)
  bool graphs_valid = false;

  // ABI 7: the in-library RCCL communicator (data mode over ranks): the score all-reduce inside
  // the captured slot graphs, and an agreement all-reduce of (status, iters) at every poll
  void* comm = nullptr;
  int comm_ranks = 1;
  bool inslot_comm = false;  // set while capturing a whole slot
  DevBuf agree;               // 2 x 4 doubles (double-buffered polls)
  double* h_agree = nullptr;  // pinned 2 x 4

  ~midagma_solver() {
    destroy_graphs();
    if (stream) (void)hipStreamSynchronize(stream);
    comm_destroy(comm);
    agree.release();
    if (h_agree) (void)hipHostFree(h_agree);
    for (DevBuf* b : {&W, &m, &v, &Mt, &cov, &covs, &covsT, &minc, &mexc, &P, &R, &C, &pivlog, &partials, &bc_table,
                      &zown, &scratch, &Gtmp, &X, &Y, &Zparts, &loss_part, &cov_parts, &Pstore, &Malt, &Pst2, &Pst2b,
                      &nmY0, &nmY1, &nmQ0, &nmQ1, &nmP, &nmPart, &nmDone, &nmLW, &nmLZ, &nmLPZ, &nmSync, &npart, &XT, &IW, &scarry,
                      &sprev, &cupart_ctr})
      b->release();
#ifdef MIDAGMA_EXPERIMENTS
    for (DevBuf* b : {&dfA, &dfY, &dfQ, &dfP, &dfCtl, &dfTasks[0], &dfTasks[1], &dfWoff[0], &dfWoff[1], &dfStamps})
      b->release();
#endif
    for (DevBuf& b : tbufs) b.release();
    for (DevBuf* b : {&tpairs, &tsmall, &Gtrek, &tslices, &cA, &cMi, &cS, &cvec, &cpart, &cP, &cR, &cC}) b->release();
    if (cgates) (void)hipFree(cgates);
    if (tgates) (void)hipFree(tgates);
    if (d_state_probe) (void)hipFree(d_state_probe);
    if (d_params) (void)hipFree(d_params);
    if (d_state) (void)hipFree(d_state);
    if (d_ckpt) (void)hipFree(d_ckpt);
    if (h_state) (void)hipHostFree(h_state);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
    if (side) (void)hipStreamDestroy(side);
    for (hipEvent_t e : {ev_fork, ev_join})
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : la_ev) (void)hipEventDestroy(e);
  }

  void destroy_graphs() {
    for (hipGraphExec_t* ge : {&g_part1, &g_part2, &g_full, &g_fast, &g_fastN, &g_fast2, &g_fastN2})
      if (*ge) {
        (void)hipGraphExecDestroy(*ge);
        *ge = nullptr;
      }
    graphs_valid = false;
  }

  GJWork gj() { return GJWork{P.p, R.p, C.p, pivlog.p, Pstore.p}; }
  BInvWork binv() {
    return BInvWork{Malt.p,
                    Pst2.p,
                    Pst2b.p,
                    {nmY0.p, nmY1.p},
                    {nmQ0.p, nmQ1.p},
                    nmP.p,
                    nmPart.p,
                    reinterpret_cast<int*>(nmDone.p),
                    nmLW.p,
                    nmLZ.p,
                    nmLPZ.p,
                    reinterpret_cast<int*>(nmSync.p)};
  }
  bool blocked() const { return B2 > 0; }
  // k extent of the GEMMs whose K is the padded node dimension: the rows of A past d are zero
  // (X^T, ((-mu) cov)^T), so the k loop stops at the first 16-multiple >= d (the pipelined
  // 128-tile kernel, D % 128 == 0; bit-identical: the skipped terms are exact zeros)
  int64_t Kd() const { return D % 128 == 0 ? (d + 15) / 16 * 16 : D; }
  bool forked_inverse() const { return side != nullptr && !blocked() && mode == MIDAGMA_MODE_DATA; }
  // cov mode at large D (the 128-tile trailing update): the score GEMM beside the inverse
  // (experiment knob MIDAGMA_EXP_COV_FORK: 1 on, 0 off)
  bool cov_fork = knob("MIDAGMA_EXP_COV_FORK", 0) != 0;
  bool cov_fork_all = knob("MIDAGMA_EXP_COV_FORK", 0) == 2;  // 2: at every blocked D, not only large D
  // cov mode at large D, fast slots: the trailing-update look-ahead on two streams (blockinv.hip
  // blocked_inverse_lookahead; experiment knob MIDAGMA_EXP_COV_LA: 1 on, 0 off)
  bool cov_la = knob("MIDAGMA_EXP_COV_LA", 0) != 0;
  std::vector<hipEvent_t> la_ev;
  // blocked slots enqueued launch by launch instead of replayed graphs (experiment knob
  // MIDAGMA_EXP_EAGER: at large D the host runs far ahead of a multi-ms slot, and cross-stream
  // waits are plain queue barriers instead of graph edges)
  bool eager = knob("MIDAGMA_EXP_EAGER", 0) != 0;
  void run_eager(bool fast, int passes, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
      enqueue_part1(fast, passes);
      enqueue_part2(fast);
    }
  }
  bool cov_la_on() const { return cov_la && side != nullptr && mode == MIDAGMA_MODE_COV && blocked() && D - B2 >= 1792; }
  bool cov_fork_on() const {
    return cov_fork && side != nullptr && mode == MIDAGMA_MODE_COV && blocked() && (D - B2 >= 1792 || cov_fork_all) &&
           !trek_on;
  }
  bool data_binv = !knob_set("MIDAGMA_EXP_DATA_FLAT_GJ");
  // small data-mode shards: the blocked inverse (fast or pivoted) forked beside the GEMMs
  // (default-priority side stream; logistic d=1000, n=1e4: 1085 -> 1118, l2 1130 -> 1168 steps/s;
  // MIDAGMA_EXP_DATA_FORK_FAST=0 runs it in sequence)
  bool data_fork_fast = knob("MIDAGMA_EXP_DATA_FORK_FAST", 1) != 0;
  bool data_binv_on() const { return data_binv && mode == MIDAGMA_MODE_DATA && binv_block(D) > 0; }

  // ---- the slot -----------------------------------------------------------
  // fast: the outer diagonal blocks by the warm-started product form (blocked() only)
  void enqueue_part1(bool fast = false, int passes = NM_PASSES_RUN) {
    bool gemm_done = false;
    if (cov_fork_on()) {
      // large D, cov mode: the score GEMM (W and cov only) on the main stream beside the inverse
      // on the high-priority side stream, so its tiles fill the CUs the inverse's serial
      // series / panel phases leave idle; joined before anything reads Mt
      launch_build_at(W.p, D, /*square=*/true, binv_build_target(Mt.p, D, binv()), D, d, 0.0, d_params, d_state,
                      stream, IW.p);
      HIP_TRY(hipEventRecord(ev_fork, stream));
      HIP_TRY(hipStreamWaitEvent(side, ev_fork, 0));
      launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, side, passes, nullptr);
      HIP_TRY(hipEventRecord(ev_join, side));
      enqueue_score_cov(zbuf, d_state, /*sum=*/!fast);
      HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
      gemm_done = true;
    } else if (blocked() && data_fork_fast && side != nullptr && mode == MIDAGMA_MODE_DATA) {
      // small data-mode shard: the blocked inverse (fast or pivoted) on the side stream beside
      // the n x d GEMMs, joined before the update
      launch_build_at(W.p, D, /*square=*/true, binv_build_target(Mt.p, D, binv()), D, d, 0.0, d_params, d_state,
                      stream, IW.p);
      HIP_TRY(hipEventRecord(ev_fork, stream));
      HIP_TRY(hipStreamWaitEvent(side, ev_fork, 0));
      launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, side, passes, nullptr);
      HIP_TRY(hipEventRecord(ev_join, side));
      enqueue_data_partial(W.p, d_state, IW.p);
      enqueue_slot_allreduce();
      HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
      gemm_done = true;
    } else if (blocked()) {
      // cov fast slot: the score GEMM rides in the last trailing update's launch (its split-K
      // slices are what fused_update sums anyway); MIDAGMA_EXP_FUSE_GEMM=0 keeps it apart
      GemmSpec gs{};
      const bool fuse = fast && mode == MIDAGMA_MODE_COV && cov_split > 1 && fuse_gemm;
      if (fuse) gs = score_cov_spec();
      gemm_done = enqueue_build_inverse(fast, passes, fuse ? &gs : nullptr);
    } else if (forked_inverse()) {
      // fork: the inverse (latency-bound, a few % of the chip) on the side stream, the n x d
      // GEMMs on the main one; joined before anything reads Mt.  With the blocked layout the
      // slow (pivoted, no warm start) two-level inverse: ~5x fewer workgroup-microseconds
      // taken from the GEMMs than the flat Gauss-Jordan's 32 x 1024 workgroups
      const bool bl = data_binv_on();
      launch_build_at(W.p, D, /*square=*/true, bl ? binv_build_target(Mt.p, D, binv()) : Mt.p, D, d, 0.0, d_params,
                      d_state, stream, IW.p);
      HIP_TRY(hipEventRecord(ev_fork, stream));
      HIP_TRY(hipStreamWaitEvent(side, ev_fork, 0));
      if (bl)
        launch_blocked_inverse(Mt.p, D, binv(), /*fast=*/false, gj(), d_state, side);
      else
        launch_gj_inverse(Mt.p, D, D, gj(), d_state, side);
      HIP_TRY(hipEventRecord(ev_join, side));
    } else {
      launch_build_at(W.p, D, /*square=*/true, Mt.p, D, d, 0.0, d_params, d_state, stream, IW.p);
      launch_gj_inverse(Mt.p, D, D, gj(), d_state, stream);
    }
    // (a fork/join of the score GEMMs onto a second stream inside the graph measured slower:
    // the cross-queue dependencies cost more than the overlap gains)
    if (mode == MIDAGMA_MODE_COV) {
      // rhs = ((-mu) cov) @ (I - W)    (linear.py:244); a fast slot leaves the split-K slices
      // for fused_update to sum (its only reader there)
      if (!gemm_done) enqueue_score_cov(zbuf, d_state, /*sum=*/!(fast && blocked()));
    } else if (!gemm_done) {
      enqueue_data_partial(W.p, d_state, IW.p);
      enqueue_slot_allreduce();  // beside the forked inverse, before the join
      if (forked_inverse()) HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
    }
    // trek regularizer of this slot's W (linear.py:251-258): every slot in 'opt' mode; in 'log'
    // mode only checkpoint slots, which are never fast slots
    if (trek_on && (tcfg.mode == 2 || !(fast && blocked()))) {
      if (trek_tcc)
        launch_trek_tcc(W.p, d, D, ccfg, cw, d_state, Gtrek.p, stream);
      else
        launch_trek_pst(W.p, d, D, tcfg, tw, d_state, Gtrek.p, stream);
    }
  }

  // the score partial (and the logistic loss tail) summed over the ranks, in place on the
  // solver stream, while a whole slot is being captured with a communicator attached
  void enqueue_slot_allreduce() {
    if (inslot_comm) comm_allreduce(comm, zbuf, (size_t)(D * D + 64), false, stream);
  }

  // every rank's (status, iters) at a poll: one max all-reduce into agree[slot], copied to h_agree
  void enqueue_agree(int slot) {
    if (!comm) return;
    launch_agree_pack(d_state, agree.p + 4 * slot, stream);
    comm_allreduce(comm, agree.p + 4 * slot, 4, true, stream);
    HIP_TRY(hipMemcpyAsync(h_agree + 4 * slot, agree.p + 4 * slot, 4 * sizeof(double), hipMemcpyDeviceToHost, stream));
  }
  void check_agree(int slot) const {
    if (!comm) return;
    const double* a = h_agree + 4 * slot;
    if (a[0] != -a[2] || a[1] != -a[3])
      throw std::runtime_error("data-parallel replicas diverged: (status, iters) ranges over ranks [" +
                               std::to_string(-a[2]) + ", " + std::to_string(a[0]) + "], [" + std::to_string(-a[3]) +
                               ", " + std::to_string(a[1]) + "] (pin NCCL_ALGO=Ring)");
  }

  // blocked layout: build_at and the two-level inverse (fast: warm-started diagonal blocks, as
  // one dataflow launch when df_on)
  // fuse (nullable): a GEMM the inverse may carry in its last trailing launch; returns whether it did
  bool enqueue_build_inverse(bool fast, int passes, const GemmSpec* fuse = nullptr) {
#ifdef MIDAGMA_EXPERIMENTS
    if (fast && df_on) {
      launch_build_at(W.p, D, /*square=*/true, dfw.A[0], D, d, 0.0, d_params, d_state, stream, IW.p);
      launch_df_inverse(Mt.p, D, dfw, binv(), passes <= 2 ? 2 : 3, d_state, stream);
      return false;
    }
#endif
    // experiments build, MIDAGMA_EXP_BUILD_RESID0=1: outer block 0's residual rides in build_at's
    // launch on fast slots at B2 = 256 (one dependent launch fewer, but measured slower: DESIGN 8)
#ifdef MIDAGMA_EXPERIMENTS
    const bool resid0 = fast && IW.p == nullptr && binv_block(D) == 256 && !cov_la_on() && build_resid0_on();
    if (resid0)
      launch_build_resid0(W.p, D, binv_build_target(Mt.p, D, binv()), D, d, d_params, binv(), d_state, stream);
    else
#else
    const bool resid0 = false;
#endif
      launch_build_at(W.p, D, /*square=*/true, binv_build_target(Mt.p, D, binv()), D, d, 0.0, d_params, d_state,
                      stream, IW.p);
    if (fast && cov_la_on()) {
      const int64_t K2 = D / B2;
      if ((int64_t)la_ev.size() < 2 * K2 + 2) {
        for (size_t i = la_ev.size(); i < (size_t)(2 * K2 + 2); ++i) {
          hipEvent_t e = nullptr;
          HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
          la_ev.push_back(e);
        }
      }
      const TrailLookAhead tla{side, la_ev.data()};
      return launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, stream, passes, fuse, &tla);
    }
    return launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, stream, passes, fuse, nullptr, resid0);
  }
#ifdef MIDAGMA_EXPERIMENTS
  // experiment knob MIDAGMA_EXP_BUILD_RESID0=1: build_at and block 0's residual in one launch
  static bool build_resid0_on() {
    static const bool on = knob("MIDAGMA_EXP_BUILD_RESID0", 0) != 0;
    return on;
  }
#endif
  bool fuse_gemm = knob("MIDAGMA_EXP_FUSE_GEMM", 1) != 0;

  // the cov score GEMM as enqueue_cov_gemm launches it on a fast slot (split-K slices, unsummed)
  GemmSpec score_cov_spec() const {
    GemmSpec gs{};
    gs.M = D;
    gs.N = D;
    gs.K = Kd();
    gs.A = cov_at ? covsT.p : covs.p;
    gs.lda = D;
    gs.a_trans = cov_at;
    gs.B = IW.p ? IW.p : W.p;
    gs.ldb = D;
    gs.bmode = IW.p ? B_PLAIN : B_IMINUS;
    gs.C = cov_parts.p;
    gs.ldc = D;
    gs.split = cov_split;
    gs.slice_stride = D * D;
    return gs;
  }

  // rhs = ((-mu) cov) @ (I - W) from the slot's operands: A read k-major from ((-mu) cov)^T
  // (cov_at), B = I - W formed by build_at (IW, plain B) when the slot keeps it
  void enqueue_score_cov(double* out, const State* st, bool sum) {
    const double* A = cov_at ? covsT.p : covs.p;
    if (IW.p)
      enqueue_cov_gemm(A, IW.p, out, st, sum, cov_at, B_PLAIN);
    else
      enqueue_cov_gemm(A, W.p, out, st, sum, cov_at, B_IMINUS);
  }

  // out = Cm @ (I - Wp) on the d x d problem; split-K over fixed slices when the tile grid
  // alone cannot fill the chip (summed in fixed order: deterministic)
  // a_trans: Cm holds the transpose of the left operand
  // (bmode B_PLAIN: Wp already holds I - W)
  void enqueue_cov_gemm(const double* Cm, const double* Wp, double* out, const State* st, bool sum = true,
                        bool a_trans = false, GemmB bmode = B_IMINUS) {
#ifdef MIDAGMA_EXPERIMENTS
    // experiment: the forked score GEMM confined to the first MIDAGMA_EXP_GEMM_SES shader engines of
    // every XCD, so the inverse's launches on the side stream keep the other CUs to themselves
    static const int gemm_ses = (int)knob("MIDAGMA_EXP_GEMM_SES", 0);
    if (gemm_ses > 0 && cov_fork_on() && D % 128 == 0) {
      if (!cupart_ctr.p) throw std::logic_error("cupart counter not allocated");
      double* dst = cov_split > 1 ? cov_parts.p : out;
      launch_gemm_cupart(D, D, Kd(), Cm, D, a_trans, Wp, D, bmode, dst, D, cov_split, D * D, st, gemm_ses,
                         reinterpret_cast<int*>(cupart_ctr.p), stream);
      if (cov_split > 1 && sum) launch_sum_slices(cov_parts.p, cov_split, D * D, D * D, out, st, stream);
      return;
    }
#endif
    if (cov_split > 1) {
      launch_gemm(D, D, Kd(), Cm, D, a_trans, Wp, D, bmode, cov_parts.p, D, EPI_STORE, cov_split, D * D, nullptr, 0,
                  0, st, stream);
      if (sum) launch_sum_slices(cov_parts.p, cov_split, D * D, D * D, out, st, stream);
    } else {
      launch_gemm(D, D, Kd(), Cm, D, a_trans, Wp, D, bmode, out, D, EPI_STORE, 1, 0, nullptr, 0, 0, st, stream);
    }
  }

  // Z_k = X_k^T (X_k (I - W))  (l2)   or   X_k^T expit(X_k W)  (logistic, + loss partial)
  // iw (nullable): I - W already formed (build_at), the plain-B form of the GEMM
  void enqueue_data_partial(const double* Wp, const State* st, const double* iw = nullptr) {
    if (loss == MIDAGMA_LOSS_L2) {
      launch_gemm(n_pad, D, Kd(), xw_a(), xw_lda(), use_xt, iw ? iw : Wp, D, iw ? B_PLAIN : B_IMINUS, Y.p, D, EPI_STORE, 1,
                  0, nullptr, 0, 0, st, stream);
    } else {
      launch_gemm(n_pad, D, Kd(), xw_a(), xw_lda(), use_xt, Wp, D, B_PLAIN, Y.p, D, EPI_SIGMOID, sig_split,
                  sig_split > 1 ? n_pad * D : 0, loss_part.p, n_local, d, st, stream);
      launch_sum_vector(loss_part.p, loss_part_count, zbuf + D * D, st, stream);
    }
    if (split == 1) {
      launch_gemm(D, D, n_pad, X.p, D, true, Y.p, D, B_PLAIN, zbuf, D, EPI_STORE, 1, 0, nullptr, 0, 0, st, stream);
    } else {
      launch_gemm(D, D, n_pad, X.p, D, true, Y.p, D, B_PLAIN, Zparts.p, D, EPI_STORE, split, D * D, nullptr, 0, 0,
                  st, stream);
      launch_sum_slices(Zparts.p, split, D * D, D * D, zbuf, st, stream);
    }
  }

  // fast (blocked cov slots): the domain flags come from the inverse's last outer step and the
  // score slices are summed inside fused_update; fast slots never carry a checkpoint
  void enqueue_part2(bool fast = false) {
    const bool lean = fast && blocked();
    if (!lean) launch_reduce_check(Mt.p, W.p, zbuf, d_params, d_state, partials.p, d, D, stream);
    launch_control(d_params, d_state, partials.p, pivlog.p, zbuf + D * D, bc_table.p, d_ckpt, ckpt_cap, npart.p, d,
                   trek_on ? (trek_tcc ? cw.scal : tw.scal) : nullptr, stream);
    const bool slices = lean && mode == MIDAGMA_MODE_COV && cov_split > 1;
    launch_fused_update(d_params, d_state, W.p, m.p, v.p, Mt.p, slices ? cov_parts.p : zbuf,
                        slices ? cov_split : 1, D * D, cov.p, has_inc ? minc.p : nullptr, has_exc ? mexc.p : nullptr,
                        trek_on && tcfg.mode == 2 ? Gtrek.p : nullptr, d, D, npart.p, stream);
  }

  hipGraphExec_t capture(int which, int reps = 1, int passes = NM_PASSES_RUN) {
    hipGraph_t graph = nullptr;
    HIP_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    inslot_comm = comm != nullptr && mode == MIDAGMA_MODE_DATA && (which & 3) == 3;
    try {
      for (int r = 0; r < reps; ++r) {
        if (which & 1) enqueue_part1((which & 4) != 0, passes);
        if (which & 2) enqueue_part2((which & 4) != 0);
      }
      inslot_comm = false;
    } catch (...) {
      inslot_comm = false;
      (void)hipStreamEndCapture(stream, &graph);
      if (graph) (void)hipGraphDestroy(graph);
      throw;
    }
    HIP_TRY(hipStreamEndCapture(stream, &graph));
    hipGraphExec_t exec = nullptr;
    HIP_TRY(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    HIP_TRY(hipGraphDestroy(graph));
    return exec;
  }

  void ensure_graphs() {
    if (graphs_valid) return;
    destroy_graphs();
    g_full = capture(3);
    g_part1 = capture(1);
    g_part2 = capture(2);
    if (blocked()) {
      g_fast = capture(3 | 4);
      if (fast_group > 1) g_fastN = capture(3 | 4, fast_group);
      if (nm_adapt) {
        g_fast2 = capture(3 | 4, 1, 2);
        if (fast_group > 1) g_fastN2 = capture(3 | 4, fast_group, 2);
      }
    }
    graphs_valid = true;
  }

  // ---- trek regularizer ---------------------------------------------------------
  void set_trek(int seq, int agg, int tmode, double weight, double eps_inv, int64_t K, const int64_t* pairs,
                int64_t mpairs) {
    if (tmode == 0 || mpairs <= 0 || weight == 0.0) {  // TrekRegularizer.enabled() false, or no pairs
      trek_on = false;
      graphs_valid = false;
      return;
    }
    if (seq < 0 || seq > 3 || agg < 0 || agg > 3 || tmode < 1 || tmode > 2)
      throw std::invalid_argument("set_trek: bad seq / agg / mode");
    if (seq == TREK_LOG && K < 1) throw std::invalid_argument("set_trek: K_log must be >= 1");
    const size_t DD = (size_t)D * D;
    int nq = 2;
    if (seq == TREK_EXP) nq = TREK_TAYLOR_M + 1;
    if (seq == TREK_BINOM) nq = 64 - __builtin_clzll((unsigned long long)d) + 2;
    const int nbuf = 11 + nq + TREK_SMAX + 1 + 2;
    if ((int)tbufs.size() < nbuf) tbufs.resize(nbuf);
    for (int i = 0; i < nbuf; ++i) tbufs[i].alloc(DD);
    int b = 0;
    TrekWork w{};
    w.gj = gj();
    for (double** slot : {&w.X, &w.F, &w.H, &w.S, &w.GT, &w.L, &w.tmp, &w.tmp2, &w.tmp3, &w.tmp4}) *slot = tbufs[b++].p;
    ++b;  // spare
    for (int i = 0; i < nq; ++i) w.Q[i] = tbufs[b++].p;
    for (int i = 0; i <= TREK_SMAX; ++i) w.E[i] = tbufs[b++].p;
    w.dQ[0] = tbufs[b++].p;
    w.dQ[1] = tbufs[b++].p;
    if (D % 128 == 0 && (D / 128) * (D / 128) < 256) {
      tslices.alloc(4 * DD);
      w.slices = tslices.p;
    }
    tsmall.alloc((size_t)(D / 64) * D + 4 * 256 + 16);
    w.colpart = tsmall.p;
    w.part = tsmall.p + (D / 64) * D;
    w.scal = w.part + 4 * 256;
    HIP_TRY(hipMemsetAsync(tsmall.p, 0, tsmall.n * sizeof(double), stream));
    if (!tgates) HIP_TRY(hipMalloc(&tgates, (1 + 2 * TREK_SMAX) * sizeof(State)));
    HIP_TRY(hipMemsetAsync(tgates, 0, (1 + 2 * TREK_SMAX) * sizeof(State), stream));
    w.gates = tgates;
    Gtrek.alloc(DD);
    HIP_TRY(hipMemsetAsync(Gtrek.p, 0, DD * sizeof(double), stream));
    std::vector<int32_t> pr(2 * mpairs);
    for (int64_t i = 0; i < 2 * mpairs; ++i) {
      if (pairs[i] < 0 || pairs[i] >= d) throw std::invalid_argument("set_trek: pair index out of range");
      pr[i] = (int32_t)pairs[i];
    }
    tpairs.alloc((size_t)(mpairs + 1));  // 2 int32 per double slot
    HIP_TRY(hipMemcpy(tpairs.p, pr.data(), pr.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    TrekCfg c{};
    c.seq = seq;
    c.agg = agg;
    c.mode = tmode;
    c.weight = weight;
    c.eps_inv = eps_inv;
    c.K = seq == TREK_BINOM ? (int)d : (int)K;
    c.smax = TREK_SMAX;
    c.m = mpairs;
    c.pairs = reinterpret_cast<const int32_t*>(tpairs.p);
    tcfg = c;
    tw = w;
    trek_on = true;
    trek_tcc = false;
    ensure_probe();
    graphs_valid = false;
  }

  void ensure_probe() {
    if (!d_state_probe) {
      HIP_TRY(hipMalloc(&d_state_probe, sizeof(State)));
      State probe{};
      probe.status = ST_RUNNING;
      probe.ckpt_pending = 1;
      HIP_TRY(hipMemcpy(d_state_probe, &probe, sizeof(State), hipMemcpyHostToDevice));
    }
  }

  // TCC (notreks TCCRegularizer as trek_value_grad runs it): w multiplies S, eps as the reference
  void set_trek_tcc(int tmode, double weight, double wS, double eps, const int64_t* pairs, int64_t mpairs) {
    if (tmode == 0 || mpairs <= 0 || weight == 0.0) {
      trek_on = false;
      graphs_valid = false;
      return;
    }
    if (tmode < 1 || tmode > 2) throw std::invalid_argument("set_trek_tcc: bad mode");
    std::vector<double> S((size_t)D * D, 0.0);
    for (int64_t k = 0; k < mpairs; ++k) {
      const int64_t i = pairs[2 * k], j = pairs[2 * k + 1];
      if (i < 0 || i >= d || j < 0 || j >= d) throw std::invalid_argument("set_trek_tcc: pair index out of range");
      S[(size_t)i * D + j] = 1.0;  // S[rows, cols] = 1 (notreks _indicator_from_pairs)
    }
    const int64_t D2 = round_up64(2 * d);
    const int64_t nch = (2 * d + 63) / 64;
    cA.alloc((size_t)D2 * D2);
    cMi.alloc((size_t)D2 * D2);
    cS.alloc((size_t)D * D);
    cvec.alloc((size_t)6 * D2 + 16);
    cpart.alloc((size_t)nch * D2);
    cP.alloc(2 * 32 * 32);
    cR.alloc((size_t)2 * 32 * D2);
    cC.alloc((size_t)2 * D2 * 32);
    HIP_TRY(hipMemcpy(cS.p, S.data(), S.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(cvec.p, 0, cvec.n * sizeof(double)));  // warm flag off, vectors 0
    if (!cgates) HIP_TRY(hipMalloc(&cgates, (1 + TCC_NODA_MAX) * sizeof(State)));
    HIP_TRY(hipMemset(cgates, 0, (1 + TCC_NODA_MAX) * sizeof(State)));
    TccWork w{};
    w.gj = GJWork{cP.p, cR.p, cC.p, nullptr, nullptr};
    w.D2 = D2;
    w.A = cA.p;
    w.Mi = cMi.p;
    w.S = cS.p;
    double* v = cvec.p;
    for (double** slot : {&w.x, &w.y, &w.u, &w.z, &w.vprev, &w.uprev}) {
      *slot = v;
      v += D2;
    }
    w.scal = v;
    w.part = cpart.p;
    w.gates = cgates;
    cw = w;
    ccfg = TccCfg{tmode, weight, wS, eps, mpairs};
    Gtrek.alloc((size_t)D * D);
    HIP_TRY(hipMemset(Gtrek.p, 0, (size_t)D * D * sizeof(double)));
    tcfg = TrekCfg{};
    tcfg.mode = tmode;
    tcfg.weight = weight;
    tcfg.m = mpairs;
    trek_on = true;
    trek_tcc = true;
    ensure_probe();
    graphs_valid = false;
  }

  // ---- buffers -------------------------------------------------------------
  void alloc_core() {
    const size_t DD = (size_t)D * D;
    for (DevBuf* b : {&W, &m, &v, &Mt, &cov, &covs, &covsT}) {
      b->alloc(DD);
      HIP_TRY(hipMemsetAsync(b->p, 0, DD * sizeof(double), stream));
    }
    P.alloc(64 * 64);
    R.alloc((size_t)64 * D);
    C.alloc((size_t)D * 64);
    pivlog.alloc(D);
    Pstore.alloc((size_t)D * 32);
    partials.alloc(2 * NRED);
    npart.alloc((size_t)((d + NTHREADS - 1) / NTHREADS) * d * NORM_FIELDS);
    HIP_TRY(hipMemsetAsync(npart.p, 0, npart.n * sizeof(double), stream));
    scarry.alloc(NORM_FIELDS + 1);
    HIP_TRY(hipMemsetAsync(scarry.p, 0, scarry.n * sizeof(double), stream));
    if (small_block(d) > 0) sprev.alloc(2 * (size_t)small_block(d) * small_block(d));
    if (D % 128 == 0) {
      // split-K of the cov score GEMM: small grids get slices to fill the chip; large ones the
      // split that best rounds the last wave of 128-tiles (2 workgroups per CU resident:
      // 1600 tiles at d = 5000 leave the 4th wave 1/8 full, split 4 -> 13 full-ish waves)
      const int64_t tiles = (D / 128) * (D / 128), slots = 2 * 256;
      if (tiles < 256) {
        // about one workgroup per CU: round(256 / tiles + 1/4), at most 4 and D / 128 (measured,
        // fused with the last trailing update: D = 1152 split 3 2909 vs 4 2770 steps/s; D = 1408
        // split 2 2016 vs 4 1985; D = 1792 split 2 1480 vs 4 1452 vs 1 1406; D = 1024 split 4)
        cov_split = (int)std::max<int64_t>(
            1, std::min<int64_t>({4, D / 128, (int64_t)(256.0 / (double)tiles + 0.75)}));
      } else if (tiles >= 1024) {  // (256..1023 tiles: split 1 measured best at d = 2000)
        double best = 1e30;
        for (int sp = 1; sp <= 4; ++sp) {
          const double waves = (double)((tiles * sp + slots - 1) / slots) / sp * (1.0 + 0.03 * (sp - 1));
          if (waves < best) best = waves, cov_split = sp;
        }
      }
      if (knob_set("MIDAGMA_EXP_COV_SPLIT")) cov_split = (int)knob("MIDAGMA_EXP_COV_SPLIT", cov_split);
      if (cov_split > 1) cov_parts.alloc((size_t)cov_split * DD);
    }
    if (mode == MIDAGMA_MODE_COV) B2 = binv_block(D);
    // cov mode: build_at also writes I - W for the score GEMM's plain-B form
    if (mode == MIDAGMA_MODE_COV && ((D % 128 == 0 && cov_iw) || w32)) IW.alloc(DD);
    if (blocked() || data_binv_on()) {
      const int64_t b2 = binv_block(D);
      Malt.alloc(DD);
      Pst2.alloc((size_t)D * b2);
      Pst2b.alloc((size_t)D * b2);
      for (DevBuf* b : {&nmY0, &nmY1, &nmQ0, &nmQ1, &nmP, &nmLW, &nmLZ, &nmLPZ}) b->alloc((size_t)b2 * b2);
      nmPart.alloc((size_t)(D / b2) * (NM_PASSES + 1) * PART_STRIDE);
      nmDone.alloc(D / b2);
      nmSync.alloc((size_t)(D / b2) * 128);  // 256 ints per block (launch_trail128_series' counters)
      HIP_TRY(hipMemsetAsync(nmSync.p, 0, (size_t)(D / b2) * 128 * sizeof(double), stream));
    }
#ifdef MIDAGMA_EXPERIMENTS
    if (blocked() && mode == MIDAGMA_MODE_COV && df_available(D) && knob("MIDAGMA_EXP_DF", 0) != 0) setup_df();
#endif
    zown.alloc(DD + 64);
    HIP_TRY(hipMemsetAsync(zown.p, 0, (DD + 64) * sizeof(double), stream));
    zbuf = zown.p;
    zbuf_cap = (int64_t)DD + 64;
    HIP_TRY(hipMalloc(&d_params, sizeof(Params)));
    HIP_TRY(hipMalloc(&d_state, sizeof(State)));
    HIP_TRY(hipHostMalloc(&h_state, 2 * sizeof(State), hipHostMallocDefault));
    for (auto& e : ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if ((mode == MIDAGMA_MODE_DATA && fork_inv) ||
        (mode == MIDAGMA_MODE_COV && (cov_fork || cov_la) && B2 > 0 && (D - B2 >= 1792 || cov_fork_all))) {
      // Default priority: a fork / join between a high-priority stream and another one left the
      // process's later two-stream work ~5x slower (the config-5 step after a data-mode solver:
      // 7.5k -> 1.3k steps/s, also after a plain torch fork / join; tools/probe_after_data.py),
      // and the forked inverse hides just as well without it (config 4: 17.46 vs 17.50 steps/s
      // at n = 1e6, 133.8 vs 133.5 at the 8-GPU shard n = 125k)
      HIP_TRY(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
      if (kExperiments) cupart_ctr.alloc(1);  // (launch_gemm_cupart's counter; not while capturing)
    }
  }

#ifdef MIDAGMA_EXPERIMENTS
  // buffers and the two task plans (2 and 3 product-form passes) of the one-launch inverse
  void setup_df() {
    const int64_t K2 = D / 256, BB = 256 * 256, DD = D * D;
    int ncu = 0;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
    // workgroups per CU (the kernel's registers admit 2; every one must be resident)
    static const int per_cu = std::max(1, std::min(2, (int)knob("MIDAGMA_EXP_DF_PER_CU", 2)));
    ncu *= per_cu;
    dfA.alloc((size_t)K2 * DD);
    dfY.alloc((size_t)K2 * (NM_PASSES + 1) * BB);
    dfQ.alloc((size_t)K2 * (NM_PASSES + 1) * BB);
    dfP.alloc((size_t)K2 * BB);
    const int64_t nctl = df_ctl_ints(D);
    dfCtl.alloc((size_t)(nctl + 1) / 2);
    HIP_TRY(hipMemset(dfCtl.p, 0, (size_t)nctl * sizeof(int)));
    for (int k = 0; k < 2; ++k) {
      const DfPlanHost pl = df_plan(D, k == 0 ? 2 : 3, ncu);
      dfTasks[k].alloc((pl.tasks->size() + 1) / 2);
      dfWoff[k].alloc((pl.woff->size() + 1) / 2);
      HIP_TRY(hipMemcpy(dfTasks[k].p, pl.tasks->data(), pl.tasks->size() * sizeof(int), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(dfWoff[k].p, pl.woff->data(), pl.woff->size() * sizeof(int), hipMemcpyHostToDevice));
      dfw.tasks[k] = reinterpret_cast<const int*>(dfTasks[k].p);
      dfw.woff[k] = reinterpret_cast<const int*>(dfWoff[k].p);
    }
    for (int64_t g = 0; g < K2; ++g) dfw.A[g] = dfA.p + g * DD;
    dfw.Y = dfY.p;
    dfw.Q = dfQ.p;
    dfw.P = dfP.p;
    dfw.ctl = reinterpret_cast<int*>(dfCtl.p);
    dfw.nwg = ncu;
    if (knob_set("MIDAGMA_DF_STAMPS")) {  // diagnostics: per-task timestamps of the last launch
      dfStamps.alloc((size_t)3 * std::max(df_plan(D, 3, ncu).tasks->size(), df_plan(D, 2, ncu).tasks->size()) / 12);
      HIP_TRY(hipMemset(dfStamps.p, 0, dfStamps.n * sizeof(double)));
      dfw.stamps = reinterpret_cast<unsigned long long*>(dfStamps.p);
    }
    df_on = true;
  }
  // wait timeouts of the one-launch inverse so far (a planning bug; the solver raises on it)
  int df_timeouts() {
    if (!df_on) return 0;
    int t = 0;
    HIP_TRY(hipMemcpy(&t, dfw.ctl + 2 * 32, sizeof(int), hipMemcpyDeviceToHost));
    return t;
  }
#else
  int df_timeouts() { return 0; }
#endif

  void upload_matrix(DevBuf& dst, const double* src, int64_t ld_src) {
    HIP_TRY(hipMemcpy2DAsync(dst.p, D * sizeof(double), src, ld_src * sizeof(double), d * sizeof(double), d,
                             hipMemcpyHostToDevice, stream));
  }

  void download_matrix(double* dst, const double* src) {
    HIP_TRY(hipMemcpy2DAsync(dst, d * sizeof(double), src, D * sizeof(double), d * sizeof(double), d,
                             hipMemcpyDeviceToHost, stream));
  }

  void ensure_bc_table(double b1, double b2, int64_t max_iter) {
    if (b1 == bc_b1 && b2 == bc_b2 && max_iter <= bc_len) return;
    const int64_t len = std::max<int64_t>(max_iter, 1);
    std::vector<double> t(2 * len);
    for (int64_t it = 1; it <= len; ++it) {  // (1 - beta ** iter) exactly as Python computes it (linear.py:160-161)
      t[2 * (it - 1)] = 1 - ::pow(b1, (double)it);
      t[2 * (it - 1) + 1] = 1 - ::pow(b2, (double)it);
    }
    bc_table.alloc(2 * len);
    HIP_TRY(hipMemcpy(bc_table.p, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
    bc_b1 = b1;
    bc_b2 = b2;
    bc_len = len;
    graphs_valid = false;  // table pointer may have changed
  }

  void ensure_ckpt(int64_t max_iter, int64_t checkpoint) {
    const int64_t need = max_iter / std::max<int64_t>(checkpoint, 1) + 4;
    if (need <= ckpt_cap) return;
    if (d_ckpt) HIP_TRY(hipFree(d_ckpt));
    HIP_TRY(hipMalloc(&d_ckpt, need * sizeof(CkptRec)));
    ckpt_cap = need;
    graphs_valid = false;
  }

  void begin(const double* Wh, double mu_, int64_t max_iter, double s, double lr, double tol, double b1, double b2,
             double lambda1, int64_t checkpoint) {
    if (mode == MIDAGMA_MODE_COV && !has_cov) throw std::invalid_argument("set_cov before minimize");
    if (mode == MIDAGMA_MODE_DATA && !has_data) throw std::invalid_argument("set_data before minimize");
    if (loss == MIDAGMA_LOSS_LOGISTIC && !has_cov) throw std::invalid_argument("logistic needs cov (cov_from_zbuf)");
    if (max_iter < 1 || checkpoint < 1) throw std::invalid_argument("max_iter and checkpoint must be >= 1");
    mu = mu_;
    ensure_bc_table(b1, b2, max_iter);
    ensure_ckpt(max_iter, checkpoint);
    Params p{};
    p.mu = mu_;
    p.s = s;
    p.lambda1 = lambda1;
    p.tol = tol;
    p.beta1 = b1;
    p.beta2 = b2;
    p.c1 = 1 - b1;
    p.c2 = 1 - b2;
    // (float32 W: mu * lambda1 * sign(W) is a float32 array, linear.py:248)
    p.mu_l1 = w32 ? f32r(mu_ * lambda1) : mu_ * lambda1;
    p.w32 = w32 ? 1 : 0;
    p.d_log_s = (double)d * std::log(s);
    p.max_iter = max_iter;
    p.checkpoint = checkpoint;
    p.d = d;
    p.D = D;
    p.ld_table = bc_len;
    p.has_inc = has_inc;
    p.has_exc = has_exc;
    p.logistic = loss == MIDAGMA_LOSS_LOGISTIC;
    p.trek_weight = trek_on ? tcfg.weight : 0.0;
    p.trek_mode = trek_on ? tcfg.mode : 0;
    const double n = (double)n_global;
    if (mode == MIDAGMA_MODE_COV) {
      p.zscale = 1.0;  // Z already is ((-mu) cov) @ (I - W)
      p.cscale = 0.0;
      p.score_scale = 0.5 / (-mu_);
    } else if (loss == MIDAGMA_LOSS_L2) {
      p.zscale = -mu_ / n;
      p.cscale = 0.0;
      p.score_scale = 0.5 / n;
    } else {
      p.zscale = mu_ / n;
      p.cscale = -mu_;
      p.score_scale = 0.0;
      p.logit_scale = 1.0 / n;
    }
    hp = p;
    HIP_TRY(hipMemcpyAsync(d_params, &hp, sizeof(Params), hipMemcpyHostToDevice, stream));
    State st{};
    st.status = ST_RUNNING;
    st.lr = lr;
    st.obj_prev = 1e16;
    h_state[0] = st;
    HIP_TRY(hipMemcpyAsync(d_state, &h_state[0], sizeof(State), hipMemcpyHostToDevice, stream));
    if (mode == MIDAGMA_MODE_COV) {
      launch_scale(cov.p, -mu_, covs.p, D * D, stream);  // (-mu) * cov
      launch_transpose(covs.p, D, D, D, covsT.p, D, stream);
    }
    upload_matrix(W, Wh, d);
    const size_t DD = (size_t)D * D;
    for (DevBuf* b : {&m, &v}) HIP_TRY(hipMemsetAsync(b->p, 0, DD * sizeof(double), stream));
    HIP_TRY(hipMemsetAsync(scarry.p, 0, scarry.n * sizeof(double), stream));  // no warm start yet
    HIP_TRY(hipStreamSynchronize(stream));  // h_state[0] reused as a snapshot slot below
    fast_ready = false;  // the first slot of a call runs the GJ path (warm starts are stale)
    three_pass_left = 0;
    begun = true;
  }

  void snapshot(int slot) {
    HIP_TRY(hipMemcpyAsync(&h_state[slot], d_state, sizeof(State), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipEventRecord(ev[slot], stream));
  }

  static bool terminal(const State& s) { return s.status != ST_RUNNING; }

  // Cov mode with the blocked inverse: fast slots in batches, a GJ (slow) slot wherever a
  // log-det is due (checkpoint), there is no warm start (first slot) or a fast slot handed
  // back (ST_NEED_GJ).  Batches stop at the next checkpoint iteration, so the host knows
  // when the slow slot is due; one host sync per batch (the choices: slot_sched.h, BlockedScheduler).
  // n_slots < 0: until terminal.
  void drive_blocked(int64_t n_slots) {
    ensure_graphs();
    BlockedScheduler::Carry carry;
    carry.bmax = fast_batch;
    carry.three_pass_left = three_pass_left;
    carry.fast_ready = fast_ready;
    BlockedScheduler sc(hp.max_iter, hp.checkpoint, n_slots, fast_group, g_fast2 != nullptr, carry);
    HIP_TRY(hipMemcpyAsync(&h_state[1], d_state, sizeof(State), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    for (SlotView cur = view(h_state[1]);;) {
      const BlockedPlan p = sc.next(cur);
      if (p.done) break;
      if (p.clear_handback) {
        static const int32_t running = ST_RUNNING;
        HIP_TRY(hipMemcpyAsync(&d_state->status, &running, sizeof(int32_t), hipMemcpyHostToDevice, stream));
      }
      if (eager) {
        if (p.slow) run_eager(false, NM_PASSES_RUN, 1);
        run_eager(true, p.two_pass ? 2 : NM_PASSES_RUN, p.groups * fast_group + p.singles);
      } else {
        if (p.slow) HIP_TRY(hipGraphLaunch(g_full, stream));  // pivots + fresh warm starts
        // (a hand-back inside a group turns the group's later slots into no-op launches)
        hipGraphExec_t one = p.two_pass ? g_fast2 : g_fast, grp = p.two_pass ? g_fastN2 : g_fastN;
        for (int64_t b = 0; b < p.groups; ++b) HIP_TRY(hipGraphLaunch(grp, stream));
        for (int64_t b = 0; b < p.singles; ++b) HIP_TRY(hipGraphLaunch(one, stream));
      }
      HIP_TRY(hipMemcpyAsync(&h_state[1], d_state, sizeof(State), hipMemcpyDeviceToHost, stream));
      enqueue_agree(0);
      HIP_TRY(hipStreamSynchronize(stream));
      check_agree(0);
      cur = view(h_state[1]);
      sc.observe(cur);
    }
    fast_batch = sc.carry().bmax;
    three_pass_left = sc.carry().three_pass_left;
    fast_ready = sc.carry().fast_ready;
    handback_count += sc.handbacks();
    if (const int to = df_timeouts()) throw std::runtime_error("one-launch inverse: " + std::to_string(to) + " wait timeouts");
    static const bool dbg = knob_set("MIDAGMA_DEBUG_HANDBACKS");  // diagnostics (experiments build)
    if (dbg)
      fprintf(stderr, "drive_blocked: %lld slots, %lld hand-backs\n", (long long)sc.launched(), (long long)sc.handbacks());
  }
  static SlotView view(const State& st) {
    SlotView v;
    v.status = st.status;
    v.ckpt_pending = st.ckpt_pending;
    v.iter = st.iter;
    v.slots = st.slots;
    return v;
  }
  int64_t handback_count = 0;
  int fast_group = std::max(1, (int)knob("MIDAGMA_EXP_FAST_GROUP", 4));
  int64_t fast_batch = BlockedScheduler::kMaxBatch;

  // Small d: the whole inner loop in one persistent workgroup, kSmallBatch slots per launch
  // (one host sync per launch).  n_slots < 0: until terminal.
  static constexpr int64_t kSmallBatch = 4096;
  void drive_small(int64_t n_slots) {
    const int64_t cap = slot_cap(hp.max_iter, hp.checkpoint);
    for (int64_t launched = 0;;) {
      const int64_t B = small_next_batch(n_slots, launched, cap, kSmallBatch);
      if (B <= 0) break;
      SmallTcc tc{};
      if (trek_on && trek_tcc)
        tc = SmallTcc{cw.S, ccfg.w, ccfg.eps, (double)ccfg.m, ccfg.weight, ccfg.mode, cw.scal, cw.vprev, cw.uprev};
      launch_small_minimize(d_params, d_state, W.p, m.p, v.p, covs.p, has_inc ? minc.p : nullptr,
                            has_exc ? mexc.p : nullptr, bc_table.p, d_ckpt, ckpt_cap, scarry.p, sprev.p, d, B,
                            stream, trek_on && trek_tcc ? &tc : nullptr, w32);
      launched += B;
      HIP_TRY(hipMemcpyAsync(&h_state[1], d_state, sizeof(State), hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      if (terminal(h_state[1])) break;
    }
  }

  void run_loop(int64_t max_iter, int64_t checkpoint) {
    if (blocked()) {
      drive_blocked(-1);
      return;
    }
    if (small_on()) {
      drive_small(-1);
      return;
    }
    ensure_graphs();
    const int64_t cap = slot_cap(max_iter, checkpoint);
    int64_t launched = 0, known_iter = 0;
    int cur = 0, pending = -1;
    bool stop = false;
    while (!stop) {
      const int64_t B = graph_next_batch(max_iter, known_iter);
      for (int64_t b = 0; b < B; ++b) HIP_TRY(hipGraphLaunch(g_full, stream));
      launched += B;
      enqueue_agree(cur);
      snapshot(cur);
      if (pending >= 0) {
        HIP_TRY(hipEventSynchronize(ev[pending]));
        check_agree(pending);
        known_iter = h_state[pending].iter;
        if (terminal(h_state[pending])) stop = true;
      }
      pending = cur;
      cur ^= 1;
      if (!stop && launched > cap) throw std::runtime_error("minimize: slot budget exceeded (controller stuck)");
    }
    HIP_TRY(hipStreamSynchronize(stream));
  }

  void finish(double* Wh, midagma_result* res) {
    HIP_TRY(hipMemcpyAsync(&h_state[0], d_state, sizeof(State), hipMemcpyDeviceToHost, stream));
    download_matrix(Wh, W.p);
    HIP_TRY(hipStreamSynchronize(stream));
    begun = false;
    check_handoff(h_state[0]);
    fill_result(h_state[0], res);
  }

  // the serial split sigmoid GEMM's per-tile hand-off words (gemm.hip, sig_split_take): after the
  // output and the first halves' partial in Y
  void clear_sig_flags() {
    if (sig_split != 2) return;
    const int64_t tiles = (n_pad / 128) * (D / 128);
    HIP_TRY(hipMemsetAsync(Y.p + 2 * n_pad * D, 0, (size_t)(tiles + 1) / 2 * sizeof(double), stream));
  }
  // A bounded in-kernel hand-off wait expired (ST_HANDOFF_TIMEOUT; never expected): the late
  // first half has finished with its launch, so its word is cleared here, and the call raises
  // instead of reporting a numerical outcome.
  void check_handoff(const State& s) {
    if (s.status != ST_HANDOFF_TIMEOUT) return;
    begun = false;
    clear_sig_flags();
    HIP_TRY(hipStreamSynchronize(stream));
    throw std::runtime_error("sigmoid GEMM: a K-half hand-off wait timed out (50 ms); the step was not applied");
  }

  static void fill_result(const State& s, midagma_result* res) {
    if (!res) return;
    res->iters = s.iter;
    res->halvings = s.halvings;
    res->slots = s.slots;
    res->n_checkpoints = s.n_ckpt;
    res->status = s.status == ST_NEED_GJ ? ST_RUNNING : s.status;  // internal hand-back, not an outcome
    res->early_stop = s.early_stop;
    res->lr_final = s.lr;
    res->obj_last = s.obj_last;
    res->score_last = s.score_last;
    res->h_last = s.h_last;
    res->l1_last = s.l1_last;
  }
};

namespace {

__global__ void div_kernel(const double* __restrict__ x, double n, double* __restrict__ y, int64_t count) {
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < count; i += (int64_t)gridDim.x * NTHREADS)
    y[i] = x[i] / n;
}

int fail(midagma_solver* s, int code, const std::string& msg) {
  if (s)
    s->err = msg;
  else
    g_global_error = msg;
  return code;
}

template <class F>
int guarded(midagma_solver* s, F&& f) {
  try {
    if (s) HIP_TRY(hipSetDevice(s->device));
    return f();
  } catch (const HipError& e) {
    return fail(s, MIDAGMA_E_HIP, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(s, MIDAGMA_E_ARG, e.what());
  } catch (const std::exception& e) {
    return fail(s, MIDAGMA_E_STATE, e.what());
  }
}

std::once_flag g_attr_once;
void setup_attributes_once() {
  std::call_once(g_attr_once, [] {
    gj_setup_attributes();
    gemm_setup_attributes();
  });
}

// A minimize that ended ST_SINGULAR: the reference's sla.inv raised at that step.  scipy
// raises ValueError when sI - W*W has a non-finite entry (check_finite: W itself went
// non-finite, e.g. from non-finite data) and LinAlgError when the finite matrix is singular.
int singular_or_nonfinite(midagma_solver* s, int rc, const midagma_result* res, const double* W) {
  if (rc != MIDAGMA_OK || !res || res->status != MIDAGMA_ST_SINGULAR) return rc;
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("minimize: ") + kNonFinite);
  return fail(s, MIDAGMA_E_SINGULAR, "singular matrix: inverse of sI - W*W is not finite");
}

}  // namespace

extern "C" {

int midagma_abi_version(void) { return MIDAGMA_ABI_VERSION; }

int midagma_device_count(int* n) {
  return guarded(nullptr, [&] {
    HIP_TRY(hipGetDeviceCount(n));
    return MIDAGMA_OK;
  });
}

const char* midagma_last_error(const midagma_solver* s) { return s ? s->err.c_str() : g_global_error.c_str(); }

int midagma_create(midagma_solver** out, int loss, int mode, int64_t d, int device, void* stream) {
  if (!out || d < 1 || (loss != 0 && loss != 1) || (mode != 0 && mode != 1) ||
      (loss == MIDAGMA_LOSS_LOGISTIC && mode == MIDAGMA_MODE_COV))
    return fail(nullptr, MIDAGMA_E_ARG, "midagma_create: bad arguments (logistic needs data mode)");
  midagma_solver* s = new midagma_solver();
  s->loss = loss;
  s->mode = mode;
  s->d = d;
  // 128-multiples feed the 128x128 GEMM tiles.  Cov mode pads 129 <= d <= 192 to 256 as well: the
  // blocked inverse then has one 256-wide outer block, and its warm-started product form beats
  // the flat Gauss-Jordan's 6 block steps on 192 (data mode keeps 192: X's columns are GEMM work)
  const bool pad256 = mode == MIDAGMA_MODE_COV && knob("MIDAGMA_EXP_COV_PAD256", 1) != 0;
  s->D = d > 192 || (pad256 && d > 128) ? (d + 127) / 128 * 128 : round_up64(d);
  // Cov mode, 256 < d <= 640: D to a multiple of 256, so the blocked inverse runs B2 = 256 outer
  // blocks (2 instead of 3 at D = 384 -> 512, 3 instead of 5 at 640 -> 768: d=300 11.1k -> 11.3k,
  // d=600 6.4k -> 7.0k steps/s).  Larger D keep B2 = 128 (d=1150 even, d=1400 -3.5%, d=1700
  // even: the padded GEMM work outweighs the saved outer steps).  Knob MIDAGMA_EXP_COV_PAD_B2:
  // 0 off, 1 at every d > 256.
  const int pad_b2 = (int)knob("MIDAGMA_EXP_COV_PAD_B2", -1);
  if (mode == MIDAGMA_MODE_COV && d > 256 && (pad_b2 == 1 || (pad_b2 < 0 && d <= 640)))
    s->D = (d + 255) / 256 * 256;
  s->device = device;
  int rc = guarded(s, [&] {
    setup_attributes_once();
    if (stream) {
      s->stream = reinterpret_cast<hipStream_t>(stream);
    } else {
      HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
      s->own_stream = true;
    }
    s->alloc_core();
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
  if (rc != MIDAGMA_OK) {
    g_global_error = s->err;
    delete s;
    return rc;
  }
  *out = s;
  return MIDAGMA_OK;
}

void midagma_destroy(midagma_solver* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  delete s;
}

void* midagma_stream(midagma_solver* s) { return s ? reinterpret_cast<void*>(s->stream) : nullptr; }
int64_t midagma_padded_dim(const midagma_solver* s) { return s ? s->D : 0; }

int midagma_set_cov(midagma_solver* s, const double* cov, int64_t ld) {
  if (!s || !cov || ld < s->d) return fail(s, MIDAGMA_E_ARG, "set_cov: bad arguments");
  if (!all_finite(cov, s->d, s->d, ld)) return fail(s, MIDAGMA_E_ARG, std::string("set_cov: ") + kNonFinite);
  return guarded(s, [&] {
    s->upload_matrix(s->cov, cov, ld);
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_set_masks(midagma_solver* s, const double* mask_inc, const double* mask_exc) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "set_masks: null solver");
  return guarded(s, [&] {
    const size_t DD = (size_t)s->D * s->D;
    const bool inc = mask_inc != nullptr, exc = mask_exc != nullptr;
    if (inc) {
      s->minc.alloc(DD);
      HIP_TRY(hipMemsetAsync(s->minc.p, 0, DD * sizeof(double), s->stream));
      s->upload_matrix(s->minc, mask_inc, s->d);
    }
    if (exc) {
      s->mexc.alloc(DD);
      HIP_TRY(hipMemsetAsync(s->mexc.p, 0, DD * sizeof(double), s->stream));
      s->upload_matrix(s->mexc, mask_exc, s->d);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    const double* pi = inc ? s->minc.p : nullptr;
    const double* pe = exc ? s->mexc.p : nullptr;
    if (pi != s->cap_minc || pe != s->cap_mexc) s->graphs_valid = false;  // captured pointers changed
    s->cap_minc = pi;
    s->cap_mexc = pe;
    s->has_inc = inc;
    s->has_exc = exc;
    return MIDAGMA_OK;
  });
}

int midagma_set_data(midagma_solver* s, const double* X, int64_t n_local, int64_t n_global, int on_device) {
  if (!s || !X || n_local < 1 || n_global < n_local || s->mode != MIDAGMA_MODE_DATA)
    return fail(s, MIDAGMA_E_ARG, "set_data: bad arguments (data mode only)");
  if (!on_device && !all_finite(X, n_local, s->d, s->d))
    return fail(s, MIDAGMA_E_ARG, std::string("set_data: ") + kNonFinite);
  return guarded(s, [&] {
    const int64_t D = s->D;
    s->n_local = n_local;
    s->n_global = n_global;
    s->n_pad = (n_local + 127) / 128 * 128;
    const size_t nx = (size_t)s->n_pad * D;
    s->X.alloc(nx);
    // logistic with few 128-tiles: the sigmoid GEMM in two serial K halves when its last round of
    // tiles would be at most half full (n = 1e4, d = 1000: 632 tiles for 512 resident slots)
    const int64_t sig_tiles = (s->n_pad / 128) * (D / 128);
    const int sig_rule = (int)knob("MIDAGMA_EXP_SIG_SPLIT", 1);
    const bool sig_ok = s->loss == MIDAGMA_LOSS_LOGISTIC && D % 128 == 0 && sig_tiles % 8 == 0;
    s->sig_split = sig_ok && sig_rule > 0 && sig_tiles < 2048 && sig_tiles % 512 != 0 && sig_tiles % 512 <= 256 ? 2 : 1;
    if (s->sig_split_force == 1) s->sig_split = 1;  // midagma_debug_sig_split (tests)
    if (s->sig_split_force == 2 && sig_ok) s->sig_split = 2;
    if (s->sig_split == 2) {  // the output, the first halves' partial, then one flag word per tile
      s->Y.alloc(2 * nx + (size_t)(sig_tiles + 1) / 2);
      HIP_TRY(hipMemsetAsync(s->Y.p + 2 * nx, 0, (size_t)(sig_tiles + 1) / 2 * sizeof(double), s->stream));
    } else {
      s->Y.alloc(nx);
    }
    HIP_TRY(hipMemsetAsync(s->X.p, 0, nx * sizeof(double), s->stream));
    HIP_TRY(hipMemcpy2DAsync(s->X.p, D * sizeof(double), X, s->d * sizeof(double), s->d * sizeof(double), n_local,
                             on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s->stream));
    if (on_device) {  // the host path checked before the copy
      int* flag = reinterpret_cast<int*>(s->partials.p);
      launch_any_nonfinite(s->X.p, (int64_t)nx, flag, s->stream);
      int bad = 0;
      HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, s->stream));
      HIP_TRY(hipStreamSynchronize(s->stream));
      if (bad) throw std::invalid_argument(std::string("set_data: ") + kNonFinite);
    }
    size_t mem_free = 0, mem_total = 0;
    HIP_TRY(hipMemGetInfo(&mem_free, &mem_total));
    // (the 128-tile GEMM only: D % 128 == 0; smaller problems are not worth the copy)
    s->use_xt = getenv("MIDAGMA_NO_XT") == nullptr && D % 128 == 0 &&
                mem_free > nx * sizeof(double) + (size_t(2) << 30);
    if (s->use_xt) {
      s->XT.alloc(nx);
      launch_transpose(s->X.p, D, s->n_pad, D, s->XT.p, s->n_pad, s->stream);
    } else {
      s->XT.release();
    }
    if (s->loss == MIDAGMA_LOSS_L2 && (D % 128 == 0 || s->w32))  // (float32 W: I - W from build_at)
      s->IW.alloc((size_t)D * D);
    else
      s->IW.release();
    // split-K over the rows so the X^T Y GEMM fills the chip: (D/64)^2 tiles x split >= ~1024 workgroups
    const int64_t tiles = (D % 128 == 0) ? (D / 128) * (D / 128) : (D / 64) * (D / 64);
    const int64_t ktiles = s->n_pad / 64;
    int split = (int)std::max<int64_t>(1, std::min<int64_t>(ktiles / 8, (1024 + tiles - 1) / tiles));
    s->split = std::min(split, 32);
    if (knob_set("MIDAGMA_EXP_DATA_SPLIT")) s->split = (int)knob("MIDAGMA_EXP_DATA_SPLIT", s->split);
    if (s->split > 1) s->Zparts.alloc((size_t)s->split * D * D);
    s->loss_part_count = (s->n_pad / 64) * (D / 64);
    // small shards run the cov-mode slot structure: the warm-started fast blocked inverse in
    // sequence with the GEMMs (hand-backs and checkpoint slots on the pivoted path).  Forked beside
    // GEMMs that fill the chip, the pivoted inverse's 20-odd dependent launches wait for CU slots
    // and end after the GEMMs (logistic d=1000, n=1e4: 1.01 ms per slot for 0.70 ms of GEMMs);
    // large shards keep the fork, which hides it (MIDAGMA_EXP_DATA_FAST_ROWS: the row bound)
    static const int64_t fast_rows = knob("MIDAGMA_EXP_DATA_FAST_ROWS", 16384);
    const int b2 = binv_block(D);
    const int B2_new = (b2 > 0 && s->n_pad <= fast_rows && s->Malt.p) ? b2 : 0;
    if (B2_new != s->B2) s->graphs_valid = false;
    s->B2 = B2_new;
    if (s->loss == MIDAGMA_LOSS_LOGISTIC) {
      s->loss_part.alloc(s->loss_part_count);
      HIP_TRY(hipMemsetAsync(s->loss_part.p, 0, s->loss_part_count * sizeof(double), s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_data = true;
    s->graphs_valid = false;
    return MIDAGMA_OK;
  });
}

int midagma_data_gram(midagma_solver* s) {
  if (!s || !s->has_data) return fail(s, MIDAGMA_E_STATE, "data_gram: set_data first");
  return guarded(s, [&] {
    const int64_t D = s->D;
    if (s->split == 1)
      launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->X.p, D, B_PLAIN, s->zbuf, D, EPI_STORE, 1, 0, nullptr, 0, 0,
                  nullptr, s->stream);
    else {
      launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->X.p, D, B_PLAIN, s->Zparts.p, D, EPI_STORE, s->split, D * D,
                  nullptr, 0, 0, nullptr, s->stream);
      launch_sum_slices(s->Zparts.p, s->split, D * D, D * D, s->zbuf, nullptr, s->stream);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_cov_from_zbuf(midagma_solver* s, double n) {
  if (!s || !(n > 0)) return fail(s, MIDAGMA_E_ARG, "cov_from_zbuf: n must be > 0");
  return guarded(s, [&] {
    // cov = (X^T X) / float(n), a division as in linear.py:428
    const int64_t DD = s->D * s->D;
    hipLaunchKernelGGL(div_kernel, dim3(4096), dim3(NTHREADS), 0, s->stream, s->zbuf, n, s->cov.p, DD);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_get_cov(midagma_solver* s, double* out, int64_t ld) {
  if (!s || !out || ld < s->d) return fail(s, MIDAGMA_E_ARG, "get_cov: bad arguments");
  if (!s->has_cov) return fail(s, MIDAGMA_E_STATE, "get_cov: no cov (set_cov or cov_from_zbuf first)");
  return guarded(s, [&] {
    HIP_TRY(hipMemcpy2DAsync(out, ld * sizeof(double), s->cov.p, s->D * sizeof(double), s->d * sizeof(double), s->d,
                             hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

// ABI 7: fit()'s data preparation on device memory (linear.py:406-428), csrc/gram.hip.
int midagma_colsum_dev(const double* X, int64_t n, int64_t d, int64_t ldx, double* out_dev, void* stream) {
  if (n < 0 || d < 1 || ldx < d || !out_dev || (n > 0 && !X))
    return fail(nullptr, MIDAGMA_E_ARG, "colsum_dev: bad arguments");
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    DevBuf part;
    part.alloc((size_t)colsum_parts(n) * d);
    launch_colsum(X, n, d, ldx, part.p, out_dev, st);
    HIP_TRY(hipStreamSynchronize(st));  // the partials are freed on return
    return MIDAGMA_OK;
  });
}

int midagma_center_dev(double* X, int64_t n, int64_t d, int64_t ldx, const double* colsum_dev, double nrows,
                       void* stream) {
  if (n < 0 || d < 1 || ldx < d || !colsum_dev || (n > 0 && !X) || !(nrows > 0))
    return fail(nullptr, MIDAGMA_E_ARG, "center_dev: bad arguments");
  return guarded(nullptr, [&] {
    launch_center(X, n, d, ldx, colsum_dev, nrows, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

int midagma_gram(const double* X, int64_t n, int64_t d, int64_t ldx, int on_device, double* G_dev, int64_t ldg,
                 void* stream) {
  if (n < 0 || d < 1 || ldx < d || !G_dev || ldg < d || (n > 0 && !X))
    return fail(nullptr, MIDAGMA_E_ARG, "gram: bad arguments");
  return guarded(nullptr, [&] {
    setup_attributes_once();
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    static const int64_t chunk_rows = [] {
      const char* e = getenv("MIDAGMA_GRAM_CHUNK_ROWS");
      return e ? std::max<int64_t>(256, atoll(e)) : int64_t(262144);
    }();
    const GramPlan p = gram_plan(n, d, chunk_rows);
    const int64_t D = p.D, DD = D * D;
    DevBuf S, Z, fl;
    S.alloc((size_t)p.chunk * D);
    Z.alloc((size_t)(p.split + 2) * DD);  // [0] the running sum, [1..split] a chunk's slices, [split+1] the new sum
    fl.alloc(1);
    int* flag = reinterpret_cast<int*>(fl.p);
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), st));
    HIP_TRY(hipMemsetAsync(Z.p, 0, DD * sizeof(double), st));
    if (!on_device) HIP_TRY(hipMemsetAsync(S.p, 0, (size_t)p.chunk * D * sizeof(double), st));
    for (int64_t c = 0; c < p.nchunks; ++c) {
      const int64_t r0 = c * p.chunk, rows = std::min(p.chunk, n - r0);
      const int64_t rpad = (rows + 255) / 256 * 256;
      if (on_device) {
        launch_stage_rows(X + r0 * ldx, ldx, rows, d, S.p, D, rpad, flag, st);
      } else {
        if (rows < rpad) HIP_TRY(hipMemsetAsync(S.p + rows * D, 0, (rpad - rows) * D * sizeof(double), st));
        HIP_TRY(hipMemcpy2DAsync(S.p, D * sizeof(double), X + r0 * ldx, ldx * sizeof(double), d * sizeof(double),
                                 rows, hipMemcpyHostToDevice, st));
        launch_nonfinite_or(S.p, rows, d, D, flag, st);
      }
      launch_gemm(D, D, rpad, S.p, D, true, S.p, D, B_PLAIN, Z.p + DD, D, EPI_STORE, p.split, DD, nullptr, 0, 0,
                  nullptr, st);
      launch_sum_slices(Z.p, p.split + 1, DD, DD, Z.p + (p.split + 1) * DD, nullptr, st);
      HIP_TRY(hipMemcpyAsync(Z.p, Z.p + (p.split + 1) * DD, DD * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(hipMemcpy2DAsync(G_dev, ldg * sizeof(double), Z.p, D * sizeof(double), d * sizeof(double), d,
                             hipMemcpyDeviceToDevice, st));
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (bad) throw std::invalid_argument(std::string("gram: ") + kNonFinite);
    return MIDAGMA_OK;
  });
}

int midagma_set_cov_dev(midagma_solver* s, const double* G_dev, int64_t ldg, double divisor) {
  if (!s || !G_dev || ldg < s->d || !(divisor > 0)) return fail(s, MIDAGMA_E_ARG, "set_cov_dev: bad arguments");
  return guarded(s, [&] {
    // cov = (X^T X) / float(n), a division as in linear.py:428 (the caller all-reduced the Gram)
    int* flag = reinterpret_cast<int*>(s->partials.p);
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), s->stream));
    launch_div_block(G_dev, ldg, divisor, s->d, s->cov.p, s->D, flag, s->stream);
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (bad) throw std::invalid_argument(std::string("set_cov_dev: ") + kNonFinite);
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_comm_unique_id(void* out, int64_t cap) {
  if (!out || cap < 128) return fail(nullptr, MIDAGMA_E_ARG, "comm_unique_id: needs a 128-byte buffer");
  return guarded(nullptr, [&] { return comm_unique_id(out); });
}

int midagma_comm_init(midagma_solver* s, const void* id, int64_t id_len, int nranks, int rank) {
  if (!s || !id || id_len != 128 || nranks < 1 || rank < 0 || rank >= nranks || s->mode != MIDAGMA_MODE_DATA)
    return fail(s, MIDAGMA_E_ARG, "comm_init: bad arguments (data mode, a 128-byte unique id, 0 <= rank < nranks)");
  return guarded(s, [&] {
    HIP_TRY(hipStreamSynchronize(s->stream));
    comm_destroy(s->comm);
    s->comm = nullptr;
    s->comm = comm_create(id, nranks, rank);
    s->comm_ranks = nranks;
    s->agree.alloc(8);
    if (!s->h_agree) HIP_TRY(hipHostMalloc(&s->h_agree, 8 * sizeof(double), hipHostMallocDefault));
    s->graphs_valid = false;  // the slot graphs now carry the all-reduce
    return MIDAGMA_OK;
  });
}

int midagma_comm_ranks(const midagma_solver* s) { return s ? (s->comm ? s->comm_ranks : 0) : 0; }

int midagma_comm_allreduce_zbuf(midagma_solver* s) {
  if (!s || !s->comm) return fail(s, MIDAGMA_E_STATE, "comm_allreduce_zbuf: comm_init first");
  return guarded(s, [&] {
    comm_allreduce(s->comm, s->zbuf, (size_t)(s->D * s->D + 64), false, s->stream);
    return MIDAGMA_OK;
  });
}

int64_t midagma_zbuf_len(const midagma_solver* s) { return s ? s->D * s->D + 64 : 0; }

int midagma_bind_zbuf(midagma_solver* s, void* dev_ptr, int64_t len) {
  if (!s || len < s->D * s->D + 64) return fail(s, MIDAGMA_E_ARG, "bind_zbuf: buffer too small");
  return guarded(s, [&] {
    s->zbuf = dev_ptr ? static_cast<double*>(dev_ptr) : s->zown.p;
    s->graphs_valid = false;
    return MIDAGMA_OK;
  });
}

int midagma_minimize(midagma_solver* s, double* W, double mu, int64_t max_iter, double s_dom, double lr, double tol,
                     double beta1, double beta2, double lambda1, int64_t checkpoint, midagma_result* res) {
  if (!s || !W) return fail(s, MIDAGMA_E_ARG, "minimize: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("minimize: ") + kNonFinite);
  int rc = guarded(s, [&] {
    s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
    s->run_loop(max_iter, checkpoint);
    s->finish(W, res);
    return MIDAGMA_OK;
  });
  return singular_or_nonfinite(s, rc, res, W);
}

int midagma_begin(midagma_solver* s, const double* W, double mu, int64_t max_iter, double s_dom, double lr,
                  double tol, double beta1, double beta2, double lambda1, int64_t checkpoint) {
  if (!s || !W) return fail(s, MIDAGMA_E_ARG, "begin: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("begin: ") + kNonFinite);
  return guarded(s, [&] {
    s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
    s->ensure_graphs();
    return MIDAGMA_OK;
  });
}

int midagma_run_slots(midagma_solver* s, int64_t n) {
  if (!s || !s->begun || n < 0) return fail(s, MIDAGMA_E_STATE, "run_slots: call begin first");
  return guarded(s, [&] {
    if (s->blocked()) {
      s->drive_blocked(n);
      return MIDAGMA_OK;
    }
    if (s->small_on()) {
      s->drive_small(n);
      return MIDAGMA_OK;
    }
    for (int64_t i = 0; i < n; ++i) HIP_TRY(hipGraphLaunch(s->g_full, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_sync(midagma_solver* s) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_profile_parts(midagma_solver* s, int reps, double* ms_out) {
  if (!s || !s->begun || reps < 1 || !ms_out) return fail(s, MIDAGMA_E_STATE, "profile_parts: call begin first");
  return guarded(s, [&] {
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    auto timed = [&](auto&& body) {
      HIP_TRY(hipEventRecord(a, s->stream));
      for (int r = 0; r < reps; ++r) body();
      HIP_TRY(hipEventRecord(b, s->stream));
      HIP_TRY(hipEventSynchronize(b));
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, a, b));
      return (double)ms / reps;
    };
    const int64_t D = s->D;
    // [0] build (sI - W o W)^T   [1] GJ inverse   [2] score GEMM(s)   [3] whole slot (graph)
    // data mode: [4] Y = X (I - W) GEMM   [5] Z = X^T Y GEMM (+ slice sum)
    ms_out[0] = timed([&] { launch_build_at(s->W.p, D, true, s->Mt.p, D, s->d, 0.0, s->d_params, s->d_state,
                                            s->stream, s->IW.p); });
    ms_out[1] = timed([&] { launch_gj_inverse(s->Mt.p, D, D, s->gj(), s->d_state, s->stream); });
    if (s->mode == MIDAGMA_MODE_COV) {
      ms_out[2] = timed([&] { s->enqueue_score_cov(s->zbuf, s->d_state, true); });
      ms_out[4] = ms_out[5] = 0.0;
    } else {
      ms_out[2] = timed([&] { s->enqueue_data_partial(s->W.p, s->d_state, s->IW.p); });
      ms_out[4] = timed([&] {
        if (s->loss == MIDAGMA_LOSS_L2)
          launch_gemm(s->n_pad, D, s->Kd(), s->xw_a(), s->xw_lda(), s->use_xt, s->IW.p ? s->IW.p : s->W.p, D,
                      s->IW.p ? B_PLAIN : B_IMINUS, s->Y.p, D, EPI_STORE, 1, 0, nullptr, 0, 0, s->d_state, s->stream);
        else
          launch_gemm(s->n_pad, D, s->Kd(), s->xw_a(), s->xw_lda(), s->use_xt, s->W.p, D, B_PLAIN, s->Y.p, D, EPI_SIGMOID,
                      s->sig_split, s->sig_split > 1 ? s->n_pad * D : 0, s->loss_part.p, s->n_local, s->d,
                      s->d_state, s->stream);
      });
      ms_out[5] = timed([&] {
        if (s->split == 1)
          launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->Y.p, D, B_PLAIN, s->zbuf, D, EPI_STORE, 1, 0, nullptr, 0, 0,
                      s->d_state, s->stream);
        else {
          launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->Y.p, D, B_PLAIN, s->Zparts.p, D, EPI_STORE, s->split,
                      D * D, nullptr, 0, 0, s->d_state, s->stream);
          launch_sum_slices(s->Zparts.p, s->split, D * D, D * D, s->zbuf, s->d_state, s->stream);
        }
      });
    }
    ms_out[3] = timed([&] { HIP_TRY(hipGraphLaunch(s->g_full, s->stream)); });
    ms_out[6] = ms_out[7] = 0.0;
    if (s->blocked()) {
      // [6] build + fast blocked inverse, less [0]   [7] whole fast slot (graph).  Both need a
      // warm start and no pending checkpoint: one slow slot first.
      HIP_TRY(hipGraphLaunch(s->g_full, s->stream));
      ms_out[6] = timed([&] { s->enqueue_build_inverse(/*fast=*/true, 2); }) - ms_out[0];
      ms_out[7] = timed([&] { HIP_TRY(hipGraphLaunch(s->g_fast, s->stream)); });
      State st{};
      HIP_TRY(hipMemcpy(&st, s->d_state, sizeof(State), hipMemcpyDeviceToHost));
      if (st.status == ST_NEED_GJ) {  // the fast path did not run: report it, leave a clean state
        ms_out[6] = ms_out[7] = -1.0;
        static const int32_t running = ST_RUNNING;
        HIP_TRY(hipMemcpy(&s->d_state->status, &running, sizeof(int32_t), hipMemcpyHostToDevice));
        s->fast_ready = false;
      }
    }
    HIP_TRY(hipEventDestroy(a));
    HIP_TRY(hipEventDestroy(b));
    return MIDAGMA_OK;
  });
}

int midagma_step_partial(midagma_solver* s) {
  if (!s || !s->begun) return fail(s, MIDAGMA_E_STATE, "step_partial: call begin first");
  return guarded(s, [&] {
    HIP_TRY(hipGraphLaunch(s->g_part1, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_step_finish(midagma_solver* s) {
  if (!s || !s->begun) return fail(s, MIDAGMA_E_STATE, "step_finish: call begin first");
  return guarded(s, [&] {
    HIP_TRY(hipGraphLaunch(s->g_part2, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_poll(midagma_solver* s, midagma_result* res) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    HIP_TRY(hipMemcpyAsync(&s->h_state[1], s->d_state, sizeof(State), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->check_handoff(s->h_state[1]);
    midagma_solver::fill_result(s->h_state[1], res);
    return MIDAGMA_OK;
  });
}

int midagma_end(midagma_solver* s, double* W, midagma_result* res) {
  if (!s || !W || !s->begun) return fail(s, MIDAGMA_E_STATE, "end: call begin first");
  int rc = guarded(s, [&] {
    s->finish(W, res);
    return MIDAGMA_OK;
  });
  return singular_or_nonfinite(s, rc, res, W);
}

int midagma_set_w_float32(midagma_solver* s, int float32) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    const bool on = float32 != 0;
    if (on && (s->mode == MIDAGMA_MODE_COV || s->loss == MIDAGMA_LOSS_L2) && !s->IW.p) {
      // the score GEMM's I - W (float32 diagonal) comes from build_at, not the GEMM's staging
      s->IW.alloc((size_t)s->D * s->D);
      HIP_TRY(hipMemsetAsync(s->IW.p, 0, (size_t)s->D * s->D * sizeof(double), s->stream));
      s->graphs_valid = false;
    }
    s->w32 = on;
    return MIDAGMA_OK;
  });
}

// Test hook (not in the public header): choose the logistic sigmoid GEMM's form for the next
// set_data (0: the size rule, 1: the one-pass kernel, 2: the serial K split wherever the shape
// allows it; -1: no change).  Returns the form the current data uses (1 or 2).
extern "C" int midagma_debug_sig_split(midagma_solver* s, int mode) {
  if (!s || mode < -1 || mode > 2) return -1;
  if (mode >= 0) s->sig_split_force = mode;
  return s->sig_split;
}

// Test hooks (not in the public header) for the hand-back path of the blocked inverse:
// spoil_warm zeroes the stored diagonal-block inverses of the last two slots, so the next fast
// slot's warm start is 0, its residual I, and its first product-form pass hands the slot back
// (ST_NEED_GJ) while the rest of the slot (in data mode: the score GEMMs beside the forked
// inverse) is running; handbacks counts the hand-backs the scheduler has re-run.
extern "C" int midagma_debug_spoil_warm(midagma_solver* s) {
  if (!s || !s->blocked()) return -1;
  return guarded(s, [&] {
    for (DevBuf* b : {&s->Pst2, &s->Pst2b})
      if (b->p) HIP_TRY(hipMemsetAsync(b->p, 0, b->n * sizeof(double), s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}
extern "C" int64_t midagma_debug_handbacks(const midagma_solver* s) { return s ? s->handback_count : -1; }

// Diagnostics of the fast blocked inverse (not in the public header): per outer block g,
// out[g*(NM_PASSES+2) + 0] = done word, out[... + 1 + p] = ||Q_p||_inf of pass p (stale for
// passes that did not run in the last slot).
extern "C" int midagma_debug_blocked(midagma_solver* s, double* out, int64_t cap) {
  if (!s || !s->blocked()) return 0;
  const int64_t K2 = s->D / s->B2, per = NM_PASSES + 2;
  if (cap < K2 * per) return -1;
  std::vector<double> part((size_t)K2 * (NM_PASSES + 1) * PART_STRIDE);
  std::vector<int> done(K2);
  if (hipMemcpy(part.data(), s->nmPart.p, part.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (hipMemcpy(done.data(), s->nmDone.p, K2 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  const int B2 = s->B2, NT = B2 / 16;
  for (int64_t g = 0; g < K2; ++g) {
    out[g * per] = done[g];
    for (int p = 0; p <= NM_PASSES; ++p) {
      const double* rp = part.data() + ((size_t)g * (NM_PASSES + 1) + p) * PART_STRIDE;
      double m = 0.0;
      for (int r = 0; r < B2; ++r) {
        double acc = 0.0;
        for (int t = 0; t < NT; ++t) acc += rp[r * NT + t];
        m = std::max(m, acc);
      }
      out[g * per + 1 + p] = m;
    }
  }
  return (int)K2;
}

int64_t midagma_checkpoints(midagma_solver* s, midagma_ckpt* out, int64_t cap) {
  if (!s || !s->d_ckpt) return 0;
  int64_t n = 0;
  int rc = guarded(s, [&] {
    State st{};
    HIP_TRY(hipMemcpy(&st, s->d_state, sizeof(State), hipMemcpyDeviceToHost));
    n = std::min<int64_t>(std::min<int64_t>(st.n_ckpt, s->ckpt_cap), cap);
    static_assert(sizeof(midagma_ckpt) == sizeof(CkptRec), "ckpt layout");
    if (n > 0 && out) HIP_TRY(hipMemcpy(out, s->d_ckpt, n * sizeof(CkptRec), hipMemcpyDeviceToHost));
    return MIDAGMA_OK;
  });
  return rc == MIDAGMA_OK ? n : rc;
}

int midagma_set_trek(midagma_solver* s, int seq, int agg, int mode, double weight, double eps_inv, int64_t K,
                     const int64_t* pairs, int64_t m) {
  if (!s || (m > 0 && !pairs) || m < 0) return fail(s, MIDAGMA_E_ARG, "set_trek: bad arguments");
  return guarded(s, [&] {
    s->set_trek(seq, agg, mode, weight, eps_inv, K, pairs, m);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_set_trek_tcc(midagma_solver* s, int mode, double weight, double w, double eps, const int64_t* pairs,
                         int64_t m) {
  if (!s || (m > 0 && !pairs) || m < 0) return fail(s, MIDAGMA_E_ARG, "set_trek_tcc: bad arguments");
  return guarded(s, [&] {
    s->set_trek_tcc(mode, weight, w, eps, pairs, m);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_trek(midagma_solver* s, const double* W, double* value, double* G) {
  if (!s || !W || !value) return fail(s, MIDAGMA_E_ARG, "trek: null argument");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    if (!s->trek_on) {  // trek_value_grad: (0, zeros) when disabled (notreks.py)
      *value = 0.0;
      if (G) std::fill(G, G + d * d, 0.0);
      return MIDAGMA_OK;
    }
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    const double* scal;
    if (s->trek_tcc) {
      TccCfg c = s->ccfg;
      c.weight = 1.0;  // the bare gradient, as trek_value_grad returns it
      launch_trek_tcc(s->scratch.p, d, D, c, s->cw, s->d_state_probe, s->Gtrek.p, s->stream);
      scal = s->cw.scal;
    } else {
      TrekCfg c = s->tcfg;
      c.weight = 1.0;
      launch_trek_pst(s->scratch.p, d, D, c, s->tw, s->d_state_probe, s->Gtrek.p, s->stream);
      scal = s->tw.scal;
    }
    HIP_TRY(hipMemcpyAsync(value, scal, sizeof(double), hipMemcpyDeviceToHost, s->stream));
    if (G) {
      if (s->tcfg.mode == 2) {
        HIP_TRY(hipMemcpy2DAsync(G, d * sizeof(double), s->Gtrek.p, D * sizeof(double), d * sizeof(double), d,
                                 hipMemcpyDeviceToHost, s->stream));
      } else {
        std::fill(G, G + d * d, 0.0);
      }
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_h(midagma_solver* s, const double* W, double s_dom, double* h, double* G) {
  if (!s || !W || !h) return fail(s, MIDAGMA_E_ARG, "h: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("h: ") + kNonFinite);
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    DevBuf work;
    work.alloc(DD);
    launch_build_at(s->scratch.p, D, true, work.p, D, d, s_dom, nullptr, nullptr, s->stream);
    GJWork gw = s->gj();
    gw.Pstore = nullptr;
    launch_gj_inverse(work.p, D, D, gw, nullptr, s->stream);
    std::vector<double> pl(D);
    HIP_TRY(hipMemcpyAsync(pl.data(), s->pivlog.p, D * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    if (G) {
      s->Gtmp.alloc((size_t)d * d);
      launch_h_grad(s->scratch.p, work.p, s->Gtmp.p, d, D, s->stream);
      HIP_TRY(hipMemcpyAsync(G, s->Gtmp.p, (size_t)d * d * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    work.release();
    double ld = 0.0;
    for (int64_t i = 0; i < d; ++i) ld += pl[i];
    *h = -ld + (double)d * std::log(s_dom);
    return MIDAGMA_OK;
  });
}

static void host_trace_l1(midagma_solver* s, const double* Wd, const double* Z, double* sd, double* l1) {
  launch_trace_l1(Wd, Z, s->partials.p, s->d, s->D, s->stream);
  std::vector<double> part(2 * NRED);
  HIP_TRY(hipMemcpyAsync(part.data(), s->partials.p, part.size() * sizeof(double), hipMemcpyDeviceToHost,
                         s->stream));
  HIP_TRY(hipStreamSynchronize(s->stream));
  double a = 0.0, b = 0.0;
  for (int i = 0; i < NRED; ++i) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  *sd = a;
  if (l1) *l1 = b;
}

int midagma_score(midagma_solver* s, const double* W, double* loss, double* G) {
  if (!s || !W || !loss) return fail(s, MIDAGMA_E_ARG, "score: null argument");
  if (s->mode != MIDAGMA_MODE_COV || !s->has_cov) return fail(s, MIDAGMA_E_STATE, "score: cov mode with set_cov");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    DevBuf rhs;
    rhs.alloc(DD);
    s->enqueue_cov_gemm(s->cov.p, s->scratch.p, rhs.p, nullptr);  // rhs = cov @ (I - W)   (linear.py:85-86)
    double sd = 0;
    host_trace_l1(s, s->scratch.p, rhs.p, &sd, nullptr);
    *loss = 0.5 * sd;
    if (G) {
      s->Gtmp.alloc((size_t)d * d);
      launch_scale(rhs.p, -1.0, rhs.p, DD, s->stream);  // G_loss = -rhs
      s->download_matrix(G, rhs.p);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    rhs.release();
    return MIDAGMA_OK;
  });
}

int midagma_score_partial(midagma_solver* s, const double* W) {
  if (!s || !W || s->mode != MIDAGMA_MODE_DATA || !s->has_data)
    return fail(s, MIDAGMA_E_STATE, "score_partial: data mode with set_data");
  return guarded(s, [&] {
    const int64_t DD = s->D * s->D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, s->d);
    HIP_TRY(hipMemsetAsync(s->zbuf + DD, 0, 64 * sizeof(double), s->stream));
    // Force loss partials: pass no state (st == nullptr computes them unconditionally).
    s->enqueue_data_partial(s->scratch.p, nullptr);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_score_finish(midagma_solver* s, double* loss, double* G) {
  if (!s || !loss || s->mode != MIDAGMA_MODE_DATA) return fail(s, MIDAGMA_E_STATE, "score_finish: data mode");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    const double n = (double)s->n_global;
    if (s->loss == MIDAGMA_LOSS_L2) {
      // loss = 0.5 tr((I-W)^T cov (I-W)) with cov (I-W) = Z / n ; G = -Z / n
      double sd = 0;
      host_trace_l1(s, s->scratch.p, s->zbuf, &sd, nullptr);
      *loss = 0.5 * (sd / n);
      if (G) {
        std::vector<double> z((size_t)d * d);
        s->download_matrix(z.data(), s->zbuf);
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (size_t i = 0; i < z.size(); ++i) G[i] = -(z[i] / n);
      }
    } else {
      double tail = 0;
      HIP_TRY(hipMemcpyAsync(&tail, s->zbuf + DD, sizeof(double), hipMemcpyDeviceToHost, s->stream));
      HIP_TRY(hipStreamSynchronize(s->stream));
      *loss = 1.0 / n * tail;
      if (G) {
        std::vector<double> z((size_t)d * d), c((size_t)d * d);
        s->download_matrix(z.data(), s->zbuf);
        s->download_matrix(c.data(), s->cov.p);
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (size_t i = 0; i < z.size(); ++i) G[i] = (1.0 / n) * z[i] - c[i];
      }
    }
    return MIDAGMA_OK;
  });
}

}  // extern "C"

// ---- device-pointer log-det / inverse for torch (DagmaMLP.h_func) ------------
namespace {
struct LogdetWorkspace {
  int device = -1;
  int64_t D = 0;
  DevBuf A, P, R, C, piv;
};
std::mutex g_ws_mu;
std::vector<LogdetWorkspace*> g_ws;
}  // namespace

// the 32-padded workspace of the h log-det for this device (created on first use)
static LogdetWorkspace* logdet_h_ws(int64_t d) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  const int64_t D = (d + 31) / 32 * 32;  // the 32-block Gauss-Jordan's own granularity
  std::lock_guard<std::mutex> lock(g_ws_mu);
  for (auto* w : g_ws)
    if (w->device == dev && w->D == D) return w;
  LogdetWorkspace* ws = new LogdetWorkspace();
  ws->device = dev;
  ws->D = D;
  ws->A.alloc((size_t)D * D);
  ws->P.alloc(64 * 64);
  ws->R.alloc((size_t)64 * D);
  ws->C.alloc((size_t)D * 64);
  ws->piv.alloc(D);
  g_ws.push_back(ws);
  return ws;
}

// part 0: build + the Gauss-Jordan prologue; parts 1 .. D/32: its block steps; part D/32 + 1: the
// epilogue (h and (sI - A)^-T).  part < 0: all of them.
static void logdet_h_enqueue(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev,
                             int64_t ldm, hipStream_t st, int part) {
  setup_attributes_once();
  LogdetWorkspace* ws = logdet_h_ws(d);
  const int64_t D = ws->D;
  const int K = (int)(D / 32);
  const GJWork w{ws->P.p, ws->R.p, ws->C.p, ws->piv.p};
  if (part < 0 || part == 0) {
    launch_build_at(A, lda, false, ws->A.p, D, d, s, nullptr, nullptr, st);
    launch_gj_prologue(ws->A.p, D, D, w, nullptr, st);
  }
  for (int k = 0; k < K; ++k)
    if (part < 0 || part == k + 1) launch_gj_step(ws->A.p, D, D, w, nullptr, k, st);
  if (part < 0 || part == K + 1)
    launch_logdet_post(ws->piv.p, d, (double)d * std::log(s), h_dev, ws->A.p, D, Mt_dev, ldm, st);
}

extern "C" int midagma_logdet_h_dev(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev,
                                    int64_t ldm, void* stream) {
  if (!A || !h_dev || d < 1 || lda < d || !(s > 0.0) || (Mt_dev && ldm < d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_h_dev: bad arguments");
  return guarded(nullptr, [&] {
    logdet_h_enqueue(A, d, lda, s, h_dev, Mt_dev, ldm, reinterpret_cast<hipStream_t>(stream), -1);
    return MIDAGMA_OK;
  });
}

extern "C" int64_t midagma_logdet_h_parts(int64_t d) { return d < 1 ? 0 : (d + 31) / 32 + 2; }

// ---- the h log-det's warm-started fast path (ABI 6; mlp.hip) -------------------------------------
struct midagma_ldfast {
  int device = 0;
  int64_t d = 0, Dgj = 0;  // Gauss-Jordan workspace: 32-padded, as midagma_logdet_h_dev
  int B = 0;               // series block: 128 or 256 (0: d > 256, every step exact)
  DevBuf ring0, ring1, Y0, Y1, Q0, Q1, P, part, done, hlast;
  DevBuf A, Pgj, Rgj, Cgj, piv;
  State* st = nullptr;    // the ring's state (slots: step index; warm_run; status of the series)
  State* gjst = nullptr;  // the Gauss-Jordan gate of a fast step (ST_RUNNING: run the chain)
  int64_t* counter = nullptr;  // advanced by a fast step's end (midagma_ldfast_set_counter)
  std::string err;
  ~midagma_ldfast() {
    for (DevBuf* b : {&ring0, &ring1, &Y0, &Y1, &Q0, &Q1, &P, &part, &done, &hlast, &A, &Pgj, &Rgj, &Cgj, &piv})
      b->release();
    if (st) (void)hipFree(st);
    if (gjst) (void)hipFree(gjst);
  }
  GJWork gjw() const { return GJWork{Pgj.p, Rgj.p, Cgj.p, piv.p}; }
  SeriesWork sw() const {
    return SeriesWork{ring0.p, ring1.p, {Y0.p, Y1.p}, {Q0.p, Q1.p}, P.p, part.p, reinterpret_cast<int*>(done.p)};
  }
};

extern "C" int midagma_ldfast_create(midagma_ldfast** out, int64_t d) {
  if (!out || d < 1) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_create: bad arguments");
  auto* h = new midagma_ldfast();
  int rc = guarded(nullptr, [&] {
    setup_attributes_once();
    HIP_TRY(hipGetDevice(&h->device));
    h->d = d;
    h->Dgj = (d + 31) / 32 * 32;
    h->B = d <= 128 ? 128 : (d <= 256 ? 256 : 0);
    const size_t DD = (size_t)h->Dgj * h->Dgj;
    h->A.alloc(DD);
    h->Pgj.alloc(64 * 64);
    h->Rgj.alloc((size_t)64 * h->Dgj);
    h->Cgj.alloc((size_t)h->Dgj * 64);
    h->piv.alloc(h->Dgj);
    h->hlast.alloc(1);
    if (h->B) {
      const size_t BB = (size_t)h->B * h->B;
      for (DevBuf* b : {&h->ring0, &h->ring1, &h->Y0, &h->Y1, &h->Q0, &h->Q1, &h->P}) b->alloc(BB);
      h->part.alloc((size_t)(NM_PASSES + 1) * PART_STRIDE);
      h->done.alloc(1);
    }
    HIP_TRY(hipMalloc(&h->st, sizeof(State)));
    HIP_TRY(hipMalloc(&h->gjst, sizeof(State)));
    return midagma_ldfast_reset(h);
  });
  if (rc != MIDAGMA_OK) {
    delete h;
    return rc;
  }
  *out = h;
  return MIDAGMA_OK;
}

extern "C" void midagma_ldfast_destroy(midagma_ldfast* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  delete h;
}

extern "C" int midagma_ldfast_reset(midagma_ldfast* h) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_reset: null handle");
  return guarded(nullptr, [&] {
    HIP_TRY(hipSetDevice(h->device));
    State st{};
    st.status = ST_RUNNING;
    st.slots = -1;        // step 0: opened by ldfast_begin (exact) or counted by the fast step's end
    st.ckpt_pending = 1;  // no warm start: the first step runs the Gauss-Jordan chain
    State gj{};
    gj.status = ST_DONE;
    HIP_TRY(hipMemcpy(h->st, &st, sizeof(State), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->gjst, &gj, sizeof(State), hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(h->hlast.p, 0, sizeof(double)));
    if (h->done.p) HIP_TRY(hipMemset(h->done.p, 0, sizeof(double)));
    return MIDAGMA_OK;
  });
}

// fast: 0 the series residual (opening the step), 1 .. 3 the passes, 4 certificate + the gated
// chain with the step's end; exact: 0 begin + build + prologue, 1 .. Dgj/32 the block steps, last
// the end
static constexpr int kLdfastPasses = 3;
extern "C" int64_t midagma_ldfast_parts(const midagma_ldfast* h, int exact) {
  if (!h) return 0;
  return (exact || !h->B) ? h->Dgj / 32 + 2 : kLdfastPasses + 2;
}

extern "C" int midagma_ldfast_enqueue(midagma_ldfast* h, const double* A, int64_t d_in, int64_t lda, double s,
                                      double* h_dev, double* Mt_dev, int64_t ldm, void* stream, int exact, int64_t part) {
  if (!h || d_in != h->d)  // the handle's buffers and warm-start ring are sized for its d
    return fail(nullptr, MIDAGMA_E_ARG, "ldfast_enqueue: A's d differs from the handle's");
  if (!A || !h_dev || !Mt_dev || lda < h->d || ldm < h->d || !(s > 0.0) || part >= midagma_ldfast_parts(h, exact))
    return fail(nullptr, MIDAGMA_E_ARG, "ldfast_enqueue: bad arguments");
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t d = h->d, D = h->Dgj;
    const int K = (int)(D / 32);
    const double dls = (double)d * std::log(s);
    const bool ex = exact || !h->B;
    auto want = [&](int64_t p) { return part < 0 || part == p; };
    if (ex) {  // the Gauss-Jordan chain, ungated
      if (want(0)) {
        launch_ldfast_begin(h->st, h->gjst, st);
        launch_build_at(A, lda, false, h->A.p, D, d, s, nullptr, nullptr, st);
        launch_gj_prologue(h->A.p, D, D, h->gjw(), nullptr, st);
      }
      for (int k = 0; k < K; ++k)
        if (want(k + 1)) launch_gj_step(h->A.p, D, D, h->gjw(), nullptr, k, st);
      if (want(K + 1))
        launch_ldfast_post(h->piv.p, d, dls, h_dev, h->A.p, D, Mt_dev, ldm, h->P.p, h->B, h->ring0.p, h->ring1.p,
                           h->st, h->gjst, h->hlast.p, true, st);
      return MIDAGMA_OK;
    }
    const SeriesWork w = h->sw();
    if (want(0)) launch_ldfast_resid(A, lda, d, s, h->B, w, h->st, h->gjst, st);
    // the passes one by one (each its own part: the caller interleaves them)
    for (int p = 1; p <= kLdfastPasses; ++p)
      if (want(p)) launch_series_pass(h->B, w, h->st, p, st);
    if (want(kLdfastPasses + 1)) {
      launch_ldfast_certify(h->P.p, h->B, d, Mt_dev, ldm, h->st, reinterpret_cast<const int*>(h->done.p), h->gjst,
                            h->ring0.p, h->ring1.p, st);
      // gated: opened by the certificate.  One launch, the whole Gauss-Jordan chain in one
      // workgroup (bit-identical; slow when open, which the bench window never is): a closed gate
      // costs one launch instead of the chain's 2 + D/32, and that launch also ends the step
      // (ldfast_post's fast-step work in the same workgroup: one dependent launch fewer)
      const LdfastEnd end{h->piv.p, d, dls, h_dev, Mt_dev, ldm, h->B, h->ring0.p, h->ring1.p, h->st, h->hlast.p,
                          h->counter};
      launch_gj_inverse_1wg(A, lda, h->A.p, D, d, s, h->gjw(), h->gjst, st, end);
    }
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_ldfast_set_counter(midagma_ldfast* h, int64_t* counter) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_set_counter: null handle");
  h->counter = counter;
  return MIDAGMA_OK;
}

extern "C" int midagma_ldfast_stats(midagma_ldfast* h, int64_t* steps, int64_t* exact_steps) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_stats: null handle");
  return guarded(nullptr, [&] {
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    State st{};
    HIP_TRY(hipMemcpy(&st, h->st, sizeof(State), hipMemcpyDeviceToHost));
    if (steps) *steps = st.iter;
    if (exact_steps) *exact_steps = st.halvings;
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_logdet_h_dev_part(const double* A, int64_t d, int64_t lda, double s, double* h_dev,
                                         double* Mt_dev, int64_t ldm, void* stream, int64_t part) {
  if (!A || !h_dev || d < 1 || lda < d || !(s > 0.0) || (Mt_dev && ldm < d) || part < 0 ||
      part >= midagma_logdet_h_parts(d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_h_dev_part: bad arguments");
  return guarded(nullptr, [&] {
    logdet_h_enqueue(A, d, lda, s, h_dev, Mt_dev, ldm, reinterpret_cast<hipStream_t>(stream), (int)part);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_logdet_inv_dev(const double* A, int64_t d, int64_t lda, double s_dom, double* logdet_dev,
                                      double* Mt_dev, int64_t ldm, void* stream) {
  if (!A || d < 1 || lda < d || (Mt_dev && ldm < d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_inv_dev: bad arguments");
  return guarded(nullptr, [&] {
    setup_attributes_once();
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    const int64_t D = round_up64(d);
    std::lock_guard<std::mutex> lock(g_ws_mu);
    LogdetWorkspace* ws = nullptr;
    for (auto* w : g_ws)
      if (w->device == dev && w->D == D) ws = w;
    if (!ws) {
      ws = new LogdetWorkspace();
      ws->device = dev;
      ws->D = D;
      ws->A.alloc((size_t)D * D);
      ws->P.alloc(64 * 64);
      ws->R.alloc((size_t)64 * D);
      ws->C.alloc((size_t)D * 64);
      ws->piv.alloc(D);
      g_ws.push_back(ws);
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    launch_build_at(A, lda, false, ws->A.p, D, d, s_dom, nullptr, nullptr, st);
    launch_gj_inverse(ws->A.p, D, D, GJWork{ws->P.p, ws->R.p, ws->C.p, ws->piv.p}, nullptr, st);
    if (logdet_dev) launch_sum_vector(ws->piv.p, d, logdet_dev, nullptr, st);
    if (Mt_dev)
      HIP_TRY(hipMemcpy2DAsync(Mt_dev, ldm * sizeof(double), ws->A.p, D * sizeof(double), d * sizeof(double), d,
                               hipMemcpyDeviceToDevice, st));
    return MIDAGMA_OK;
  });
}

// ---------------------------------------------------------------------------
// Linear-SEM generator (sem.hip; utils.py:99-172)
extern "C" int midagma_sem_linear(const double* W, int64_t d, int64_t row0, int64_t n_rows, int sem_type,
                                  const double* noise_scale, uint64_t seed, double* X_dev, int64_t ldx,
                                  void* stream) {
  if (!W || d < 1 || d > (1 << 30)) return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: bad W / d");
  SemGraph g;
  if (!sem_levels(W, d, g)) return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: W must be a DAG");
  if (row0 < 0 || n_rows < 0 || ldx < d || sem_type < 0 || sem_type > 5 || (n_rows > 0 && !X_dev))
    return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: bad arguments");
  if (n_rows == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    std::vector<double> scale(d, 1.0);
    if (noise_scale) std::copy(noise_scale, noise_scale + d, scale.begin());
    // slab: rows of the node-major scratch, even, ~MIDAGMA_SEM_SLAB_MB (default 2048) MB
    int64_t budget = 2048;
    if (const char* e = getenv("MIDAGMA_SEM_SLAB_MB")) budget = std::max<int64_t>(1, atoll(e));
    const int64_t first = row0 & ~int64_t(1), end = row0 + n_rows;
    int64_t S = std::max<int64_t>(1024, (budget << 20) / (8 * d));
    S = std::min<int64_t>(S, (end - first + 1) & ~int64_t(1));
    S = (S + 1) & ~int64_t(1);
    const size_t nnz = g.pidx.size();
    struct Raw {
      void* p = nullptr;
      ~Raw() {
        if (p) (void)hipFree(p);
      }
    } ints, dbls, xt;
    const size_t n_int = g.nodes.size() + g.pptr.size() + std::max<size_t>(nnz, 1);
    HIP_TRY(hipMalloc(&ints.p, n_int * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&dbls.p, (std::max<size_t>(nnz, 1) + d) * sizeof(double)));
    HIP_TRY(hipMalloc(&xt.p, static_cast<size_t>(S) * d * sizeof(double)));
    int32_t* ip = static_cast<int32_t*>(ints.p);
    double* dp = static_cast<double*>(dbls.p);
    SemDev dev{ip, ip + g.nodes.size(), ip + g.nodes.size() + g.pptr.size(), dp, dp + std::max<size_t>(nnz, 1)};
    HIP_TRY(hipMemcpyAsync(ip, g.nodes.data(), g.nodes.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ip + g.nodes.size(), g.pptr.data(), g.pptr.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, st));
    if (nnz) {
      HIP_TRY(hipMemcpyAsync(const_cast<int32_t*>(dev.pidx), g.pidx.data(), nnz * sizeof(int32_t),
                             hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(dp, g.pw.data(), nnz * sizeof(double), hipMemcpyHostToDevice, st));
    }
    HIP_TRY(hipMemcpyAsync(const_cast<double*>(dev.scale), scale.data(), d * sizeof(double), hipMemcpyHostToDevice,
                           st));
    for (int64_t a = first; a < end; a += S) {
      const int64_t rows = std::min<int64_t>(S, end - a);
      const int64_t skip = a < row0 ? row0 - a : 0;
      launch_sem_slab(dev, g.level_off, d, sem_type, seed, a, rows, skip, static_cast<double*>(xt.p), S,
                      X_dev + (a + skip - row0) * ldx, ldx, st);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));  // the scratch is freed on return
    return MIDAGMA_OK;
  });
}

// ---------------------------------------------------------------------------
// Gated Adam step (adam.hip) for DagmaNonlinear on torch tensors
extern "C" int64_t midagma_mlp_tail_scratch(int64_t n, int64_t d, int64_t m1) {
  if (n < 1 || d < 1 || m1 < 1) return 0;
  return mlp_tail_scratch(n, d, m1);
}

extern "C" int midagma_mlp_tail_fwd(const double* Z, const double* b1, const double* w2, const double* b2,
                                    const double* X, int64_t n, int64_t d, int64_t m1, double* R, double* scratch,
                                    double* ssq, void* stream) {
  if (!Z || !w2 || !b2 || !X || !R || !scratch || !ssq || n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_fwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_fwd(Z, b1, w2, b2, X, n, d, (int)m1, R, scratch, ssq, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd(const double* Z, const double* b1, const double* w2, const double* R,
                                    const double* g, int64_t n, int64_t d, int64_t m1, double* dZ, double* dw2,
                                    double* db2, double* db1, double* scratch, void* stream) {
  if (!Z || !w2 || !R || !g || !dZ || !dw2 || !db2 || !scratch || n < 1 || d < 1 || m1 < 1 ||
      d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd(Z, b1, w2, R, g, n, d, (int)m1, dZ, dw2, db2, db1, scratch,
                        reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int64_t midagma_fc1_terms_parts(int64_t d) { return d < 1 ? 0 : fc1_terms_parts(d); }

extern "C" int midagma_fc1_terms(const double* W1, int64_t d, int64_t m1, double* A, double* l1part, void* stream) {
  if (!W1 || !A || !l1part || d < 1 || m1 < 1) return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms(W1, d, (int)m1, A, l1part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_fc1_terms_bwd(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gscale,
                                     const double* gl1part, const double* lin, int64_t nlin, double* dW1,
                                     void* stream) {
  if (!W1 || !gA || !gl1part || !dW1 || d < 1 || m1 < 1 || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms_bwd(W1, d, (int)m1, gA, gscale, gl1part, lin, (int)nlin, dW1,
                         reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective(const double* ssq, const double* l1part, int64_t np, const double* h, double mu,
                                     double lambda1, double half_d, double inv_n, double* obj, void* stream) {
  if (!ssq || !l1part || !h || !obj || np < 1) return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective(ssq, l1part, np, h, mu, lambda1, half_d, inv_n, obj, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective_bwd(const double* g, const double* ssq, int64_t np, double mu, double lambda1,
                                         double half_d, double inv_n, double* gssq, double* gl1part, double* gh,
                                         void* stream) {
  if (!g || (!ssq) != (!gssq) || !gl1part || !gh || np < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective_bwd(g, ssq, np, mu, lambda1, half_d, inv_n, gssq, gl1part, gh,
                             reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

// ABI 6: the [d, m1, 1] objective's step with the scalar objective's backward folded into its
// consumers (no mlp_sum / mlp_objective_bwd launches): the tail forward leaves its n row partials,
// the objective sums them (and advances the Adam table counter), the tail backward and the fc1
// terms' backward derive d obj / d ssq, d h and d l1 from gobj themselves.  Bit-identical to the
// ABI-5 sequence (the same sums in the same order, the same scalar arithmetic).
extern "C" int midagma_mlp_tail_fwd_part(const double* Z, const double* b1, const double* w2, const double* b2,
                                         const double* X, int64_t n, int64_t d, int64_t m1, double* R, double* part,
                                         void* stream) {
  if (!Z || !w2 || !b2 || !X || !R || !part || n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_fwd_part: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_fwd(Z, b1, w2, b2, X, n, d, (int)m1, R, part, nullptr, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd_obj(const double* Z, const double* b1, const double* w2, const double* R,
                                        const double* part, const double* gobj, double mu, double half_d,
                                        double inv_n, int64_t n, int64_t d, int64_t m1, double* dZ, double* dw2,
                                        double* db2, double* db1, double* scratch, void* stream) {
  // (ABI 9: dw2 = db2 = db1 = NULL leaves the chunk partials in scratch for midagma_mlp_step)
  const bool sums = dw2 || db2 || db1;
  if (!Z || !w2 || !R || !part || !gobj || !dZ || (sums && (!dw2 || !db2)) || !scratch || n < 1 || d < 1 ||
      m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd_obj: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd(Z, b1, w2, R, nullptr, n, d, (int)m1, dZ, dw2, db2, db1, scratch,
                        reinterpret_cast<hipStream_t>(stream), part, gobj, mu, half_d, inv_n, sums);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_step(double* const* params, double* const* exp_avg, double* const* exp_avg_sq, int64_t n,
                                int64_t d, int64_t m1, const double* gA, const double* gobj, double mu,
                                double lambda1, const double* lin, int64_t nlin, const double* scratch,
                                const double* table, const int64_t* counter, double w1, double beta2, double c2,
                                double eps, double wd, const double* gate, double* A, double* l1part, void* stream) {
  if (!params || !exp_avg || !exp_avg_sq || !gA || !gobj || !scratch || !table || !counter || !A || !l1part ||
      n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_step: bad arguments");
  for (int q = 0; q < 4; ++q)
    if (!params[q] || !exp_avg[q] || !exp_avg_sq[q]) return fail(nullptr, MIDAGMA_E_ARG, "mlp_step: bad tensor");
  const MlpStepPtrs p{params[0], params[1], params[2], params[3], exp_avg[0], exp_avg_sq[0], exp_avg[1],
                      exp_avg_sq[1], exp_avg[2], exp_avg_sq[2], exp_avg[3], exp_avg_sq[3]};
  return guarded(nullptr, [&] {
    launch_mlp_step(p, n, d, (int)m1, gA, gobj, mu, lambda1, lin, (int)nlin, scratch, table, counter, w1, beta2, c2,
                    eps, wd, gate, A, l1part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

#ifdef MIDAGMA_EXPERIMENTS
// fc1 and the tail fused on the MFMA (mlp.hip; measured slower at config 5):
// not in the public header, bound by nonlinear.py when the loaded library has them
extern "C" int64_t midagma_mlp_fused_parts(int64_t n, int64_t d, int64_t m1) { return mlp_fused_parts(n, d, m1); }

extern "C" int64_t midagma_mlp_fused_splits(int64_t n) { return n < 1 ? 0 : mlp_fused_splits(n); }

extern "C" int midagma_mlp_fc1_tail_fwd(const double* X, const double* W1, const double* b1, const double* w2,
                                        const double* b2, int64_t n, int64_t d, int64_t m1, double* S, double* R,
                                        double* part, void* stream) {
  if (!X || !W1 || !w2 || !b2 || !S || !R || !part || mlp_fused_parts(n, d, m1) < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_fc1_tail_fwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_fc1_tail_fwd(X, W1, b1, w2, b2, n, d, (int)m1, S, R, part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd_lin(const double* S, const double* w2, const double* R, const double* X,
                                        const double* part, int64_t npart, const double* gobj, double mu,
                                        double half_d, double inv_n, int64_t n, int64_t d, int64_t m1, double* lin,
                                        double* dw2, double* db2, double* db1, double* scratch, void* stream) {
  if (!S || !w2 || !R || !X || !part || npart < 1 || !gobj || !lin || !dw2 || !db2 || !scratch ||
      mlp_fused_parts(n, d, m1) < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd_lin: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd_lin(S, w2, R, X, part, npart, gobj, mu, half_d, inv_n, n, d, (int)m1, lin, dw2, db2, db1,
                            scratch, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}
#endif

extern "C" int midagma_fc1_terms_bwd_obj(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gobj,
                                         double mu, double lambda1, const double* lin, int64_t nlin, double* dW1,
                                         void* stream) {
  if (!W1 || !gA || !gobj || !dW1 || d < 1 || m1 < 1 || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms_bwd_obj: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms_bwd(W1, d, (int)m1, gA, nullptr, nullptr, lin, (int)nlin, dW1,
                         reinterpret_cast<hipStream_t>(stream), gobj, mu, lambda1);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective_part(const double* part, int64_t npart, const double* l1part, int64_t np,
                                          const double* h, double mu, double lambda1, double half_d, double inv_n,
                                          double* obj, int64_t* counter, void* stream) {
  if (!part || npart < 1 || !l1part || !h || !obj || np < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective_part: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective(nullptr, l1part, np, h, mu, lambda1, half_d, inv_n, obj,
                         reinterpret_cast<hipStream_t>(stream), part, npart, counter);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step(double* p, const double* g, double* m, double* v, int64_t n, double step_size,
                                 double w1, double beta2, double c2, double bc2_sqrt, double eps, double wd,
                                 const double* gate, void* stream) {
  if (!p || !g || !m || !v || n < 0) return fail(nullptr, MIDAGMA_E_ARG, "adam_step: bad arguments");
  if (n == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated(p, g, m, v, n, AdamCoef{step_size, w1, beta2, c2, bc2_sqrt, eps, wd}, gate,
                      reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step_table(double* p, const double* g, double* m, double* v, int64_t n,
                                       const double* table, const int64_t* counter, double w1, double beta2,
                                       double c2, double eps, double wd, const double* gate, void* stream) {
  if (!p || !g || !m || !v || !table || !counter || n < 0) return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table: bad arguments");
  if (n == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated_table(p, g, m, v, n, AdamCoef{0.0, w1, beta2, c2, 1.0, eps, wd}, table, counter, gate,
                            reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step_table_multi(int64_t k, double* const* p, const double* const* g, double* const* m,
                                             double* const* v, const int64_t* n, const double* table,
                                             const int64_t* counter, double w1, double beta2, double c2, double eps,
                                             double wd, const double* gate, void* stream) {
  if (k < 1 || k > ADAM_MULTI || !p || !g || !m || !v || !n || !table || !counter)
    return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table_multi: bad arguments");
  AdamSet set{};
  set.k = (int)k;
  set.off[0] = 0;
  for (int64_t q = 0; q < k; ++q) {
    if (!p[q] || !g[q] || !m[q] || !v[q] || n[q] < 0)
      return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table_multi: bad tensor");
    set.p[q] = p[q];
    set.g[q] = g[q];
    set.m[q] = m[q];
    set.v[q] = v[q];
    set.off[q + 1] = set.off[q] + n[q];
  }
  if (set.off[k] == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated_table_multi(set, AdamCoef{0.0, w1, beta2, c2, 1.0, eps, wd}, table, counter, gate,
                                  reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_counter_advance(int64_t* counter, void* stream) {
  if (!counter) return fail(nullptr, MIDAGMA_E_ARG, "counter_advance: null counter");
  return guarded(nullptr, [&] {
    launch_counter_advance(counter, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

#ifdef MIDAGMA_EXPERIMENTS
// Diagnostics (not part of the ABI header): the one-launch inverse's task plan for D, passes
// and nwg workgroups, as planned on the host (no GPU needed).  tasks (12 ints per task, grouped
// by workgroup) and woff (nwg + 1) may be null to query the sizes.  Returns 0, or -1.
extern "C" int midagma_debug_df_plan(int64_t D, int passes, int nwg, double* est_us, int64_t* ntasks, int* tasks,
                                     int* woff, int* nctr) {
  try {
    if (!df_available(D) || (passes != 2 && passes != 3) || nwg < 1) return -1;
    const DfPlanHost p = df_plan(D, passes, nwg);
    if (est_us) *est_us = p.est_us;
    if (ntasks) *ntasks = (int64_t)(p.tasks->size() / 12);
    if (nctr) *nctr = p.nctr;
    if (tasks) std::memcpy(tasks, p.tasks->data(), p.tasks->size() * sizeof(int));
    if (woff) std::memcpy(woff, p.woff->data(), p.woff->size() * sizeof(int));
    return 0;
  } catch (const std::exception& e) {
    fprintf(stderr, "midagma_debug_df_plan: %s\n", e.what());
    return -1;
  }
}

// Diagnostics: the one-launch inverse's per-task timestamps of the last launch (3 per task in
// plan order: wait start, go, done; 100 MHz ticks), with MIDAGMA_DF_STAMPS set at create.
// Returns the number of values copied, or -1.
extern "C" int64_t midagma_debug_df_stamps(midagma_solver* s, unsigned long long* out, int64_t cap) {
  if (!s || !s->dfw.stamps) return -1;
  const int64_t n = std::min<int64_t>(cap, (int64_t)s->dfStamps.n);
  if (hipStreamSynchronize(s->stream) != hipSuccess) return -1;
  if (hipMemcpy(out, s->dfStamps.p, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}
#endif  // MIDAGMA_EXPERIMENTS
