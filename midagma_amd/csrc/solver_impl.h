// The data-mode / cov-mode solver object behind the C ABI (include/midagma_hip.h): its device
// buffers, the captured slot graphs and the host drivers that replay them.  Shared by solver.hip
// (the C ABI of one solver) and group.hip (ABI 11: a single-process group of data-mode solvers
// over several devices).
//
// One "slot" = one pass of the reference's loop body (linear.py:225-331):
//   part 1  build (sI - W∘W)^T -> blocked GJ inverse (+ log|pivots|) -> score GEMM(s)
//   part 2  domain check / checkpoint partials -> control (1 WG) -> fused update
// The control decision lives in device memory, so slots are replayed from a
// hipGraph in batches with no host round trip per step; the host only polls
// the state every batch.  Slots after termination are
// no-ops (every kernel early-exits on the status word).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/midagma_hip.h"
#include "launch.h"
#include "slot_sched.h"

namespace midagma {

struct DevBuf {
  double* p = nullptr;
  size_t n = 0;
  double* base = nullptr;  // the allocation (p = base + an offset, alloc_shifted)
  void alloc(size_t count) {
    if (count <= n && p && p == base) return;
    release();
    HIP_TRY(hipMalloc(&base, std::max<size_t>(count, 1) * sizeof(double)));
    p = base;
    n = count;
  }
  // count entries starting `off` entries into a fresh allocation (placement experiments)
  void alloc_shifted(size_t count, size_t off) {
    if (off == 0) return alloc(count);
    release();
    HIP_TRY(hipMalloc(&base, (count + off) * sizeof(double)));
    p = base + off;
    n = count;
  }
  void release() {
    if (base) (void)hipFree(base);
    base = p = nullptr;
    n = 0;
  }
};

// group.hip: the slot graphs of an emulated group (every member on one device, the score sum a
// fixed-order device sum) are captured over all members' streams at once, and a hand-back clears
// every member's status word
hipGraphExec_t group_capture(midagma_group* g, const midagma_solver* caller, int which, int reps, int passes);
void group_clear_handback(midagma_group* g);

}  // namespace midagma

using namespace midagma;

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
  DevBuf l1w;    // float32 W: [0] numpy's float32 L1 sum, then its chunk sums (np_l1_kernel)
  // cov mode, l2, d <= 64, no trek regularizer: the one-workgroup persistent loop (small.hip)
  DevBuf scarry, sprev;  // between two small-loop launches: pending norms + warm count, last inverses
  bool use_small = !knob_set("MIDAGMA_EXP_NO_SMALL");
  bool small_tcc = knob("MIDAGMA_EXP_SMALL_TCC", 1) != 0;  // experiments: 0 keeps TCC on the graph slots
  // (the TCC regularizer runs inside it up to d = 32, tcc_blk.h; PST keeps the graph-replayed slots)
  bool small_on() const {
    // (float32 W: DS <= 32, whose LDS has room for the float32 |W| image of numpy's L1 sum)
    return use_small && mode == MIDAGMA_MODE_COV && loss == MIDAGMA_LOSS_L2 && small_block(d) > 0 &&
           (!w32 || small_block(d) <= 32) && (!trek_on || (trek_tcc && small_block(d) <= 32 && small_tcc && !w32));
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
  DevBuf cA, cMi, cS, cvec, cpart, cP, cR, cC, cAalt, cPst, cPst1;
  DevBuf cY0, cY1, cQ0, cQ1, cPb, cPart2, cDone;  // the TCC fast-block inverse's series buffers
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
  DevBuf prepad;  // (experiments: MIDAGMA_EXP_PREPAD_MB)
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
  // ABI 11: member of a single-process device group (group.hip).  group: set in an emulated group
  // (its slot graphs are the group's, captured over every member's stream); group_stop: set while a
  // threaded group's minimize runs, raised when another member failed (checked at every poll)
  midagma_group* group = nullptr;
  const std::atomic<bool>* group_stop = nullptr;
  void check_group_stop() const {
    if (group_stop && group_stop->load()) throw std::runtime_error("device group: another member failed");
  }

  ~midagma_solver() {
    destroy_graphs();
    if (stream) (void)hipStreamSynchronize(stream);
    comm_destroy(comm);
    agree.release();
    if (h_agree) (void)hipHostFree(h_agree);
    for (DevBuf* b : {&W, &m, &v, &Mt, &cov, &covs, &covsT, &minc, &mexc, &P, &R, &C, &pivlog, &partials, &bc_table,
                      &zown, &scratch, &Gtmp, &X, &Y, &Zparts, &loss_part, &cov_parts, &Pstore, &Malt, &Pst2, &Pst2b,
                      &nmY0, &nmY1, &nmQ0, &nmQ1, &nmP, &nmPart, &nmDone, &nmLW, &nmLZ, &nmLPZ, &nmSync, &npart, &XT, &IW, &scarry,
                      &sprev, &cupart_ctr, &l1w, &ctl_ticket, &A0, &prepad})
      b->release();
#ifdef MIDAGMA_EXPERIMENTS
    for (DevBuf* b : {&dfA, &dfY, &dfQ, &dfP, &dfCtl, &dfTasks[0], &dfTasks[1], &dfWoff[0], &dfWoff[1], &dfStamps})
      b->release();
#endif
    for (DevBuf& b : tbufs) b.release();
    for (DevBuf* b : {&tpairs, &tsmall, &Gtrek, &tslices, &cA, &cMi, &cS, &cvec, &cpart, &cP, &cR, &cC, &cAalt, &cPst,
                      &cPst1, &cY0, &cY1, &cQ0, &cQ1, &cPb, &cPart2, &cDone})
      b->release();
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
    if (cap) (void)hipStreamDestroy(cap);
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
    bool gemm_done = false, trek_done = false;
    ctl_folded = false;
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
      // TCC ('opt', 2d > 128) on a fast cov slot: first, with a short Noda chain that hands the slot
      // back when it does not converge in time (the inverse, GEMM and control of the slot are then
      // no-ops and the host re-runs it with the whole chain); it reads W only, so its place in the
      // slot does not change any result
      if (fast && tcc_fast_steps > 0 && trek_on && trek_tcc && tcfg.mode == 2 && 2 * d > 128 &&
          mode == MIDAGMA_MODE_COV) {
        launch_trek_tcc(W.p, d, D, ccfg, cw, d_state, Gtrek.p, stream, d_state, tcc_fast_steps);
        trek_done = true;
      }
      // cov fast slot: the score GEMM rides in the last trailing update's launch (its split-K
      // slices are what fused_update sums anyway); MIDAGMA_EXP_FUSE_GEMM=0 keeps it apart
      GemmSpec gs{};
      const bool fuse = fast && mode == MIDAGMA_MODE_COV && cov_split > 1 && fuse_gemm;
      if (fuse) gs = score_cov_spec();
      gemm_done = enqueue_build_inverse(fast, passes, fuse ? &gs : nullptr);
      ctl_folded = fuse && gemm_done && gs.ctl_ticket != nullptr;
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
    if (trek_on && !trek_done && (tcfg.mode == 2 || !(fast && blocked()))) {
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
    double* ain0 = fast && at_fold_on() ? A0.p : nullptr;  // (built by the previous slot's update)
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
    if (!ain0)
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
      return launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, stream, passes, fuse, &tla, false, ain0);
    }
    return launch_blocked_inverse(Mt.p, D, binv(), fast, gj(), d_state, stream, passes, fuse, nullptr, resid0, ain0);
  }
#ifdef MIDAGMA_EXPERIMENTS
  // experiment knob MIDAGMA_EXP_BUILD_RESID0=1: build_at and block 0's residual in one launch
  static bool build_resid0_on() {
    static const bool on = knob("MIDAGMA_EXP_BUILD_RESID0", 0) != 0;
    return on;
  }
#endif
  bool fuse_gemm = knob("MIDAGMA_EXP_FUSE_GEMM", 1) != 0;
  // build_at folded into the previous slot's update (MIDAGMA_EXP_AT_FOLD): fast slots read outer
  // step 0's A^T from A0, which fused_update_at (fast slots) or a build_at after the update (slow
  // slots) wrote from the slot's new W; every call starts with a slow slot, so A0 is never stale
  // Measured (profiles/r06_probe_atfold.log): D = 1024 +1.7 %, 1408 +0.6 %, 512 -4 % (128 update
  // workgroups of 8 rows x 256 columns), 2048 -1.2 %; on for 1024 <= D <= 1408 (-1: that rule)
  long at_fold_knob = knob("MIDAGMA_EXP_AT_FOLD", -1);
  bool at_fold = at_fold_knob > 0;
  DevBuf A0;
  bool at_fold_on() const {
    if (!at_fold || !A0.p || cov_fork_on()) return false;
#ifdef MIDAGMA_EXPERIMENTS
    if (df_on || build_resid0_on()) return false;
#endif
    return true;
  }
  // the fast cov slot's control decided by the last workgroup of the trailing launch that carries
  // the score GEMM (control.h; MIDAGMA_EXP_CTL_FOLD=0 launches control_kernel instead)
  bool ctl_fold = knob("MIDAGMA_EXP_CTL_FOLD", 1) != 0;
  bool ctl_folded = false;  // set by enqueue_part1 for the enqueue_part2 of the same slot
  // TCC on fast cov slots (2d > 128), without the fixed-shift stage (tcc_fix = 0): Noda steps
  // enqueued before the slot hands back (the full TCC_NODA_MAX on pivoted slots); with the stage the
  // fast chain is the stage alone (tcc.hip launch_trek_tcc).  MIDAGMA_EXP_TCC_FAST_STEPS=0: every
  // slot runs the whole gated chain
  int tcc_fast_steps = (int)knob("MIDAGMA_EXP_TCC_FAST_STEPS", 5);
  // TCC (2d > 128): the fixed-shift stage before Noda (tcc.hip; MIDAGMA_EXP_TCC_FIX=0 off)
  int tcc_fix = (int)knob("MIDAGMA_EXP_TCC_FIX", 1);
  int tcc_fix_pre = (int)knob("MIDAGMA_EXP_TCC_FIX_PRE", 1);  // ... after this many Noda steps on fast slots
  // ... for this many slots after a stage that did not settle (with the Noda step only after such a
  // stage, holding it 8 slots instead of 1 takes d = 1000 from W = 0 from 9.8 to 8.0 ms a step and
  // d = 300 from 1.30 to 0.98, and costs nothing later: profiles/r06_probe_tccfix9_easyall.log)
  int tcc_fix_hold = (int)knob("MIDAGMA_EXP_TCC_FIX_HOLD", 8);
  // ... and (D2 >= 2048) its inverse on fast slots with every outer block but the last on the
  // product-form series (tcc.hip tcc_inverse_fix; read by set_trek_tcc).  Measured at d = 1000
  // (profiles/r06_probe_tccfastblk.log): 1.83 -> 1.40 ms a step after 1300 steps; from W = 0, where
  // the warm starts are poor, 8.0 -> 10.4 ms over the first 30-odd steps
  bool tcc_fastblk = knob("MIDAGMA_EXP_TCC_FASTBLK", 1) != 0;
  DevBuf ctl_ticket;

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
    if (ctl_fold && ctl_ticket.p) {
      gs.ctl_pr = d_params;
      gs.ctl_table = bc_table.p;
      gs.ctl_ticket = reinterpret_cast<int*>(ctl_ticket.p);
    }
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
      // (experiments build, MIDAGMA_EXP_XW_FULLK=1: the k loop over all of D, as round 4 ran it)
      static const int64_t kfull = knob("MIDAGMA_EXP_XW_FULLK", 0);
      launch_gemm(n_pad, D, kfull ? D : Kd(), xw_a(), xw_lda(), use_xt, iw ? iw : Wp, D, iw ? B_PLAIN : B_IMINUS, Y.p, D,
                  EPI_STORE, 1,
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
    // float32 W: numpy's float32 L1 sum for the checkpoint objective (np_sum.h; checkpoint slots
    // are never lean)
    const bool l1f = w32 && l1w.p && !lean;
    if (l1f) launch_np_l1(W.p, d, D, d_state, reinterpret_cast<float*>(l1w.p + 1), l1w.p, stream);
    if (!(lean && ctl_folded))  // (else decided at the end of the slot's last trailing launch)
      launch_control(d_params, d_state, partials.p, pivlog.p, zbuf + D * D, bc_table.p, d_ckpt, ckpt_cap, npart.p, d,
                     trek_on ? (trek_tcc ? cw.scal : tw.scal) : nullptr, stream, l1f ? l1w.p : nullptr);
    const bool slices = lean && mode == MIDAGMA_MODE_COV && cov_split > 1;
    const double* trek = trek_on && tcfg.mode == 2 ? Gtrek.p : nullptr;
    if (lean && at_fold_on()) {  // the next slot's build_at in the update
      launch_fused_update_at(d_params, d_state, W.p, m.p, v.p, Mt.p, slices ? cov_parts.p : zbuf, slices ? cov_split : 1,
                             D * D, cov.p, has_inc ? minc.p : nullptr, has_exc ? mexc.p : nullptr, trek, d, D, A0.p,
                             IW.p, npart.p, stream);
      return;
    }
    launch_fused_update(d_params, d_state, W.p, m.p, v.p, Mt.p, slices ? cov_parts.p : zbuf,
                        slices ? cov_split : 1, D * D, cov.p, has_inc ? minc.p : nullptr, has_exc ? mexc.p : nullptr,
                        trek, d, D, npart.p, stream);
    if (blocked() && at_fold_on())  // slow slot: the next (fast) slot's A^T and I - W from the new W
      launch_build_at(W.p, D, /*square=*/true, A0.p, D, d, 0.0, d_params, d_state, stream, IW.p);
  }

  // Slot graphs are captured on a stream of the solver's own and launched on `stream`: a caller
  // (torch's process group, DagmaLinear's host-driven all-reduce) may record events on `stream`, and
  // HIP refuses any query of an event recorded on a stream that is capturing (torch's NCCL
  // watchdog aborted the process on such a query while a capture ran).
  hipStream_t cap = nullptr;
  hipStream_t capture_stream() {
    if (!cap) HIP_TRY(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
    return cap;
  }
  struct StreamSwap {  // `stream` set to another stream for a scope (the captures)
    midagma_solver* s;
    hipStream_t saved;
    StreamSwap(midagma_solver* s_, hipStream_t to) : s(s_), saved(s_->stream) { s->stream = to; }
    ~StreamSwap() { s->stream = saved; }
  };

  hipGraphExec_t capture(int which, int reps = 1, int passes = NM_PASSES_RUN) {
    if (group) return group_capture(group, this, which, reps, passes);
    hipGraph_t graph = nullptr;
    StreamSwap on_cap(this, capture_stream());
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
    cvec.alloc((size_t)6 * D2 + 32);
    cpart.alloc((size_t)nch * D2);
    cP.alloc(2 * 32 * 32);
    cR.alloc((size_t)2 * 32 * D2);
    cC.alloc((size_t)2 * D2 * 32);
    HIP_TRY(hipMemcpy(cS.p, S.data(), S.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(cvec.p, 0, cvec.n * sizeof(double)));  // warm flag off, vectors 0
    if (!cgates) HIP_TRY(hipMalloc(&cgates, TCC_GATES * sizeof(State)));
    HIP_TRY(hipMemset(cgates, 0, TCC_GATES * sizeof(State)));
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
    w.fix = tcc_fix != 0 ? 1 : 0;
    w.fix_pre = tcc_fix_pre;
    w.fix_hold = tcc_fix_hold;
    w.fix_easy = (int)knob("MIDAGMA_EXP_TCC_FIX_EASY", 0);
    // D2 >= 2048: the shifted inverses on the two-level blocked inverse (pivoted path; measured,
    // profiles/r06_probe_tccbinv2.log: d = 1000 (D2 = 2048) 6.01 -> 5.36 ms a step, but d = 500
    // (D2 = 1024) 2.04 -> 2.41 and d = 300 (D2 = 640) 1.07 -> 1.34 ms; MIDAGMA_EXP_TCC_BINV=0: always
    // the flat Gauss-Jordan, 2: from D2 >= 512)
    const long tbinv = knob("MIDAGMA_EXP_TCC_BINV", 1);
    if (D2 >= (tbinv == 2 ? 512 : 2048) && binv_block(D2) > 0 && tbinv != 0) {
      const int64_t b2 = binv_block(D2);
      cAalt.alloc((size_t)D2 * D2);
      cPst.alloc((size_t)D2 * b2);
      cPst1.alloc((size_t)D2 * b2);
      w.Aalt = cAalt.p;
      w.Pst = cPst.p;
      w.Pst1 = cPst1.p;
      // fast slots: every outer block but the last on the product-form series (tcc.hip
      // tcc_inverse_fix; MIDAGMA_EXP_TCC_FASTBLK=0 off); one warm-start slot (Pst1 = Pst)
      if (tcc_fastblk) {
        for (DevBuf* b : {&cY0, &cY1, &cQ0, &cQ1, &cPb}) b->alloc((size_t)b2 * b2);
        cPart2.alloc((size_t)(D2 / b2) * (NM_PASSES + 1) * PART_STRIDE);
        cDone.alloc((size_t)(D2 / b2));
        HIP_TRY(hipMemset(cPst.p, 0, (size_t)D2 * b2 * sizeof(double)));
        w.Pst1 = cPst.p;
        w.Y0 = cY0.p;
        w.Y1 = cY1.p;
        w.Q0 = cQ0.p;
        w.Q1 = cQ1.p;
        w.Pblk = cPb.p;
        w.part2 = cPart2.p;
        w.done = reinterpret_cast<int*>(cDone.p);
      }
    }
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
    if (mode == MIDAGMA_MODE_COV && B2 > 0) {  // the folded control's workgroup ticket (control.h)
      ctl_ticket.alloc(1);
      HIP_TRY(hipMemsetAsync(ctl_ticket.p, 0, sizeof(double), stream));
    }
    // cov mode: build_at also writes I - W for the score GEMM's plain-B form
    if (mode == MIDAGMA_MODE_COV && ((D % 128 == 0 && cov_iw) || w32)) IW.alloc(DD);
    // the next slot's A^T written by fused_update_at (at_fold_on)
    if (at_fold_knob < 0) at_fold = D >= 1024 && D <= 1408;
    if (at_fold && mode == MIDAGMA_MODE_COV && B2 > 0) A0.alloc(DD);
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
        if (group)
          group_clear_handback(group);
        else
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
      check_group_stop();
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
        tc = SmallTcc{cw.S, ccfg.w, ccfg.eps, (double)ccfg.m, ccfg.weight, ccfg.mode, cw.scal, cw.vprev, cw.uprev,
                      cw.fix};
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
        check_group_stop();
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
