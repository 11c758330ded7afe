// Host-side slot scheduling of the device-resident inner loop (solver.hip drives the graphs and
// the device with it).  Pure C++: no HIP header, no device call, so it is unit-tested on the CPU
// under AddressSanitizer / UBSan against scripted device behaviour (tests/sched/sched_test.cpp,
// tests/test_sched.py).
//
// A slot is one pass of the reference's loop body (linear.py:225-331); the device controller
// decides every branch and the host only chooses WHICH captured graph to replay and how many,
// reading the State once per batch:
//  * blocked cov mode (drive_blocked): a pivoted Gauss-Jordan ("slow") slot where a log-det is
//    due (checkpoint), where no warm start exists (first slot of a call) or after a fast slot
//    handed back (ST_NEED_GJ); otherwise batches of warm-started ("fast") slots, cut at the next
//    checkpoint iteration, 1 after a hand-back doubling to 64, on the 2-pass graphs unless a
//    2-pass hand-back happened in the last 512 fast slots;
//  * the one-workgroup small-d loop (drive_small): launches of up to 4096 slots;
//  * the generic graph-replayed slot (run_loop): batches of up to 64, polled one batch late.
#pragma once

#include <stdint.h>

#include "status.h"

namespace midagma {

// The State fields the host reads after a sync.
struct SlotView {
  int32_t status = ST_RUNNING;
  int32_t ckpt_pending = 0;
  int64_t iter = 0;
  int64_t slots = 0;
};

// Slot launches one minimize call may take: every step, the objective slots of its
// checkpoints, and slack for line-search re-steps and hand-backs.
int64_t slot_cap(int64_t max_iter, int64_t checkpoint);

// One host batch of the blocked cov-mode loop.
struct BlockedPlan {
  bool done = false;            // nothing to launch: terminal status, or n_slots launched
  bool clear_handback = false;  // reset the device status ST_NEED_GJ -> ST_RUNNING first
  bool slow = false;            // one pivoted (GJ) slot first
  int64_t groups = 0;           // launches of the fast_group-slot fast graph
  int64_t singles = 0;          // launches of the one-slot fast graph
  bool two_pass = false;        // the 2-pass fast graphs (else the 3-pass ones)
};

class BlockedScheduler {
 public:
  // Persists across batches and calls of one solver (begin() resets fast_ready and
  // three_pass_left; bmax carries over).
  struct Carry {
    int64_t bmax = 64;             // fast batch cap
    int64_t three_pass_left = 0;   // fast slots still to run on the 3-pass graphs
    bool fast_ready = false;       // the last slot stored outer-block inverses (a warm start)
  };
  static constexpr int64_t kMaxBatch = 64;
  static constexpr int64_t kThreePassHold = 512;

  // n_slots < 0: until the device reports a terminal status (then a stuck controller throws
  // std::runtime_error once slot_cap is exceeded).  fast_group: slots per group graph (>= 1;
  // 1 disables groups).  have_two_pass: the 2-pass fast graphs exist.
  BlockedScheduler(int64_t max_iter, int64_t checkpoint, int64_t n_slots, int fast_group, bool have_two_pass,
                   const Carry& carry);
  // The batch to launch given the State after the last sync.
  BlockedPlan next(const SlotView& cur);
  // The State after the batch's sync.
  void observe(const SlotView& after);

  const Carry& carry() const { return c_; }
  int64_t launched() const { return launched_; }
  int64_t handbacks() const { return handbacks_; }
  int64_t batches() const { return batches_; }

 private:
  int64_t max_iter_, checkpoint_, n_slots_, cap_;
  int fast_group_;
  bool have_two_pass_;
  Carry c_;
  bool last_two_ = false;
  int64_t launched_ = 0, handbacks_ = 0, batches_ = 0;
};

// The small-d persistent loop: slots for the next launch (0: stop).  Throws when an unbounded
// run (n_slots < 0) exceeds cap without a terminal status.
int64_t small_next_batch(int64_t n_slots, int64_t launched, int64_t cap, int64_t max_batch);

// The generic graph-replayed slot: graph launches of the next batch, given the last known
// iteration (the host polls one batch late, so batches run ahead by at most one).
int64_t graph_next_batch(int64_t max_iter, int64_t known_iter);

}  // namespace midagma
