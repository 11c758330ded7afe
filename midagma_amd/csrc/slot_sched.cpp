// Host-side slot scheduling (slot_sched.h).  Compiled as plain C++ into the library and, under
// -fsanitize=address,undefined, into tests/sched/sched_test.cpp.
#include "slot_sched.h"

#include <algorithm>
#include <stdexcept>

namespace midagma {

int64_t slot_cap(int64_t max_iter, int64_t checkpoint) {
  return max_iter + max_iter / std::max<int64_t>(checkpoint, 1) + 512;
}

BlockedScheduler::BlockedScheduler(int64_t max_iter, int64_t checkpoint, int64_t n_slots, int fast_group,
                                   bool have_two_pass, const Carry& carry)
    : max_iter_(max_iter),
      checkpoint_(std::max<int64_t>(checkpoint, 1)),
      n_slots_(n_slots),
      cap_(slot_cap(max_iter, checkpoint)),
      fast_group_(std::max(1, fast_group)),
      have_two_pass_(have_two_pass),
      c_(carry) {
  c_.bmax = std::min<int64_t>(kMaxBatch, std::max<int64_t>(1, c_.bmax));
}

BlockedPlan BlockedScheduler::next(const SlotView& cur) {
  BlockedPlan p;
  if (cur.status != ST_RUNNING && cur.status != ST_NEED_GJ) {
    p.done = true;
    return p;
  }
  if (n_slots_ >= 0 && launched_ >= n_slots_) {
    p.done = true;
    return p;
  }
  if (n_slots_ < 0 && (cur.slots > cap_ || launched_ > 4 * cap_))
    throw std::runtime_error("minimize: slot budget exceeded (controller stuck)");
  int64_t it_hi = cur.iter;  // the iteration after the slots planned so far
  if (cur.status == ST_NEED_GJ || cur.ckpt_pending || !c_.fast_ready) {
    if (cur.status == ST_NEED_GJ) {
      ++handbacks_;
      c_.bmax = 1;
      p.clear_handback = true;
    }
    p.slow = true;  // pivots for the log-det, and fresh warm starts
    ++launched_;
    ++it_hi;
    c_.fast_ready = true;
  }
  // fast slots up to the next checkpoint iteration (the slot after it must be slow)
  const int64_t next_ck = std::min(max_iter_, (it_hi / checkpoint_ + 1) * checkpoint_);
  int64_t B = std::max<int64_t>(0, std::min<int64_t>(c_.bmax, next_ck - it_hi));
  if (n_slots_ >= 0) B = std::max<int64_t>(0, std::min<int64_t>(B, n_slots_ - launched_));
  p.two_pass = have_two_pass_ && c_.three_pass_left <= 0;
  p.groups = fast_group_ > 1 ? B / fast_group_ : 0;
  p.singles = B - p.groups * fast_group_;
  if (!p.two_pass) c_.three_pass_left -= B;
  launched_ += B;
  last_two_ = p.two_pass;
  ++batches_;
  return p;
}

void BlockedScheduler::observe(const SlotView& after) {
  if (after.status != ST_NEED_GJ)
    c_.bmax = std::min<int64_t>(kMaxBatch, 2 * c_.bmax);
  else if (last_two_)
    c_.three_pass_left = kThreePassHold;  // residuals this far need 3 passes: stay there a while
}

int64_t small_next_batch(int64_t n_slots, int64_t launched, int64_t cap, int64_t max_batch) {
  const int64_t B = std::min<int64_t>(max_batch, (n_slots < 0 ? cap : n_slots) - launched);
  if (B <= 0) {
    if (n_slots < 0) throw std::runtime_error("minimize: slot budget exceeded (controller stuck)");
    return 0;
  }
  return B;
}

int64_t graph_next_batch(int64_t max_iter, int64_t known_iter) {
  return std::min<int64_t>(64, std::max<int64_t>(2, max_iter - known_iter + 2));
}

}  // namespace midagma
