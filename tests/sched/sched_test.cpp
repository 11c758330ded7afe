// The host slot scheduler (midagma_amd/csrc/slot_sched.h) against a scripted device, on the CPU.
// Built and run by tests/test_sched.py with -fsanitize=address,undefined.
//
// The simulated device follows the controller's contract (csrc/step.hip control_kernel,
// linear.py:224-331): a slot on a terminal status is a no-op; a slot with ckpt_pending evaluates
// the objective of the current W (early stop, or the end at max_iter) before its step; a step
// that lands on a checkpoint iteration (or max_iter) sets ckpt_pending for the next slot.  Fast
// slots need a warm start (the previous slot ran) and no pending log-det, and hand back
// (ST_NEED_GJ) at scripted iterations or when the scheduler breaks that rule -- which the
// checker counts as a scheduling bug.
#include <cstdio>
#include <cstdlib>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "slot_sched.h"

using namespace midagma;

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                                              \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                              \
      std::fprintf(stderr, "\n");                                     \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

struct Script {
  int64_t max_iter = 1000, checkpoint = 100;
  std::set<int64_t> handback_at;        // a fast slot at this iteration hands back (once)
  std::set<int64_t> handback_always;    // ... every time (warm start never good enough there)
  int64_t early_stop_at = -1;           // the objective at this checkpoint iteration meets tol
  int64_t fail_at = -1;                 // the domain test fails at this iteration: ST_FAILED
  bool stuck = false;                   // the controller never advances (a device bug)
};

struct Device {
  Script sc;
  SlotView st;
  bool warm = false;  // the last slot stored the outer-block inverses
  int64_t fast_run = 0, slow_run = 0, bad_fast = 0, handbacks = 0, noops = 0;
  std::vector<int64_t> objective_at;  // iterations whose objective was evaluated

  void slot(bool slow) {
    if (st.status != ST_RUNNING) {
      ++noops;
      return;
    }
    ++st.slots;
    if (sc.stuck) return;
    if (!slow) {
      if (st.ckpt_pending || !warm) {  // the device refuses; the scheduler should never ask
        ++bad_fast;
        st.status = ST_NEED_GJ;
        return;
      }
      if (sc.handback_always.count(st.iter + 1) || sc.handback_at.erase(st.iter + 1)) {
        st.status = ST_NEED_GJ;
        ++handbacks;
        return;
      }
      ++fast_run;
    } else {
      ++slow_run;
    }
    warm = true;
    if (st.ckpt_pending) {
      objective_at.push_back(st.iter);
      st.ckpt_pending = 0;
      if (st.iter == sc.early_stop_at || st.iter == sc.max_iter) {
        st.status = ST_DONE;
        return;
      }
    }
    if (st.iter + 1 == sc.fail_at) {
      st.status = ST_FAILED;
      return;
    }
    ++st.iter;
    if (st.iter % sc.checkpoint == 0 || st.iter == sc.max_iter) st.ckpt_pending = 1;
  }
};

struct RunResult {
  Device dev;
  int64_t launched = 0, batches = 0, handbacks = 0;
  bool threw = false;
  std::vector<int64_t> batch_sizes;
  std::vector<bool> batch_two;
};

RunResult run_blocked(const Script& s, int64_t n_slots, int fast_group, bool two_pass,
                      BlockedScheduler::Carry carry = {}, Device* resume = nullptr) {
  RunResult r;
  if (resume) r.dev = *resume;
  r.dev.sc = s;
  BlockedScheduler sch(s.max_iter, s.checkpoint, n_slots, fast_group, two_pass, carry);
  int64_t guard = 0;
  try {
    for (SlotView cur = r.dev.st;;) {
      const BlockedPlan p = sch.next(cur);
      if (p.done) break;
      CHECK(p.groups >= 0 && p.singles >= 0, "negative launch counts");
      CHECK(!p.clear_handback || cur.status == ST_NEED_GJ, "clear without a hand-back");
      CHECK(cur.status != ST_NEED_GJ || (p.clear_handback && p.slow), "hand-back not re-run slow");
      CHECK(!cur.ckpt_pending || p.slow, "pending objective without a slow slot (iter %lld)", (long long)cur.iter);
      if (p.clear_handback) r.dev.st.status = ST_RUNNING;
      if (p.slow) r.dev.slot(true);
      const int64_t B = p.groups * fast_group + p.singles;
      if (fast_group <= 1) CHECK(p.groups == 0, "groups with fast_group 1");
      CHECK(p.singles < fast_group || fast_group <= 1, "singles %lld >= group %d", (long long)p.singles, fast_group);
      for (int64_t b = 0; b < B; ++b) r.dev.slot(false);
      r.batch_sizes.push_back(B);
      r.batch_two.push_back(p.two_pass);
      cur = r.dev.st;
      sch.observe(cur);
      if (++guard > 10000000) {
        CHECK(false, "scheduler does not terminate");
        break;
      }
    }
  } catch (const std::runtime_error&) {
    r.threw = true;
  }
  r.launched = sch.launched();
  r.batches = sch.batches();
  r.handbacks = sch.handbacks();
  return r;
}

// 1. A plain run: every step taken, every checkpoint objective evaluated on a slow slot, no
//    fast slot refused, batches capped at 64 and cut at checkpoints.
void test_plain(int fast_group, bool two) {
  Script s;
  s.max_iter = 1000;
  s.checkpoint = 100;
  RunResult r = run_blocked(s, -1, fast_group, two);
  CHECK(!r.threw, "threw");
  CHECK(r.dev.st.status == ST_DONE && r.dev.st.iter == 1000, "status %d iter %lld", r.dev.st.status,
        (long long)r.dev.st.iter);
  CHECK(r.dev.bad_fast == 0, "%lld fast slots refused", (long long)r.dev.bad_fast);
  CHECK(r.dev.objective_at.size() == 10, "objectives %zu", r.dev.objective_at.size());
  for (size_t i = 0; i < r.dev.objective_at.size(); ++i)
    CHECK(r.dev.objective_at[i] == 100 * (int64_t)(i + 1), "objective at %lld", (long long)r.dev.objective_at[i]);
  // slow slots: the first slot, and the 10 objective slots (the last one ends the call)
  CHECK(r.dev.slow_run == 11, "slow %lld", (long long)r.dev.slow_run);
  CHECK(r.dev.fast_run == 1000 - 10, "fast %lld", (long long)r.dev.fast_run);
  CHECK(r.launched == r.dev.st.slots + r.dev.noops, "launched %lld slots %lld noops %lld", (long long)r.launched,
        (long long)r.dev.st.slots, (long long)r.dev.noops);
  for (int64_t b : r.batch_sizes) CHECK(b <= BlockedScheduler::kMaxBatch, "batch %lld", (long long)b);
  for (bool t : r.batch_two) CHECK(t == two, "pass count");
  // 99 fast slots per checkpoint interval at most 64 per batch: 2 batches each
  CHECK(r.batches <= 2 * 10 + 1, "batches %lld", (long long)r.batches);
}

// 2. Hand-backs: the slot is re-run slow, the batch cap falls to 1 and doubles back; a 2-pass
//    hand-back switches to the 3-pass graphs for 512 fast slots.
void test_handbacks() {
  Script s;
  s.max_iter = 3000;
  s.checkpoint = 1000;
  s.handback_at = {150, 151, 900, 2500};
  RunResult r = run_blocked(s, -1, 4, true);
  CHECK(!r.threw, "threw");
  CHECK(r.dev.st.status == ST_DONE && r.dev.st.iter == 3000, "end");
  CHECK(r.dev.handbacks == 4 && r.handbacks == 4, "handbacks dev %lld sched %lld", (long long)r.dev.handbacks,
        (long long)r.handbacks);
  CHECK(r.dev.bad_fast == 0, "refused %lld", (long long)r.dev.bad_fast);
  // after the hand-back at 150: a batch of 1 (plus its slow slot), then 2, 4, ...
  bool seen_one = false, doubled = false;
  for (size_t i = 0; i + 1 < r.batch_sizes.size(); ++i) {
    if (r.batch_sizes[i] == 1) seen_one = true;
    if (r.batch_sizes[i] == 1 && r.batch_sizes[i + 1] == 2) doubled = true;
  }
  CHECK(seen_one && doubled, "cap 1 then doubling");
  int64_t three = 0;
  for (size_t i = 0; i < r.batch_sizes.size(); ++i)
    if (!r.batch_two[i]) three += r.batch_sizes[i];
  CHECK(three >= BlockedScheduler::kThreePassHold, "3-pass slots %lld", (long long)three);
  CHECK(r.dev.st.slots <= slot_cap(s.max_iter, s.checkpoint), "slots %lld", (long long)r.dev.st.slots);
}

// 3. A warm start that never converges at one iteration: every try hands back, the slow slot
//    takes that step, the run still ends.
void test_persistent_handback() {
  Script s;
  s.max_iter = 500;
  s.checkpoint = 100;
  s.handback_always = {37, 38, 39, 250};
  RunResult r = run_blocked(s, -1, 4, true);
  CHECK(!r.threw && r.dev.st.status == ST_DONE && r.dev.st.iter == 500, "end");
  CHECK(r.dev.bad_fast == 0, "refused");
}

// 4. Early stop at a checkpoint and a domain failure: the run ends there; later launches of
//    the batch are device no-ops.
void test_early_stop_and_failure() {
  Script s;
  s.max_iter = 5000;
  s.checkpoint = 1000;
  s.early_stop_at = 3000;
  RunResult r = run_blocked(s, -1, 4, true);
  CHECK(r.dev.st.status == ST_DONE && r.dev.st.iter == 3000, "early stop iter %lld", (long long)r.dev.st.iter);
  Script f;
  f.max_iter = 5000;
  f.checkpoint = 1000;
  f.fail_at = 1234;
  RunResult q = run_blocked(f, -1, 4, true);
  CHECK(q.dev.st.status == ST_FAILED && q.dev.st.iter == 1233, "failure iter %lld", (long long)q.dev.st.iter);
  CHECK(!q.threw, "threw");
}

// 5. n_slots >= 0 (run_slots): exactly n launches, across calls that resume the same device and
//    carry the scheduler state; the slow slot after a boundary is taken only when due.
void test_bounded_chunks() {
  Script s;
  s.max_iter = 2000;
  s.checkpoint = 700;
  Device dev;
  dev.sc = s;
  BlockedScheduler::Carry carry;
  int64_t total = 0;
  for (int64_t n : {1, 5, 63, 64, 65, 200, 7, 1000}) {
    BlockedScheduler sch(s.max_iter, s.checkpoint, n, 4, true, carry);
    int64_t before = dev.st.slots + dev.noops;
    for (SlotView cur = dev.st;;) {
      const BlockedPlan p = sch.next(cur);
      if (p.done) break;
      if (p.clear_handback) dev.st.status = ST_RUNNING;
      if (p.slow) dev.slot(true);
      for (int64_t b = 0; b < p.groups * 4 + p.singles; ++b) dev.slot(false);
      cur = dev.st;
      sch.observe(cur);
    }
    CHECK(sch.launched() == n || dev.st.status != ST_RUNNING, "chunk %lld launched %lld", (long long)n,
          (long long)sch.launched());
    CHECK(dev.st.slots + dev.noops - before == sch.launched(), "device saw %lld", (long long)(dev.st.slots + dev.noops - before));
    carry = sch.carry();
    total += sch.launched();
  }
  CHECK(dev.bad_fast == 0, "refused %lld", (long long)dev.bad_fast);
  // every slot steps (an objective slot evaluates, then steps) until the run ends
  CHECK(dev.st.iter == total, "iter %lld total %lld", (long long)dev.st.iter, (long long)total);
  CHECK(dev.objective_at.size() == 2, "objectives %zu", dev.objective_at.size());
}

// 6. A stuck controller: an unbounded run throws once the slot budget is exceeded.
void test_stuck() {
  Script s;
  s.max_iter = 300;
  s.checkpoint = 100;
  s.stuck = true;
  RunResult r = run_blocked(s, -1, 4, true);
  CHECK(r.threw, "no throw");
  CHECK(r.launched <= 4 * slot_cap(300, 100) + BlockedScheduler::kMaxBatch + 1, "launched %lld",
        (long long)r.launched);
}

// 7. The small-d and generic graph batches.
void test_small_and_graph() {
  const int64_t cap = slot_cap(10000, 1000);
  CHECK(small_next_batch(-1, 0, cap, 4096) == 4096, "first");
  CHECK(small_next_batch(-1, cap - 5, cap, 4096) == 5, "tail");
  bool threw = false;
  try {
    small_next_batch(-1, cap, cap, 4096);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw, "small cap");
  CHECK(small_next_batch(100, 100, cap, 4096) == 0 && small_next_batch(100, 40, cap, 4096) == 60, "bounded");
  CHECK(graph_next_batch(1000, 0) == 64 && graph_next_batch(1000, 990) == 12 && graph_next_batch(1000, 1000) == 2,
        "graph batches");
}

}  // namespace

int main() {
  for (int g : {1, 4, 7})
    for (bool two : {true, false}) test_plain(g, two);
  test_handbacks();
  test_persistent_handback();
  test_early_stop_and_failure();
  test_bounded_chunks();
  test_stuck();
  test_small_and_graph();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
#if defined(__SANITIZE_ADDRESS__)
  std::printf("sched_test: AddressSanitizer on\n");
#endif
  std::printf("sched_test: all checks passed\n");
  return 0;
}
