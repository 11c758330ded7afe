// The controller's per-slot decisions (linear.py:230-241 and the step bookkeeping), one thread,
// shared by step.hip's control_kernel and the fast cov slot's last trailing-update launch
// (gemm.hip gemm_trail_kernel: the workgroup that finishes that launch last decides, so the fast
// slot needs no control launch of its own).
#pragma once

#include "common.h"

namespace midagma {

// the slot's bookkeeping before any decision
__device__ inline void control_open(State* st) {
  if (st->slots == 0) st->t0 = __builtin_amdgcn_s_memrealtime();
  st->slots += 1;
  st->warm_valid = 1;  // this slot's GJ pass stored every diagonal-block inverse
  st->warm_run = st->warm_run < 2 ? st->warm_run + 1 : 2;
}

// after the (checkpoint) objective: the domain line search or the next Adam step
__device__ inline void control_decide(const Params* pr, State* st, int flags, const double* bc_table) {
  if (flags & 2) {
    st->status = ST_SINGULAR;
    st->action = ACT_NOOP;
    return;
  }
  if (flags & 1) {  // sI - W∘W is not an M-matrix (linear.py:230-241)
    if (st->iter == 0 || pr->s <= 0.9) {
      st->status = ST_FAILED;
      st->action = ACT_NOOP;
      return;
    }
    st->warm_run = 1;  // W turns back: the last two inverses do not extrapolate the path
    const double lr_old = st->lr;
    st->lr = lr_old * .5;
    st->halvings += 1;
    st->lr_a = lr_old;
    st->lr_b = st->lr;
    if (st->lr <= 1e-16) {
      st->status = ST_LR_UNDERFLOW;
      st->action = ACT_REVERT;
      return;
    }
    st->action = ACT_HALVE;
    return;
  }
  const int64_t it = st->iter + 1;
  st->bc1 = bc_table[2 * (it - 1)];
  st->bc2 = bc_table[2 * (it - 1) + 1];
  st->lr_a = st->lr;
  st->action = ACT_STEP;
  st->iter = it;
  if (it % pr->checkpoint == 0 || it == pr->max_iter) st->ckpt_pending = 1;
}

// The control of a fast (non-checkpoint) slot folded into a multi-workgroup launch: every
// workgroup calls it once at its end; the one that finishes last takes the domain flags the
// launch's workgroups ORed into st->flags and decides.  *ticket counts the launch's workgroups
// (reset by the last).  A pending checkpoint never reaches a fast slot (the host runs those on
// the pivoted path); if one did, the slot hands back (ST_NEED_GJ) instead of deciding.
// No release fence: an agent-scope fence writes the XCD's L2 back (measured: 229 -> 246 us a slot
// at d = 1000 with one per workgroup).  The only data the decision reads from this launch are the
// domain flags, which arrive by device-scope atomics like the ticket itself; __syncthreads and the
// wait below retire this workgroup's atomicOr before its ticket.
__device__ inline void control_fold_tail(const Params* pr, State* st, const double* bc_table, int* ticket) {
  __syncthreads();
  if (threadIdx.x != 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (int)gridDim.x - 1) return;
  __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int flags = __hip_atomic_exchange(&st->flags, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (st->ckpt_pending) {
    st->status = ST_NEED_GJ;
    st->action = ACT_NOOP;
    return;
  }
  control_open(st);
  control_decide(pr, st, flags, bc_table);
}

}  // namespace midagma
