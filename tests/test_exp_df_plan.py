"""The one-launch blocked inverse's host plan (experiments/dfinv.hip), checked on the CPU: every
counter a task waits for gets exactly its target number of signals, and the per-workgroup
task lists finish under random task durations (each workgroup runs its list in order and a
task starts only when its counters are full) -- the plan cannot deadlock whatever the timing,
given the whole grid resident."""
import ctypes as C
import heapq

import numpy as np
import pytest

pytestmark = pytest.mark.experiment  # the plan lives in the experiments build (knobs.h)

from midagma_amd import _lib

TASK_INTS = 12


def _plan(D, passes, nwg):
    L = _lib.load()
    f = L.midagma_debug_df_plan
    f.restype = C.c_int
    f.argtypes = [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_void_p,
                  C.c_void_p, C.POINTER(C.c_int)]
    est, nt, nc = C.c_double(), C.c_int64(), C.c_int()
    assert f(D, passes, nwg, C.byref(est), C.byref(nt), None, None, C.byref(nc)) == 0
    tasks = np.zeros(nt.value * TASK_INTS, dtype=np.int32)
    woff = np.zeros(nwg + 1, dtype=np.int32)
    assert f(D, passes, nwg, None, None, tasks.ctypes.data, woff.ctypes.data, None) == 0
    return tasks.reshape(-1, TASK_INTS), woff, nc.value, est.value


def _simulate(tasks, woff, nctr, rng):
    """Event simulation: returns the makespan, or raises on a deadlock."""
    nwg = len(woff) - 1
    dur = rng.uniform(0.2, 5.0, size=len(tasks))
    nsig = np.zeros(nctr, dtype=np.int64)
    for t in tasks:
        if t[5] >= 0:
            nsig[t[5]] += 1
    count = np.zeros(nctr, dtype=np.int64)
    full_at = np.full(nctr, np.inf)
    ptr = woff[:-1].copy()
    free = np.zeros(nwg)
    heap = [(0.0, w) for w in range(nwg) if ptr[w] < woff[w + 1]]
    heapq.heapify(heap)
    blocked = {}  # counter -> workgroups waiting on it
    done = 0
    makespan = 0.0

    def try_start(w):
        t = tasks[ptr[w]]
        ready = free[w]
        for k in range(3):
            c, tgt = t[6 + k], t[9 + k]
            if c < 0:
                continue
            assert tgt == nsig[c], "counter target differs from its signal count"
            if count[c] < tgt:
                blocked.setdefault(c, []).append(w)
                return
            ready = max(ready, full_at[c])
        heapq.heappush(heap, (ready, w))

    pending = []
    while heap:
        start, w = heapq.heappop(heap)
        i = ptr[w]
        t = tasks[i]
        # re-check: the task was pushed only when all its counters were full
        fin = start + dur[i]
        makespan = max(makespan, fin)
        free[w] = fin
        done += 1
        ptr[w] += 1
        s = t[5]
        if s >= 0:
            count[s] += 1
            if count[s] == nsig[s]:
                full_at[s] = fin if not np.isfinite(full_at[s]) else max(full_at[s], fin)
                for ww in blocked.pop(s, []):
                    pending.append(ww)
            else:
                full_at[s] = fin if not np.isfinite(full_at[s]) else max(full_at[s], fin)
        if ptr[w] < woff[w + 1]:
            pending.append(w)
        while pending:
            try_start(pending.pop())
    assert done == len(tasks), f"deadlock: {done} of {len(tasks)} tasks ran"
    return makespan


@pytest.mark.parametrize("D,passes,nwg", [(512, 2, 256), (512, 3, 64), (1024, 2, 256), (1024, 3, 256),
                                          (1024, 2, 80), (1536, 2, 256)])
def test_plan_counts_and_no_deadlock(D, passes, nwg):
    tasks, woff, nctr, est = _plan(D, passes, nwg)
    K2 = D // 256
    per_step = 256 * (1 + passes) + 2 * 8 * (D // 32 - 8) + 64 + (D // 32 - 8) ** 2
    assert len(tasks) == K2 * per_step
    assert woff[0] == 0 and woff[-1] == len(tasks) and np.all(np.diff(woff) >= 0)
    # every (type, g, p, a, b) exactly once
    keys = {tuple(t[:5]) for t in tasks}
    assert len(keys) == len(tasks)
    rng = np.random.default_rng(D + passes + nwg)
    for _ in range(2):
        span = _simulate(tasks, woff, nctr, rng)
        assert np.isfinite(span)
    print(f"D={D} passes={passes} nwg={nwg}: {len(tasks)} tasks, planned {est:.1f} us")
