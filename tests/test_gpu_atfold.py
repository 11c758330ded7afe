"""build_at folded into the previous slot's update (solver_impl.h at_fold, step.hip
fused_update_at_kernel): fast cov slots read outer step 0's A^T from the buffer the previous
slot's update wrote.  The fold only moves where A^T = s I - (W o W)^T and I - W are formed, so
every result is bit-identical to the unfolded slot: W, iterations, halvings, lr and the
checkpoint records, over slow/fast interleavings (checkpoints), the line search, hand-backs,
several calls on one solver, float32 W and the TCC regularizer."""
import numpy as np
import pytest

from midagma_amd.simulate import make_dataset
from oracle.dagma_oracle import LinearOracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _cov(d, seed=7):
    X, _, _ = make_dataset(d, 2 * d, seed=seed)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    return o.cov


def _run(d, cov, fold, calls, w32=False, trek=None):
    from midagma_amd.solver import HipSolver
    s = HipSolver(d, "l2", "cov", device=0)
    try:
        s.set_cov(cov)
        if w32:
            s.set_w_float32(True)
        if trek is not None:
            s.set_trek_tcc(trek, mode="opt", weight=0.2)
        assert s.debug_at_fold(fold) in (0, 1)
        W = np.zeros((d, d))
        out = []
        for mu, K, lr, ck in calls:
            res = s.minimize(W, mu, K, 1.0, lr, tol=-1.0, lambda1=0.03, checkpoint=ck, want_checkpoints=True)
            cks = [c._replace(elapsed=0.0) if hasattr(c, "_replace") else c for c in res.checkpoints]
            out.append((res.iters, res.halvings, res.lr_final, res.success, cks))
        return W.copy(), out, s.debug_handbacks()
    finally:
        s.close()


@pytest.mark.parametrize("d", [300, 500, 1000])
def test_at_fold_bit_identical(d):
    cov = _cov(d)
    calls = [(1.0, 45, 3e-4, 15), (0.1, 30, 3e-4, 1000)]
    W0, r0, _ = _run(d, cov, False, calls)
    W1, r1, _ = _run(d, cov, True, calls)
    assert np.array_equal(W0, W1), np.abs(W0 - W1).max()
    assert r0 == r1


def test_at_fold_line_search_bit_identical():
    """lr = 0.3 at d = 300: three halvings in 60 steps (test_gpu_parity.test_blocked_path_line_search)"""
    d = 300
    cov = _cov(d)
    calls = [(1.0, 60, 0.3, 20)]
    W0, r0, _ = _run(d, cov, False, calls)
    W1, r1, _ = _run(d, cov, True, calls)
    assert r0[0][1] == 3
    assert np.array_equal(W0, W1)
    assert r0 == r1


def test_at_fold_float32_and_tcc_bit_identical():
    d = 300
    cov = _cov(d)
    rng = np.random.default_rng(7)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    calls = [(1.0, 40, 3e-4, 13)]
    for kw in (dict(w32=True), dict(trek=pairs)):
        W0, r0, b0 = _run(d, cov, False, calls, **kw)
        W1, r1, b1 = _run(d, cov, True, calls, **kw)
        assert np.array_equal(W0, W1), kw
        assert r0 == r1 and b0 == b1, kw


def test_at_fold_rejected_where_it_cannot_apply():
    from midagma_amd.solver import HipSolver
    s = HipSolver(64, "l2", "data", device=0)  # data mode: no blocked cov slots
    try:
        assert s.debug_at_fold(True) == -1
    finally:
        s.close()
