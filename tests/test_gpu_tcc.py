"""TCC trek regularizer on the GPU (csrc/tcc.hip: Noda iteration on the Gauss-Jordan M-matrix
inverse) vs the reference's trek_value_grad / minimize (tests/golden/trek_tcc.npz) and the
oracle (oracle/trek_oracle.py::tcc_value_grad, numpy eig as the reference).

Tolerances: the Perron pair comes from a different (iterative) algorithm than LAPACK's
eigendecomposition, so value and gradient agree to the eigenvector conditioning, not bit for
bit: 1e-10 relative; W after the loop 1e-9 (the north star asks 1e-5)."""
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle.dagma_oracle import LinearOracle  # noqa: E402
from oracle.trek_oracle import tcc_value_grad  # noqa: E402


def _solver(d, cov):
    from midagma_amd.solver import HipSolver
    s = HipSolver(d, "l2", "cov", device=0)
    s.set_cov(cov)
    return s


@pytest.mark.parametrize("d", [8, 20])
@pytest.mark.parametrize("case", ["dense", "tiny", "dag"])
@pytest.mark.parametrize("w", [1.0, 2.0])
def test_tcc_value_grad_matches_reference(golden, d, case, w):
    f = golden("trek_tcc.npz")
    W, pairs = f[f"W_{case}_d{d}"], f[f"pairs_d{d}"]
    s = _solver(d, np.eye(d))
    s.set_trek_tcc(pairs, mode="opt", weight=0.5, w=w)
    v, g = s.trek_value(W)
    v_ref, g_ref = float(f[f"val_{case}_w{w:g}_d{d}"]), f[f"grad_{case}_w{w:g}_d{d}"]
    assert abs(v - v_ref) <= 1e-10 * abs(v_ref)
    assert np.abs(g - g_ref).max() <= 1e-10 * np.abs(g_ref).max()
    # again from the warm start the first call left: same answer
    v2, g2 = s.trek_value(W)
    assert abs(v2 - v_ref) <= 1e-10 * abs(v_ref)
    assert np.abs(g2 - g_ref).max() <= 1e-10 * np.abs(g_ref).max()
    s.close()


@pytest.mark.parametrize("d", [64, 300])
def test_tcc_value_grad_matches_oracle_larger(d):
    rng = np.random.default_rng(d)
    W = rng.uniform(-1, 1, (d, d)) * (0.6 / np.sqrt(d))
    np.fill_diagonal(W, 0)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.1]
    s = _solver(d, np.eye(d))
    s.set_trek_tcc(pairs, mode="opt", weight=1.0)
    v, g = s.trek_value(W)
    vr, gr = tcc_value_grad(W, pairs)
    assert abs(v - vr) <= 1e-10 * abs(vr)
    assert np.abs(g - gr).max() <= 1e-10 * np.abs(gr).max()
    s.close()


def test_tcc_at_zero_and_log_mode(golden):
    """W = 0 (a fit's start): A is nilpotent (no Perron gap) -- the gradient 2 W o G is exactly 0
    and the value finite; 'log' mode returns a zero gradient as the reference does."""
    f = golden("trek_tcc.npz")
    pairs = f["pairs_d20"]
    s = _solver(20, np.eye(20))
    s.set_trek_tcc(pairs, mode="opt", weight=0.5)
    v, g = s.trek_value(np.zeros((20, 20)))
    assert np.isfinite(v) and not g.any()
    s.set_trek_tcc(pairs, mode="log", weight=0.5)
    W = f["W_dense_d20"]
    v, g = s.trek_value(W)
    assert abs(v - float(f["val_dense_w1_d20"])) <= 1e-10 * abs(v) and not g.any()
    s.set_trek_tcc(np.zeros((0, 2), dtype=np.int64), mode="opt", weight=0.5)
    v, g = s.trek_value(W)
    assert v == 0.0 and not g.any()
    s.close()


@pytest.mark.parametrize("mode", ["opt", "log"])
@pytest.mark.parametrize("K", [1, 10, 90])
def test_minimize_with_tcc_matches_reference(golden, mode, K):
    f = golden("trek_tcc.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"]
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 40)
    s = _solver(20, o.cov)
    s.set_trek_tcc(f["pairs_d20"], mode=mode, weight=0.2)
    W = np.zeros((20, 20))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=40)
    assert res.iters == int(f[f"traj_{mode}_it_K{K}"])
    assert np.abs(W - f[f"traj_{mode}_W_K{K}"]).max() <= 1e-9
    s.close()


@pytest.mark.parametrize("d,mode", [(20, "opt"), (20, "log"), (300, "opt")])
def test_minimize_with_tcc_checkpoints_match_oracle(golden, d, mode):
    """Checkpoint records with TCC: objective (+ weight * value in 'opt'), reg_trek_value,
    grad_trek_norm.  d=300 runs the blocked fast path with the 600 x 600 Perron problem."""
    from midagma_amd.simulate import make_dataset
    X, _, _ = make_dataset(d, 1000 if d == 20 else 600, seed=5)
    rng = np.random.default_rng(5)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 40)
    o.trek = dict(kind="tcc", pairs=pairs, mode=mode, weight=0.2)
    K = 90 if d == 20 else 45
    s = _solver(d, o.cov)
    s.set_trek_tcc(pairs, mode=mode, weight=0.2)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=40, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == K
    assert np.abs(W - Wr).max() <= 1e-9
    assert [c.iter for c in res.checkpoints] == [r["iter"] for r in tr.records]
    for c, r in zip(res.checkpoints, tr.records):
        assert abs(c.obj - r["obj_total"]) <= 1e-10 * abs(r["obj_total"])
        assert abs(c.reg_trek_value - r["reg_trek_value"]) <= 1e-9 * abs(r["reg_trek_value"])
        assert abs(c.grad_trek_norm - r["grad_trek_norm"]) <= 1e-9 * r["grad_trek_norm"] + 1e-15
    s.close()


def test_dagma_linear_tcc_fit_runs(golden):
    from midagma_amd import DagmaLinear
    f = golden("trek_tcc.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"]
    pairs = f["pairs_d20"]
    reg = SimpleNamespace(name="tcc", mode="opt", weight=0.1, cycle_penalty="logdet",
                          cfg={"I": pairs, "version": "exact_trek_graph", "w": 1.0, "n_iter": 10, "eps": 1e-12,
                               "s": 1.0}, enabled=lambda: True)
    m = DagmaLinear("l2", trek_reg=reg)
    W = m.fit(X, lambda1=0.03, T=2, warm_iter=200, max_iter=300)
    assert W.shape == (20, 20) and np.isfinite(W).all()
    Wd = f["W_dense_d20"]
    obj, sc, h, tv = m._func(Wd, 0.1, 1.0)
    v_ref, _ = tcc_value_grad(Wd, pairs)   # the loop ignores cycle_penalty / version (notreks.py:691)
    assert abs(tv - v_ref) <= 1e-10 * abs(v_ref)


def _tcc_case(d, seed=7):
    from midagma_amd.simulate import make_dataset
    X, _, _ = make_dataset(d, 2 * d, seed=seed)
    rng = np.random.default_rng(seed)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    o.trek = dict(kind="tcc", pairs=pairs, mode="opt", weight=0.2)
    return o, pairs


@pytest.mark.parametrize("d", [100, 300])
def test_tcc_short_chain_hands_back(d):
    """TCC with 2d > 128 on fast cov slots.  With the fixed-shift stage (one inverse at the warm
    start's Collatz-Wielandt bound, inverse iteration for v and u) the fast slot's chain is that
    stage alone, and a slot it does not settle hands back (tcc.hip tcc_handback_kernel); without it,
    a short Noda chain first: forced to hand back nearly every slot (1 step), by default (5 steps),
    and the whole chain on every slot (0).  The re-run is a pivoted slot with the whole chain.  W after
    60 steps from W = 0 (where the Perron gap is smallest and most fast slots hand back) within 1e-9
    of the oracle each time."""
    o, pairs = _tcc_case(d)
    K = 60
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    backs = {}
    for fix, steps in ((False, 1), (False, None), (False, 0), (True, None)):
        s = _solver(d, o.cov)
        s.debug_tcc_fix(fix)
        if steps is not None:
            s.debug_tcc_fast_steps(steps)
        s.set_trek_tcc(pairs, mode="opt", weight=0.2)
        W = np.zeros((d, d))
        res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000)
        backs[fix, steps] = s.debug_handbacks()
        s.close()
        assert res.iters == K
        assert np.abs(W - Wr).max() <= 1e-9, (fix, steps, np.abs(W - Wr).max())
    assert backs[False, 1] >= K // 3  # forced: most fast slots handed back
    assert backs[False, 0] == 0


def test_tcc_fixed_stage_settles_warm_slots():
    """Past a fit's first steps the fixed-shift stage settles the fast slots by itself (d = 100:
    no more than 2 of the last 100 of 500 slots hand back), and W after the 500 steps is within 1e-9
    of the oracle's."""
    d, K0, K1 = 100, 400, 100
    o, pairs = _tcc_case(d)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K0 + K1, 1.0, 3e-4, tol=-1.0)
    s = _solver(d, o.cov)
    s.set_trek_tcc(pairs, mode="opt", weight=0.2)
    W = np.zeros((d, d))
    s.begin(W, 1.0, K0 + K1, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000)
    for _ in range(200):  # (a hand-back's re-run takes a slot of its own)
        if s.poll().iters >= K0:
            break
        s.run_slots(10)
    b0, i0 = s.debug_handbacks(), s.poll().iters
    for _ in range(200):
        if s.poll().iters >= K0 + K1:
            break
        s.run_slots(10)
    late = s.debug_handbacks() - b0
    res = s.end(W)
    s.close()
    assert res.iters == K0 + K1
    assert late <= 2, (late, K0 + K1 - i0)
    assert np.abs(W - Wr).max() <= 1e-9, np.abs(W - Wr).max()


def test_tcc_fast_blocks_match_the_pivoted_inverse_d1000():
    """d = 1000 (D2 = 2048, eight 256-blocks): the fixed-stage inverse of fast slots with every outer
    block but the last on the warm-started product-form series (tcc.hip tcc_inverse_fix) against
    the all-pivoted inverse: W after 80 steps from W = 0 (hand-backs included) within 1e-9."""
    d, K = 1000, 80
    o, pairs = _tcc_case(d)
    out = {}
    for fb in (False, True):
        s = _solver(d, o.cov)
        s.debug_tcc_fastblk(fb)
        s.set_trek_tcc(pairs, mode="opt", weight=0.2)
        W = np.zeros((d, d))
        res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000)
        assert res.iters == K
        out[fb] = (W.copy(), s.debug_handbacks())
        s.close()
    assert np.abs(out[True][0] - out[False][0]).max() <= 1e-9, np.abs(out[True][0] - out[False][0]).max()
