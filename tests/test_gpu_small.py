"""The one-workgroup small-d inner loop (csrc/small.hip: cov mode, l2, d <= 64) against the
oracle (the numpy/scipy restatement of linear.py:165-333) and across launch boundaries (run_slots chunks that
end right after a checkpoint step, so the pending checkpoint norms cross launches)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402

REC_FIELDS = ("obj", "score", "h", "lr", "w_norm", "max_abs_w", "min_abs_w_nonzero", "grad_raw_norm",
              "grad_step_norm", "grad_score_norm", "grad_dag_norm", "grad_l1_norm", "grad_inc_norm")
ORACLE_KEYS = dict(obj="obj_total", score="score_datafit", h="reg_dag_value")


def _oracle(d, n=None, seed=11, exc=None, inc=None):
    X, _, _ = make_dataset(d, n or max(200, 10 * d), seed=seed)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 50, exc, inc)
    return o


def _solver(d, cov, masks=None):
    from midagma_amd.solver import HipSolver
    s = HipSolver(d, "l2", "cov", device=0)
    s.set_cov(cov)
    if masks is not None:
        s.set_masks(*masks)
    return s


def _check_records(res, tr):
    assert [c.iter for c in res.checkpoints] == [r["iter"] for r in tr.records]
    for c, r in zip(res.checkpoints, tr.records):
        for f in REC_FIELDS:
            want = r[ORACLE_KEYS.get(f, f)]
            got = getattr(c, f)
            assert abs(got - want) <= 1e-9 * max(1.0, abs(want)), (c.iter, f, got, want)


@pytest.mark.parametrize("d", [1, 4, 16, 17, 20, 31, 32, 33, 48, 64])
def test_small_path_matches_oracle(d):
    o = _oracle(d)
    K = 300
    s = _solver(d, o.cov)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.success and res.iters == tr.iters == K and res.slots == K + 1  # + the last objective
    assert np.abs(W - Wr).max() <= 1e-9
    _check_records(res, tr)
    s.close()


def test_small_path_masks_and_early_stop():
    d = 20
    exc = ((0, 1), (3, 2), (5, 7))
    inc = ((1, 0), (4, 9))
    o = _oracle(d, exc=exc, inc=inc)
    mi, me = o.masks(1.0)
    s = _solver(d, o.cov, masks=(mi, me))
    W = np.zeros((d, d))
    # tol 1e-6: the checkpoint tolerance stops the loop (linear.py:328-331)
    res = s.minimize(W, 1.0, 20000, 1.0, 3e-4, tol=1e-6, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 20000, 1.0, 3e-4, tol=1e-6)
    assert tr.early_stop and res.early_stop and res.iters == tr.iters
    assert np.abs(W - Wr).max() <= 1e-9
    assert W[0, 1] == W[3, 2] == W[5, 7] == 0.0
    _check_records(res, tr)
    s.close()


def test_small_path_line_search_branches(golden):
    """lr halving at s = 1 and the out-of-domain failure at s <= 0.9 (linear.py:230-241), on
    the reference's own fixture (branches.npz)."""
    b = golden("branches.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 1000)
    for s_dom, key in ((1.0, "halve"), (0.9, "ood")):
        s = _solver(20, o.cov)
        W = np.zeros((20, 20))
        res = s.minimize(W, 1.0, 60, s_dom, 0.3, tol=-1.0, lambda1=0.03)
        assert res.success == bool(b[f"{key}_ok"])
        assert np.abs(W - b[f"{key}_W"]).max() <= 1e-9
        if key == "halve":
            assert res.halvings == int(b["halve_nhalvings"])
        s.close()


@pytest.mark.parametrize("d", [20, 32, 64])
def test_small_path_launch_boundaries_bit_identical(d):
    """run_slots in chunks of 50 with checkpoint = 50: every launch ends right after a
    checkpoint step, so the step's norms cross to the next launch.  Same kernel arithmetic:
    W and every checkpoint record field are bit-identical to one minimize call."""
    o = _oracle(d)
    K = 400
    a = _solver(d, o.cov)
    Wa = np.zeros((d, d))
    ra = a.minimize(Wa, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    b = _solver(d, o.cov)
    b.begin(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50)
    for _ in range(K // 50 + 2):
        b.run_slots(50)
    Wb = np.zeros((d, d))
    rb = b.end(Wb)
    cb = b.checkpoints()
    assert rb.iters == ra.iters == K
    assert np.array_equal(Wa, Wb)
    assert len(cb) == len(ra.checkpoints)
    for x, y in zip(ra.checkpoints, cb):
        for f in REC_FIELDS:
            assert getattr(x, f) == getattr(y, f), (x.iter, f)
    a.close()
    b.close()


@pytest.mark.parametrize("d", [20, 48])
def test_small_path_unaligned_launches_bit_identical(d):
    """run_slots in chunks of 37 with checkpoint = 50 and max_iter = 333 (not a multiple of it):
    launches start mid-interval, so the next checkpoint iteration each launch derives from the
    State (small.hip's next_ck) and the plain steps decided from register copies of the State must
    agree with one minimize call, bit for bit, including the final non-multiple checkpoint."""
    o = _oracle(d)
    K = 333
    a = _solver(d, o.cov)
    Wa = np.zeros((d, d))
    ra = a.minimize(Wa, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    b = _solver(d, o.cov)
    b.begin(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50)
    for _ in range(K // 37 + 3):
        b.run_slots(37)
    Wb = np.zeros((d, d))
    rb = b.end(Wb)
    cb = b.checkpoints()
    assert rb.iters == ra.iters == K
    assert [c.iter for c in cb] == [c.iter for c in ra.checkpoints] == list(range(50, K, 50)) + [K]
    assert np.array_equal(Wa, Wb)
    for x, y in zip(ra.checkpoints, cb):
        for f in REC_FIELDS:
            assert getattr(x, f) == getattr(y, f), (x.iter, f)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert np.abs(Wa - Wr).max() <= 1e-9
    a.close()
    b.close()


def test_small_path_long_trajectory_d20(golden, parity):
    """10000 steps at d=20 against the reference's own trajectory (traj_d20.npz): ~9990
    product-form slots between the Gauss-Jordan checkpoint slots."""
    t = golden("traj_d20.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 1000)
    s = _solver(20, o.cov)
    W = np.zeros((20, 20))
    res = s.minimize(W, 1.0, 10000, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    assert res.iters == 10000
    parity("config1", float(np.abs(W - t["W_K10000"]).max()), max(1e-9, 2 * float(t["env_K10000"])), "max|dW| K=10000")
    assert np.abs(W - t["W_K10000"]).max() <= max(1e-9, 2 * float(t["env_K10000"]))
    s.close()
