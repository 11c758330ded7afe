"""`DagmaLinear(devices=[...])` (ABI 11, a single-process device group) on the CPU: the product's
Python path -- the group taken instead of a process group, X handed over whole for the library to
shard, cov as the reference's host product or from the members' summed Gram matrices, masks and
dtype broadcast to every member, `_score` through the group's sum -- over a CPU double of
`HipGroup` whose loop is the oracle's data-mode restatement of linear.py:165-333 on the shards.
The GPU form is tests/test_gpu_group.py."""
import numpy as np
import pytest

from midagma_amd import _lib
from midagma_amd.solver import MinimizeResult, row_range


class _FakeGroup:
    is_group = True
    emulated = True

    def __init__(self, d, loss, devices=(0,)):
        assert loss == "l2"
        self.d, self.size = d, len(devices)
        self.calls = []
        _FakeGroup.last = self

    def set_data(self, X, n_global=None):
        self.X = np.array(X)
        self.shards = [self.X[slice(*row_range(len(X), self.size, k))] for k in range(self.size)]
        self.calls.append("set_data")

    def set_cov(self, cov):
        self.cov = np.array(cov)
        self.calls.append("set_cov")

    def gram_cov(self, n):
        G = sum(S.T @ S for S in self.shards)
        self.cov = G / float(n)
        self.calls.append("gram_cov")
        return self.cov

    def set_w_float32(self, on):
        assert not on

    def set_masks(self, mask_inc, mask_exc):
        self.masks = (mask_inc, mask_exc)

    def minimize(self, W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint, want_checkpoints=False):
        from oracle.dagma_oracle import LinearOracle
        o = LinearOracle("l2", score_mode="data")
        o.X, o.n, o.d, o.eye, o.cov = np.concatenate(self.shards), self.X.shape[0], self.d, np.eye(self.d), self.cov
        o.lambda1, o.checkpoint = lambda1, checkpoint
        inc, exc = self.masks
        o.inc = tuple(np.nonzero(inc)) if inc is not None else None
        o.exc = tuple(np.nonzero(exc == 0)) if exc is not None else None
        Wn, tr = o.minimize(W.copy(), mu, max_iter, s, lr, tol, b1, b2)
        W[...] = Wn
        return MinimizeResult(iters=tr.iters, success=tr.success, status=_lib.ST_DONE if tr.success else _lib.ST_FAILED,
                              halvings=tr.halvings, early_stop=tr.early_stop, lr_final=tr.lr_final, slots=tr.iters,
                              obj_last=0.0, score_last=0.0, h_last=0.0)

    def checkpoints(self):
        return []

    def h_value(self, W, s=1.0, grad=True):
        from oracle.dagma_oracle import h_logdet
        return h_logdet(np.asarray(W, dtype=np.float64), s)

    def trek_value(self, W, grad=True):
        return 0.0, None

    def score_partial(self, W):
        self._W = np.array(W)
        self.calls.append("score_partial")

    def comm_allreduce_zbuf(self):
        self.calls.append("allreduce")
        I = np.eye(self.d)
        self._Z = sum(S.T @ (S @ (I - self._W)) for S in self.shards)

    def score_finish(self):
        n = self.X.shape[0]
        diff = np.eye(self.d) - self._W
        return 0.5 * np.sum(diff * self._Z) / n, -(self._Z / n)


def test_fit_devices_takes_the_group_path(golden):
    from midagma_amd import DagmaLinear
    from oracle.dagma_oracle import LinearOracle
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    kw = dict(lambda1=0.03, T=2, warm_iter=800, max_iter=900, exclude_edges=((0, 1),))
    m = DagmaLinear("l2", devices=[0, 0, 0], group_factory=_FakeGroup)
    assert m.score_mode == "data"
    W = m.fit(X.copy(), **kw)
    g = _FakeGroup.last
    assert g.size == 3 and g.calls[:2] == ["set_data", "set_cov"]
    assert "allreduce" in g.calls  # score_final summed over the members
    o = LinearOracle("l2", score_mode="data")
    W_ref = o.fit(X.copy(), **kw)
    assert np.abs(W - W_ref).max() <= 1e-9 and np.array_equal(W != 0, W_ref != 0)
    assert W[0, 1] == 0
    assert abs(m.score_final - o.score_final) <= 1e-9 * abs(o.score_final)
    # gram='device': cov from the members' Gram matrices (the host-product path otherwise)
    m2 = DagmaLinear("l2", devices=[0, 0], group_factory=_FakeGroup)
    m2.fit(X.copy(), lambda1=0.03, T=1, max_iter=5, gram="device")
    assert "gram_cov" in _FakeGroup.last.calls and "set_cov" not in _FakeGroup.last.calls
    assert np.abs(m2.cov - o.cov).max() <= 1e-12 * np.abs(o.cov).max()


def test_devices_argument_validation():
    from midagma_amd import DagmaLinear
    with pytest.raises(ValueError):
        DagmaLinear("l2", devices=[])
    with pytest.raises(ValueError):
        DagmaLinear("l2", devices=[0, 1], score_mode="cov")
    with pytest.raises(ValueError):
        DagmaLinear("l2", devices=[0, 1], comm="library")
    m = DagmaLinear("logistic", devices=[1, 2])
    assert m.score_mode == "data" and m.device == 1
    with pytest.raises(ValueError):
        DagmaLinear("l2", devices=[0, 0], group_factory=_FakeGroup).fit(np.zeros((10, 4)), n_global=20)


def test_row_range_matches_linear_split():
    from midagma_amd.linear import _row_range
    for n in (3, 10, 1001):
        for p in (1, 2, 3, 7):
            assert [row_range(n, p, k) for k in range(p)] == [_row_range(n, p, k) for k in range(p)]
