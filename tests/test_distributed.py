"""Multi-rank data mode: X row-sharded over ranks, one all-reduce of the
score partial per step, W replicated.  Runs on CPU with the gloo backend, world_size 2.

The product driver `midagma_amd.solver.run_allreduce_minimize` is exercised with a CPU
test double of the HIP backend (`_ShardBackend`): the same begin / step_partial /
all-reduce / step_finish / poll / end protocol, with each step's arithmetic taken from
the oracle.  The sum over ranks must reproduce the single-process reference trajectory.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from midagma_amd import _lib  # noqa: E402
from midagma_amd.linear import _row_range  # noqa: E402


class _Res:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class _ShardBackend:
    """CPU stand-in for HipSolver in data mode: holds the rank's rows of X."""

    def __init__(self, X_local, n_global, lambda1):
        from oracle.dagma_oracle import AdamState
        self.X, self.n, self.l1 = X_local, n_global, lambda1
        self.d = X_local.shape[1]
        self.z = torch.zeros(self.d * self.d, dtype=torch.float64)
        self._Adam = AdamState

    def begin(self, W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint):
        self.W = np.array(W, dtype=np.float64)
        self.mu, self.max_iter, self.s, self.lr = mu, max_iter, s, lr
        self.b1, self.b2, self.ckpt = b1, b2, checkpoint
        self.adam = self._Adam()
        self.it, self.status, self.halvings, self.grad = 0, _lib.ST_RUNNING, 0, None

    def step_partial(self):
        if self.status != _lib.ST_RUNNING:
            return
        Zk = self.X.T @ (self.X @ (np.eye(self.d) - self.W))
        self.z.copy_(torch.from_numpy(Zk.reshape(-1)))

    def step_finish(self):
        import scipy.linalg as sla
        from oracle.dagma_oracle import adam_step
        if self.status != _lib.ST_RUNNING:
            return
        M = sla.inv(self.s * np.eye(self.d) - self.W * self.W) + 1e-16
        if np.any(M < 0):
            if self.it == 0 or self.s <= 0.9:
                self.status = _lib.ST_FAILED
                return
            self.W += self.lr * self.grad
            self.lr *= .5
            self.halvings += 1
            if self.lr <= 1e-16:
                self.status = _lib.ST_LR_UNDERFLOW
                return
            self.W -= self.lr * self.grad
            return
        Z = self.z.numpy().reshape(self.d, self.d)
        G = (-self.mu / self.n) * Z
        Gobj = G + self.mu * self.l1 * np.sign(self.W) + 2 * self.W * M.T
        self.it += 1
        self.grad = adam_step(self.adam, Gobj, self.it, self.b1, self.b2)
        self.W -= self.lr * self.grad
        if self.it >= self.max_iter:
            self.status = _lib.ST_DONE

    def poll(self):
        return _Res(status=self.status, iters=self.it)

    def end(self, W):
        W[...] = self.W
        return _Res(iters=self.it, status=self.status, success=self.status != _lib.ST_FAILED)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, X, K, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd.solver import run_allreduce_minimize
        n, d = X.shape
        lo, hi = _row_range(n, world, rank)
        be = _ShardBackend(X[lo:hi], n, 0.03)
        W = np.zeros((d, d))

        def allreduce():
            dist.all_reduce(be.z)

        res = run_allreduce_minimize(be, W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000,
                                     allreduce=allreduce, batch=7)
        out_q.put((rank, W, res.iters))
    finally:
        dist.destroy_process_group()


def test_row_range_partitions_exactly():
    for n in (1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            spans = [_row_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [2])
def test_data_parallel_matches_single_process(world, golden):
    from oracle.dagma_oracle import LinearOracle
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    X = X - X.mean(axis=0, keepdims=True)
    K = 150
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, X, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs.sort(key=lambda t: t[0])
    W0 = outs[0][1]
    for _, W, iters in outs:
        assert iters == K
        assert np.array_equal(W, W0), "replicas diverged"
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    W_ref, tr = o.minimize(np.zeros((20, 20)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert tr.iters == K
    assert np.abs(W0 - W_ref).max() <= 1e-9


class _EarlyStopBackend(_ShardBackend):
    """A replica whose controller stops early (as a rank handed different all-reduce bits
    could): it reports ST_DONE after `stop_at` steps."""

    def __init__(self, *a, stop_at):
        super().__init__(*a)
        self.stop_at = stop_at

    def step_finish(self):
        super().step_finish()
        if self.status == _lib.ST_RUNNING and self.it >= self.stop_at:
            self.status = _lib.ST_DONE


def _diverge_worker(rank, world, port, X, out_q):
    import types
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd.linear import DagmaLinear
        from midagma_amd.solver import run_allreduce_minimize
        n, d = X.shape
        lo, hi = _row_range(n, world, rank)
        be = _EarlyStopBackend(X[lo:hi], n, 0.03, stop_at=10 if rank == 1 else 10 ** 9)
        me = types.SimpleNamespace(process_group=None, device=0)

        def allreduce():
            dist.all_reduce(be.z)

        try:
            run_allreduce_minimize(be, np.zeros((d, d)), 1.0, 100, 1.0, 3e-4, tol=-1.0, lambda1=0.03,
                                   checkpoint=1000, allreduce=allreduce, batch=7,
                                   agree=lambda st, it: DagmaLinear._agree(me, st, it))
            out_q.put((rank, "returned", ""))
        except _lib.HipSolverError as e:
            out_q.put((rank, "raised", str(e)))
    finally:
        dist.destroy_process_group()


def test_divergent_replica_raises_instead_of_hanging(golden):
    """A rank whose controller decides differently stops issuing all-reduces; the poll-time
    agreement (DagmaLinear._agree) makes every rank raise instead of waiting forever."""
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    X = X - X.mean(axis=0, keepdims=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_diverge_worker, args=(r, 2, port, X, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[1] for o in outs] == ["raised", "raised"], outs
    assert "diverged" in outs[0][2]


class _ShardSolver(_ShardBackend):
    """CPU double of HipSolver for DagmaLinear.fit in data mode: the calls fit() makes
    (set_data / data_gram / torch_zbuf / cov_from_zbuf / get_cov / the step protocol / h / score),
    each on this rank's rows only."""

    def __init__(self, d, loss, mode, device=0):
        assert loss == "l2" and mode == "data"
        self.d = d
        self.zfull = torch.zeros(d * d + 64, dtype=torch.float64)  # the bound score buffer (+ tail)
        self.z = self.zfull[:d * d]
        self.rows_seen = 0

    def set_data(self, X, n_global=None):
        from oracle.dagma_oracle import AdamState
        self.X, self.n = np.array(X), int(n_global)
        self.rows_seen = self.X.shape[0]
        self._Adam = AdamState

    def torch_zbuf(self):
        import contextlib
        return self.zfull, contextlib.nullcontext

    def data_gram(self):
        self.z.copy_(torch.from_numpy((self.X.T @ self.X).reshape(-1)))

    def cov_from_zbuf(self, n):
        self.cov = self.z.numpy().reshape(self.d, self.d) / n

    def get_cov(self):
        return self.cov.copy()

    def set_masks(self, mask_inc, mask_exc):
        assert mask_inc is None and mask_exc is None

    def begin(self, W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint):
        self.l1 = lambda1
        super().begin(W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint)

    def step_partial(self):
        if self.status != _lib.ST_RUNNING:
            return
        Zk = self.X.T @ (self.X @ (np.eye(self.d) - self.W))
        self.z.copy_(torch.from_numpy(Zk.reshape(-1)))

    def end(self, W):
        from midagma_amd.solver import MinimizeResult
        W[...] = self.W
        return MinimizeResult(iters=self.it, success=self.status != _lib.ST_FAILED, status=self.status,
                              halvings=self.halvings, early_stop=False, lr_final=self.lr, slots=self.it,
                              obj_last=0.0, score_last=0.0, h_last=0.0)

    def h_value(self, W, s=1.0, grad=True):
        from oracle.dagma_oracle import h_logdet
        return h_logdet(W, s)

    def score_partial(self, W):
        self._diff = np.eye(self.d) - W
        Zk = self.X.T @ (self.X @ self._diff)
        self.z.copy_(torch.from_numpy(Zk.reshape(-1)))

    def score_finish(self):
        Z = self.z.numpy().reshape(self.d, self.d)
        return 0.5 * (np.sum(self._diff * Z) / self.n), -(Z / self.n)


def _fit_worker(rank, world, port, X_shard, n_global, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd import DagmaLinear
        m = DagmaLinear("l2", score_mode="data", solver_factory=_ShardSolver)
        Xs = X_shard.copy()
        W = m.fit(Xs, lambda1=0.03, T=2, warm_iter=300, max_iter=400, n_global=n_global)
        out_q.put((rank, W, m.cov, Xs, m._solver.rows_seen, m.h_final, m.score_final,
                   [e["iters"] for e in m.minimize_log]))
    finally:
        dist.destroy_process_group()


def test_sharded_fit_each_rank_ingests_only_its_rows(golden):
    """fit(X_shard, n_global=n) over 2 gloo ranks: every rank receives only its rows; the
    centring (all-reduced column sums) and cov (all-reduced Gram matrices) are the oracle's
    to rounding, and the fit matches the oracle's fit of the full X to 1e-9."""
    from oracle.dagma_oracle import LinearOracle
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    n, world = X.shape[0], 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    spans = [_row_range(n, world, r) for r in range(world)]
    procs = [ctx.Process(target=_fit_worker, args=(r, world, port, X[lo:hi].copy(), n, q))
             for r, (lo, hi) in enumerate(spans)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=150) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = LinearOracle("l2")
    W_ref = o.fit(X.copy(), lambda1=0.03, T=2, warm_iter=300, max_iter=400)
    for r, W, cov, Xs, rows_seen, h, sc, iters in outs:
        lo, hi = spans[r]
        assert rows_seen == hi - lo
        assert np.abs(Xs - o.X[lo:hi]).max() <= 1e-13            # centred with the global mean
        assert np.abs(cov - o.cov).max() <= 1e-12 * np.abs(o.cov).max()
        assert iters == [300, 400]
        assert np.abs(W - W_ref).max() <= 1e-9
        assert np.array_equal(W != 0, W_ref != 0)
        assert abs(h - o.h_final) <= 1e-9 and abs(sc - o.score_final) <= 1e-9
    assert np.array_equal(outs[0][1], outs[1][1]), "replicas diverged"


class _CovShardSolver:
    """CPU double of HipSolver for DagmaLinear.fit in cov mode with a row-sharded X: fit()'s
    device data preparation (gram / set_cov_gram / get_cov) on this rank's rows only, then the
    oracle's replicated cov-mode loop (no collective)."""

    def __init__(self, d, loss, mode, device=0):
        assert loss == "l2" and mode == "cov"
        self.d = d
        self.rows_seen = 0
        self.grams = 0

    def gram(self, X):
        self.rows_seen += X.shape[0]
        self.grams += 1
        return torch.from_numpy(X.T @ X)

    def set_cov_gram(self, G, n):
        self.cov = G.numpy() / n

    def get_cov(self):
        return self.cov.copy()

    def set_masks(self, mask_inc, mask_exc):
        assert mask_inc is None and mask_exc is None

    def minimize(self, W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint, want_checkpoints=False):
        from midagma_amd.solver import MinimizeResult
        from oracle.dagma_oracle import LinearOracle
        o = LinearOracle("l2")
        o.cov, o.d, o.n, o.eye = self.cov, self.d, None, np.eye(self.d)
        o.lambda1, o.checkpoint, o.inc, o.exc, o.X = lambda1, checkpoint, None, None, None
        Wn, tr = o.minimize(W, mu, max_iter, s, lr, tol, b1, b2)
        W[...] = Wn
        return MinimizeResult(iters=tr.iters, success=tr.success, status=_lib.ST_DONE if tr.success else _lib.ST_FAILED,
                              halvings=tr.halvings, early_stop=tr.early_stop, lr_final=tr.lr_final, slots=tr.iters,
                              obj_last=0.0, score_last=0.0, h_last=0.0)

    def h_value(self, W, s=1.0, grad=True):
        from oracle.dagma_oracle import h_logdet
        return h_logdet(W, s)

    def score_value(self, W):
        from oracle.dagma_oracle import score
        return score("l2", W, self.cov)


def _cov_fit_worker(rank, world, port, X_shard, n_global, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd import DagmaLinear
        m = DagmaLinear("l2", solver_factory=_CovShardSolver)
        Xs = X_shard.copy()
        W = m.fit(Xs, lambda1=0.03, T=2, warm_iter=300, max_iter=400, n_global=n_global)
        out_q.put((rank, W, m.cov, Xs, m._solver.rows_seen, m._solver.grams, m.h_final, m.score_final,
                   [e["iters"] for e in m.minimize_log], m.fit_timing["cov_on"]))
    finally:
        dist.destroy_process_group()


def test_sharded_cov_mode_fit_one_gram_allreduce(golden):
    """fit(X_shard, n_global=n) in cov mode over 2 gloo ranks (SURVEY 8e caveat):
    each rank centres with the all-reduced column sums and forms the Gram of its rows only, one
    all-reduce of the d x d sum gives every rank cov, and the replicated loop matches the oracle's
    fit of the full X to 1e-9 with no per-step collective."""
    from oracle.dagma_oracle import LinearOracle
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    n, world = X.shape[0], 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    spans = [_row_range(n, world, r) for r in range(world)]
    procs = [ctx.Process(target=_cov_fit_worker, args=(r, world, port, X[lo:hi].copy(), n, q))
             for r, (lo, hi) in enumerate(spans)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=150) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = LinearOracle("l2")
    W_ref = o.fit(X.copy(), lambda1=0.03, T=2, warm_iter=300, max_iter=400)
    for r, W, cov, Xs, rows_seen, grams, h, sc, iters, cov_on in outs:
        lo, hi = spans[r]
        assert rows_seen == hi - lo and grams == 1 and cov_on == "device"
        assert np.abs(Xs - o.X[lo:hi]).max() <= 1e-13
        assert np.abs(cov - o.cov).max() <= 1e-12 * np.abs(o.cov).max()
        assert iters == [300, 400]
        assert np.abs(W - W_ref).max() <= 1e-9
        assert abs(h - o.h_final) <= 1e-9 and abs(sc - o.score_final) <= 1e-9
    assert np.array_equal(outs[0][1], outs[1][1]), "replicas diverged"


def test_fit_gram_argument_validation():
    from midagma_amd import DagmaLinear
    X = np.random.default_rng(0).standard_normal((50, 4))
    with pytest.raises(ValueError):
        DagmaLinear("l2", solver_factory=_CovShardSolver).fit(X.copy(), gram="gpu")
    with pytest.raises(ValueError):  # a cov-mode shard needs the Gram all-reduce
        DagmaLinear("l2", solver_factory=_CovShardSolver).fit(X.copy(), n_global=100, gram="host")
