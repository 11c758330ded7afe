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
