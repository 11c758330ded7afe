"""fit()'s data preparation on the device (linear.py:406-428; ABI 7, csrc/gram.hip) and the
cov-mode fit from a device-resident or row-sharded X (SURVEY 8e caveat):
the MFMA Gram against the host product, the centring against numpy, the cov-mode fit's cov
against the host X^T X / n and its first 1000 Adam steps against the oracle."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from midagma_amd import solver as hs  # noqa: E402


def _rel(a, b):
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max()))


@pytest.mark.parametrize("n,d,ld_extra", [(1, 5, 0), (257, 20, 3), (100_000, 300, 0), (300_000, 64, 7),
                                          (20_000, 1000, 0)])
@pytest.mark.parametrize("where", ["device", "host"])
def test_gram_matches_host_product(n, d, ld_extra, where):
    """G = X^T X (rows streamed in 262144-row chunks: (300000, 64) takes two, ragged last) for a
    row stride ld >= d, against numpy's product: 1e-12 of max|G|."""
    rng = np.random.default_rng(n + d)
    Xfull = rng.standard_normal((n, d + ld_extra))
    X = Xfull[:, :d]
    ref = X.T @ X
    if where == "device":
        Xt = torch.from_numpy(Xfull).cuda()[:, :d]
        G = hs.gram(Xt).cpu().numpy()
    else:
        G = hs.gram(X, 0).cpu().numpy()
    assert G.shape == (d, d)
    assert _rel(G, ref) <= 1e-12
    assert np.array_equal(G, G.T) or _rel(G, G.T) <= 1e-15


def test_gram_is_deterministic():
    X = torch.randn(123_457, 200, dtype=torch.float64, device="cuda")
    a, b = hs.gram(X), hs.gram(X)
    assert torch.equal(a, b)


def test_gram_and_set_cov_refuse_nonfinite():
    X = np.random.default_rng(0).standard_normal((1000, 30))
    X[500, 7] = np.nan
    with pytest.raises(ValueError):
        hs.gram(X, 0)
    with pytest.raises(ValueError):
        hs.gram(torch.from_numpy(X).cuda())
    s = hs.HipSolver(30, "l2", "cov", device=0)
    G = torch.zeros(30, 30, dtype=torch.float64, device="cuda")
    G[3, 4] = float("inf")
    with pytest.raises(ValueError):
        s.set_cov_gram(G, 10.0)
    s.close()


@pytest.mark.parametrize("n,d", [(1, 3), (1000, 20), (333_333, 130)])
def test_colsum_and_center_match_numpy(n, d):
    rng = np.random.default_rng(d)
    X = rng.standard_normal((n, d)) * 3 + rng.standard_normal(d) * 10
    Xt = torch.from_numpy(X).cuda()
    cs = hs.colsum_dev(Xt).cpu().numpy()
    assert _rel(cs, X.sum(axis=0)) <= 1e-12
    hs.center_dev(Xt, torch.from_numpy(cs).cuda(), float(n))
    Xc = X - X.mean(axis=0, keepdims=True)
    assert np.abs(Xt.cpu().numpy() - Xc).max() <= 1e-12 * max(1.0, np.abs(X).max())


def test_cov_mode_fit_from_device_X_d1000(parity):
    """DagmaLinear('l2').fit(X_dev) with X a device tensor (d=1000, n=1e5, GPU SEM generator):
    cov from the device centring and Gram equals the host X^T X / n to 1e-12, and the fit's first
    1000 Adam steps equal the oracle's reference algorithm on that cov to 1e-9."""
    from midagma_amd import DagmaLinear
    from midagma_amd.simulate import simulate_er_dag, simulate_weights
    from midagma_amd.utils import simulate_linear_sem_gpu
    from oracle.dagma_oracle import LinearOracle
    d, n = 1000, 100_000
    rng = np.random.default_rng(0)
    W_true = simulate_weights(simulate_er_dag(d, d, rng), rng)
    X = simulate_linear_sem_gpu(W_true, n, "gauss", seed=17, device=0)
    Xh = X.cpu().numpy()
    Xh -= Xh.mean(axis=0, keepdims=True)
    cov_h = Xh.T @ Xh / float(n)
    del Xh
    m = DagmaLinear("l2", device=0)
    W = m.fit(X, lambda1=0.03, T=1, max_iter=1000, w_threshold=0.0)
    assert m.fit_timing["cov_on"] == "device"
    assert abs(float(X.mean()) ) < 1e-12           # centred in place, as linear.py:411
    assert _rel(m.cov, cov_h) <= 1e-12
    o = LinearOracle("l2")
    o.cov, o.d, o.eye, o.lambda1, o.checkpoint, o.inc, o.exc = m.cov, d, np.eye(d), 0.03, 1000, None, None
    o.X, o.n = None, n
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 1000, 1.0, 3e-4)
    dW = float(np.abs(W - Wr).max())
    parity("config4", dW, 1e-9, "cov-mode fit from device X (n=1e5) K=1000 max|dW|")
    assert m.minimize_log[0]["iters"] == tr.iters == 1000
    assert dW <= 1e-9


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, X, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd import DagmaLinear
        from midagma_amd.linear import _row_range
        n = X.shape[0]
        lo, hi = _row_range(n, world, rank)
        Xk = torch.from_numpy(X[lo:hi].copy()).cuda()
        m = DagmaLinear("l2", device=0)
        W = m.fit(Xk, lambda1=0.03, T=2, warm_iter=400, max_iter=500, n_global=n)
        out_q.put((rank, W, m.cov, [e["iters"] for e in m.minimize_log], m.fit_timing["cov_on"]))
    finally:
        dist.destroy_process_group()


def test_sharded_cov_mode_fit_two_ranks_one_gpu():
    """fit(X_shard_dev, n_global=n) in cov mode over 2 ranks sharing cuda:0 (gloo on the device
    tensors): one all-reduce of the column sums and one of the Gram, then the replicated loop;
    equals the single-process device fit of the whole X to 1e-9, replicas bit-identical."""
    from midagma_amd import DagmaLinear
    from midagma_amd.simulate import make_dataset
    X, _, _ = make_dataset(40, 3001, seed=6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, X, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(outs[0][1], outs[1][1]), "replicas diverged"
    m = DagmaLinear("l2", device=0)
    W = m.fit(torch.from_numpy(X.copy()).cuda(), lambda1=0.03, T=2, warm_iter=400, max_iter=500)
    for _, Wk, cov, iters, cov_on in outs:
        assert cov_on == "device" and iters == [e["iters"] for e in m.minimize_log]
        assert _rel(cov, m.cov) <= 1e-12
        assert np.abs(Wk - W).max() <= 1e-9
