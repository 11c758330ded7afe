"""Experiment paths of the experiments build (`make -C midagma_amd/csrc exp`, knobs.h): rejected
or diagnostic alternatives of the product paths, checked against the oracle and the product path
so that their DESIGN.md section 8 measurements stay repeatable.  Not part of the default
`-m gpu` tier; run with

    MIDAGMA_LIB=midagma_amd/libmidagma_hip_exp.so python -m pytest -m experiment tests
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.experiment

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402


def _solver(d, cov):
    from midagma_amd.solver import HipSolver
    s = HipSolver(d, "l2", "cov", device=0)
    s.set_cov(cov)
    return s


def _oracle(X, checkpoint):
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, checkpoint)
    return o


@pytest.mark.parametrize("d", [5, 20, 32, 50, 64])
def test_small_path_vs_graph_path(d, monkeypatch):
    """The persistent kernel (small.hip) and the graph-replayed slots it replaces
    (MIDAGMA_EXP_NO_SMALL) agree to rounding: same iterations, W within 1e-11 after 500 steps
    (checkpoint every 100: Gauss-Jordan slots between runs of product-form slots)."""
    X, _, _ = make_dataset(d, max(200, 10 * d), seed=11)
    o = _oracle(X, 50)
    K = 500
    a = _solver(d, o.cov)
    Wa = np.zeros((d, d))
    ra = a.minimize(Wa, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
    monkeypatch.setenv("MIDAGMA_EXP_NO_SMALL", "1")
    b = _solver(d, o.cov)
    monkeypatch.delenv("MIDAGMA_EXP_NO_SMALL")
    Wb = np.zeros((d, d))
    rb = b.minimize(Wb, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
    assert ra.iters == rb.iters == K and ra.slots == rb.slots
    assert np.abs(Wa - Wb).max() <= 1e-11
    a.close()
    b.close()


@pytest.mark.parametrize("d", [700, 1150])
def test_blocked_lookahead_residual_experiment(monkeypatch, d):
    """The look-ahead residual (MIDAGMA_EXP_RESID_LA=1, DESIGN.md section 8: block g's launches
    prepare block g+1's R = I - (A X0 - A(g+1,G) P_g A(G,g+1) X0)) keeps the oracle's
    iterations, W and checkpoint objectives.  d=700 -> D=768 (B2=256, 3 outer blocks),
    1150 -> 1152 (B2=128, 9)."""
    monkeypatch.setenv("MIDAGMA_EXP_RESID_LA", "1")
    X, _, _ = make_dataset(d, 2 * d, seed=d + 3)
    o = _oracle(X, 40)
    K = 130
    sol = _solver(d, o.cov)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=40, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == K and res.success
    assert np.abs(W - Wr).max() <= 1e-9
    for c, (_, obj_r, _, h_r) in zip(res.checkpoints, tr.checkpoints):
        assert abs(c[1] - obj_r) <= 1e-10 * abs(obj_r) and abs(c[3] - h_r) <= 1e-9 * max(1.0, abs(h_r))


@pytest.mark.parametrize("d", [2000, 2100])
def test_cov_lookahead_bit_identical(monkeypatch, d):
    """The trailing-update look-ahead across two streams (MIDAGMA_EXP_COV_LA=1: each outer step's
    128-tile trailing update split into block g+1's bands and the rest, the series / panel chain on
    the high-priority side stream) computes every tile with the same body: W, iterations and the
    checkpoint objectives are bit-identical to the one-stream path, and match the oracle.  d=2000 ->
    D=2048 (B2=256, 8 outer blocks), 2100 -> 2176 (B2=128, 17)."""
    X, _, _ = make_dataset(d, 2 * d, seed=d + 1)
    o = _oracle(X, 4)
    K = 12
    out = {}
    for la in ("0", "1"):
        monkeypatch.setenv("MIDAGMA_EXP_COV_LA", la)
        s = _solver(d, o.cov)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=4, want_checkpoints=True)
        s.close()
        out[la] = (W, r)
    (W0, r0), (W1, r1) = out["0"], out["1"]
    assert r0.iters == r1.iters == K and np.array_equal(W0, W1)
    assert [c[1] for c in r0.checkpoints] == [c[1] for c in r1.checkpoints]
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert np.abs(W1 - Wr).max() <= 1e-9


@pytest.mark.parametrize("loss", ["l2", "logistic"])
def test_small_shard_fork_bit_identical(monkeypatch, loss):
    """Small data-mode shards (<= 16384 rows) fork the blocked inverse (fast or pivoted) beside
    the n x d GEMMs; MIDAGMA_EXP_DATA_FORK_FAST=0 runs it in sequence.  Same kernels on the same
    data: W and iterations bit-identical after 130 steps (checkpoints every 40) at d=300, n=4000."""
    from midagma_amd.solver import HipSolver
    d, n, K = 300, 4000, 130
    X, _, _ = make_dataset(d, n, seed=5)
    if loss == "logistic":
        X = (X > 0).astype(np.float64)
    out = {}
    for ff in ("0", "1"):
        monkeypatch.setenv("MIDAGMA_EXP_DATA_FORK_FAST", ff)
        s = HipSolver(d, loss, "data", device=0)
        Xc = X - X.mean(0) if loss == "l2" else X
        s.set_data(Xc, n_global=n)
        if loss == "logistic":
            s.set_cov(Xc.T @ Xc / n)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=40)
        s.close()
        out[ff] = (W, r)
    (W0, r0), (W1, r1) = out["0"], out["1"]
    assert r0.iters == r1.iters == K and np.array_equal(W0, W1)


@pytest.mark.parametrize("d", [2000, 3000])
def test_trail_series_bit_identical(monkeypatch, d):
    """Blocks 1 .. K2 - 1's product-form series inside the previous step's trailing update
    (MIDAGMA_EXP_TRAIL_SERIES = workers, gemm.hip trail_series_kernel: the same tile bodies in the
    same order) leave W, the iterations and the checkpoint objectives bit-identical to the series
    launches.  d = 2000 -> D = 2048 (8 outer blocks), 3000 -> 3072 (12); checkpoints every 10 mix
    pivoted and fast slots; 40 steps."""
    X, _, _ = make_dataset(d, d + 500, seed=3)
    Xc = X - X.mean(0)
    cov = Xc.T @ Xc / X.shape[0]
    out = {}
    for w in ("0", "64", "32"):
        monkeypatch.setenv("MIDAGMA_EXP_TRAIL_SERIES", w)
        s = _solver(d, cov)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, 40, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=10, want_checkpoints=True)
        out[w] = (W, r.iters, [c.obj for c in r.checkpoints])
        s.close()
    for w in ("64", "32"):
        assert out[w][1] == out["0"][1] == 40
        assert np.array_equal(out[w][0], out["0"][0])
        assert out[w][2] == out["0"][2]


def test_sigmoid_serial_split_score():
    """The logistic sigmoid GEMM in two serial K halves (MIDAGMA_EXP_SIG_SPLIT=1, gemm.hip: the
    first half's partial handed to the second through a per-tile flag; d = 1000, n = 1e4: 632
    tiles) against the one-pass GEMM and numpy: the score gradient within 1e-12 of max|G| and the
    loss within 1e-12 relative (the halves change the sum order of the pre-activations only)."""
    from midagma_amd.solver import HipSolver
    d, n = 1000, 10000
    rng = np.random.default_rng(3)
    X = (rng.uniform(size=(n, d)) < 0.3).astype(np.float64)
    cov = X.T @ X / n
    W = rng.normal(scale=0.02, size=(d, d))
    np.fill_diagonal(W, 0.0)
    out = {}
    for k in ("0", "1", "0b"):
        os.environ["MIDAGMA_EXP_SIG_SPLIT"] = k[0]
        try:
            s = HipSolver(d, "logistic", "data", device=0)
            s.set_cov(cov)
            s.set_data(X, n_global=n)
            s.score_partial(W)
            out[k] = s.score_finish()
            s.close()
        finally:
            os.environ.pop("MIDAGMA_EXP_SIG_SPLIT", None)
    (l0, G0), (l1, G1), (l2, G2) = out["0"], out["1"], out["0b"]
    assert l0 == l2 and np.array_equal(G0, G2)  # the one-pass path is deterministic
    scale = np.abs(G0).max()
    assert np.abs(G1 - G0).max() <= 1e-12 * scale
    assert abs(l1 - l0) <= 1e-12 * abs(l0)
    Z = X @ W
    ref_loss = (np.logaddexp(0.0, Z) - X * Z).sum() / n
    ref_G = X.T @ (1.0 / (1.0 + np.exp(-Z))) / n - cov
    assert abs(l1 - ref_loss) <= 1e-10 * abs(ref_loss)
    assert np.abs(G1 - ref_G).max() <= 1e-10 * np.abs(ref_G).max()


@pytest.mark.parametrize("d", [2000, 3000])
def test_trail_panel_bit_identical(monkeypatch, d):
    """Block g + 1's panel inside trailing update g (MIDAGMA_EXP_TRAIL_PANEL = panel workgroups,
    gemm.hip trail_panel_kernel: band tiles first, the series, then binv_panel_job's jobs claimed
    from a counter) leaves W, the iterations and the checkpoint objectives bit-identical to the
    series-inside-the-update path with the panel launches, and to the plain launches.  The series
    runs inside the update (MIDAGMA_EXP_TRAIL_SERIES=64) at these sizes only when asked;
    checkpoints every 10 mix pivoted and fast slots; 40 steps."""
    X, _, _ = make_dataset(d, d + 500, seed=11)
    Xc = X - X.mean(0)
    cov = Xc.T @ Xc / X.shape[0]
    out = {}
    for ser, pan in (("0", "0"), ("64", "0"), ("64", "128"), ("64", "512")):
        monkeypatch.setenv("MIDAGMA_EXP_TRAIL_SERIES", ser)
        monkeypatch.setenv("MIDAGMA_EXP_TRAIL_PANEL", pan)
        s = _solver(d, cov)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, 40, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=10, want_checkpoints=True)
        out[(ser, pan)] = (W, r.iters, [c.obj for c in r.checkpoints])
        s.close()
    ref = out[("0", "0")]
    for k, v in out.items():
        assert v[1] == ref[1] == 40, k
        assert np.array_equal(v[0], ref[0]), k
        assert v[2] == ref[2], k


@pytest.mark.parametrize("d", [1000, 3000])
def test_panel_single_buffered_bit_identical(monkeypatch, d):
    """The panel launch single-buffered at a fixed prefetch depth (MIDAGMA_EXP_PANEL_SB = 1, 2, 3:
    blockinv.hip binv_panel_kernel<SBPF>, the same tile arithmetic with one LDS image per operand)
    leaves W, the iterations and the checkpoint objectives bit-identical to the product's panel.
    d = 1000 (32 x 32 trailing tiles) and 3000 (the 128-tile update with the series inside);
    checkpoints every 10; 30 steps."""
    X, _, _ = make_dataset(d, d + 500, seed=5)
    Xc = X - X.mean(0)
    cov = Xc.T @ Xc / X.shape[0]
    out = {}
    for pf in ("0", "1", "2", "3"):
        monkeypatch.setenv("MIDAGMA_EXP_PANEL_SB", pf)
        s = _solver(d, cov)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, 30, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=10, want_checkpoints=True)
        out[pf] = (W, r.iters, [c.obj for c in r.checkpoints])
        s.close()
    for pf in ("1", "2", "3"):
        assert out[pf][1] == out["0"][1] == 30
        assert np.array_equal(out[pf][0], out["0"][0])
        assert out[pf][2] == out["0"][2]


@pytest.mark.parametrize("d", [8, 20, 32])
@pytest.mark.parametrize("mode", ["opt", "log"])
def test_small_path_tcc_vs_graph_path(d, mode, monkeypatch):
    """The TCC regularizer inside the persistent small loop (small.hip + tcc_blk.h, d <= 32)
    against the graph-replayed slots with the one-workgroup TCC launch (MIDAGMA_EXP_SMALL_TCC=0):
    same iterations and checkpoints; W within 1e-11 and the checkpoints' objective,
    reg_trek_value and grad_trek_norm within 1e-10 rel after 500 steps (checkpoint every 100)."""
    _small_vs_graph(d, mode, monkeypatch, [("1", "0"), ("0", "0")])


@pytest.mark.parametrize("d", [17, 20])
@pytest.mark.parametrize("mode", ["opt", "log"])
def test_small_path_tcc_bs5_vs_graph_path(d, mode, monkeypatch):
    """The one-wave 5 x 5-block TCC body in the small loop (MIDAGMA_EXP_TCC_BS5=1, d <= 20 on the
    DS = 32 kernel: 64 of its 256 threads hold the blocks) against the graph path, same bounds."""
    _small_vs_graph(d, mode, monkeypatch, [("1", "1"), ("0", "0")])


def _small_vs_graph(d, mode, monkeypatch, cases):
    X, _, _ = make_dataset(d, max(200, 10 * d), seed=7)
    o = _oracle(X, 100)
    rng = np.random.default_rng(d)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    K = 500
    runs = []
    for small, bs5 in cases:
        monkeypatch.setenv("MIDAGMA_EXP_SMALL_TCC", small)
        monkeypatch.setenv("MIDAGMA_EXP_TCC_BS5", bs5)
        s = _solver(d, o.cov)
        s.set_trek_tcc(pairs, mode=mode, weight=0.2)
        W = np.zeros((d, d))
        r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100, want_checkpoints=True)
        runs.append((W, r))
        s.close()
    (Wa, ra), (Wb, rb) = runs[0], runs[-1]
    assert ra.iters == rb.iters == K
    assert np.abs(Wa - Wb).max() <= 1e-11
    assert [c.iter for c in ra.checkpoints] == [c.iter for c in rb.checkpoints]
    for a, b in zip(ra.checkpoints, rb.checkpoints):
        assert abs(a.obj - b.obj) <= 1e-10 * abs(b.obj)
        assert abs(a.reg_trek_value - b.reg_trek_value) <= 1e-10 * abs(b.reg_trek_value) + 1e-300
        assert abs(a.grad_trek_norm - b.grad_trek_norm) <= 1e-10 * b.grad_trek_norm + 1e-300
