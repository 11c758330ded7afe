"""Every BASELINE.json config under a GPU parity test at its own size.

* config 2 (d=1000, n=1e4): W after K = 1000 and 2000 Adam steps against the oracle's run of
  the reference algorithm at one BLAS thread (tests/golden/traj_d1000.npz,
  tests/golden/make_traj_d1000.py), where the reference's own 1e-16-perturbation envelope
  is ~1e-15: the north star's 1e-5, and 1e-9 in practice;
* config 3 (d=5000, n=5e4 -> D=5120: 20 outer blocks of the two-level inverse, split-K 3 cov
  GEMM, 128-tile trailing update): _score and 8 Adam steps with checkpoints every 4 against
  the oracle (LAPACK inverse), computed on the box's cores;
* config 5 (DagmaMLP dims [200, 10, 1], n=1000): DagmaNonlinear.minimize after K = 1, 10, 100
  steps against the CPU oracle (oracle/mlp_oracle.py, pinned to the reference's own
  trajectories in tests/test_mlp_oracle.py).
Config 1 (d=20) and config 4 (d=1000, n=1e6) are covered in test_gpu_parity.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle, score  # noqa: E402


def _rel(a, b):
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max()))


@pytest.mark.parametrize("K", [1000, 2000])
def test_config2_trajectory_d1000(golden, parity, K):
    from threadpoolctl import threadpool_limits
    from midagma_amd.solver import HipSolver
    f = golden("traj_d1000.npz")
    X, _, _ = make_dataset(1000, 10000, seed=0)
    o = LinearOracle("l2")
    with threadpool_limits(limits=1):     # the fixture's cov, bit for bit
        o.prepare(X, 0.03, 1000)
    s = HipSolver(1000, "l2", "cov", device=0)
    s.set_cov(o.cov)
    W = np.zeros((1000, 1000))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000)
    s.close()
    env = float(f[f"env_K{K}"])
    dW = float(np.abs(W - f[f"W_K{K}"]).max())
    print(f"K={K}: max|W_gpu - W_ref| = {dW:.3e} (reference envelope {env:.3e})")
    parity("config2", dW, 1e-9, f"max|dW| K={K}")
    assert res.iters == K and res.success
    assert env < 1e-6                      # the horizon is inside the calibrated range
    assert dW <= 1e-5                      # north star
    assert dW <= 1e-9                      # what the kernels deliver at this horizon


def _blas_threads():
    """The box's CPU share (16 CPUs on the GPU box; os.cpu_count() shows the whole machine)."""
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:  # pragma: no cover
        return 8


@pytest.fixture(scope="module")
def cfg3():
    """BASELINE config 3's cov (d=5000, n=5e4), prepared by the oracle once for the module."""
    from threadpoolctl import threadpool_limits
    d = 5000
    X, _, _ = make_dataset(d, 50_000, seed=0)
    o = LinearOracle("l2")
    with threadpool_limits(limits=_blas_threads()):
        o.prepare(X, 0.03, 4)
    del X
    return o


def test_config3_d5000(parity, cfg3):
    from midagma_amd.solver import HipSolver
    o, d = cfg3, 5000
    s = HipSolver(d, "l2", "cov", device=0)
    assert s.D == 5120
    s.set_cov(o.cov)
    rng = np.random.default_rng(3)
    Wd = rng.normal(size=(d, d)) * 0.01
    l, G = s.score_value(Wd)
    l_ref, G_ref = score("l2", Wd, o.cov)
    assert abs(l - l_ref) <= 1e-12 * abs(l_ref)
    assert _rel(G, G_ref) <= 1e-12
    del Wd, G, G_ref
    K = 8
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=4, want_checkpoints=True)
    s.close()
    o.checkpoint = 4
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    parity("config3", float(np.abs(W - Wr).max()), 1e-9, f"max|dW| K={K}")
    assert res.iters == tr.iters == K and res.success
    assert np.abs(W - Wr).max() <= 1e-9
    assert [c[0] for c in res.checkpoints] == [c[0] for c in tr.checkpoints] == [4, 8]
    for c, (_, obj_r, sc_r, h_r) in zip(res.checkpoints, tr.checkpoints):
        assert abs(c[1] - obj_r) <= 1e-10 * abs(obj_r)
        assert abs(c[2] - sc_r) <= 1e-10 * abs(sc_r)
        assert abs(c[3] - h_r) <= 1e-9 * max(1.0, abs(h_r))


@pytest.mark.slow
def test_config3_d5000_timed_window(parity, cfg3):
    """Config 3 over the bench's whole timed window: K = 100 Adam steps with
    checkpoints every 50 against the oracle (LAPACK inverse) at the box's CPU share.  Covers the
    trailing update's in-K-loop C0 fold (EPI_SUB_MID) over ~95 fast slots at D = 5120 (20 outer
    blocks, split-3 score GEMM), the pivoted slots at steps 1, 50 and 100, and both checkpoint
    objectives."""
    from threadpoolctl import threadpool_limits
    from midagma_amd.solver import HipSolver
    o, d, K = cfg3, 5000, 100
    s = HipSolver(d, "l2", "cov", device=0)
    s.set_cov(o.cov)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    s.close()
    o.checkpoint = 50
    with threadpool_limits(limits=_blas_threads()):
        Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    dW = float(np.abs(W - Wr).max())
    print(f"config3 K={K}: max|dW| = {dW:.3e}, max|W| = {np.abs(Wr).max():.3e}")
    parity("config3", dW, 1e-9, f"max|dW| K={K}")
    assert res.iters == tr.iters == K and res.success and res.halvings == tr.halvings == 0
    assert dW <= 1e-9
    assert [c[0] for c in res.checkpoints] == [c[0] for c in tr.checkpoints] == [50, 100]
    for c, (_, obj_r, sc_r, h_r) in zip(res.checkpoints, tr.checkpoints):
        assert abs(c[1] - obj_r) <= 1e-10 * abs(obj_r)
        assert abs(c[2] - sc_r) <= 1e-10 * abs(sc_r)
        assert abs(c[3] - h_r) <= 1e-9 * max(1.0, abs(h_r))


KEYS = ["fc1.weight", "fc1.bias", "fc2.0.weight", "fc2.0.bias"]


@pytest.mark.parametrize("K", [1, 10, 100])
def test_config5_mlp_minimize_d200(parity, K):
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    from oracle.mlp_oracle import OracleMLP, load_params, nonlinear_minimize
    d, n = 200, 1000
    X, _, _ = make_dataset(d, n, seed=0)
    gen = torch.Generator().manual_seed(5)
    ref = OracleMLP([d, 10, 1])
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(torch.randn(p.shape, generator=gen, dtype=torch.float64) * 0.05)
        ref.fc1.weight.mul_(0.3 / np.sqrt(10 * d) / 0.05)
    p0 = {k: v.detach().numpy().copy() for k, v in ref.state_dict().items() if k in KEYS}
    model = DagmaMLP(dims=[d, 10, 1], bias=True).to("cuda:0")
    load_params(model, p0)
    dn = DagmaNonlinear(model, device=0)
    dn.X = torch.from_numpy(X).to("cuda:0")
    dn.checkpoint = 1000
    ok = dn.minimize(K, 2e-4, 0.02, 0.005, 0.1, 1.0)
    ok_ref, it = nonlinear_minimize(ref, torch.from_numpy(X), K, 2e-4, 0.02, 0.005, 0.1, 1.0)
    assert ok and ok_ref and it == K
    sd, rd = model.state_dict(), ref.state_dict()
    devs = {}
    for k in KEYS:
        r = rd[k].numpy()
        dev = np.abs(sd[k].cpu().numpy() - r).max()
        print(f"K={K} {k}: max|d| = {dev:.3e} (max|p| {np.abs(r).max():.3e})")
        devs[k] = dev / max(1.0, np.abs(r).max())
    parity("config5", max(devs.values()), 1e-9, f"max|dparam|/max(1,|p|) K={K}")
    for k in KEYS:
        assert devs[k] <= 1e-9, k


@pytest.mark.parametrize("graph", [True, False])
def test_config5_logdet_side_stream_bit_identical(graph, monkeypatch):
    """The MLP objective's log-det on a side stream (overlapping the tail and the backward, joined
    before the fc1 terms' backward) runs the same kernels on the same data as the one-stream
    step: after 200 Adam steps at dims [200, 10, 1] every parameter is bit-identical, in the
    graph-replayed and the eager loop."""
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    d, n = 200, 1000
    X, _, _ = make_dataset(d, n, seed=1)
    out = {}
    for overlap in (True, False):
        if overlap:
            monkeypatch.delenv("MIDAGMA_NO_OVERLAP", raising=False)
        else:
            monkeypatch.setenv("MIDAGMA_NO_OVERLAP", "1")
        torch.manual_seed(7)
        model = DagmaMLP(dims=[d, 10, 1], bias=True).to("cuda:0")
        dn = DagmaNonlinear(model, device=0, graph=graph)
        assert dn.overlap == overlap
        dn.X = torch.from_numpy(X).to("cuda:0")
        dn.checkpoint = 50
        assert dn.minimize(200, 2e-4, 0.02, 0.005, 0.1, 1.0)
        out[overlap] = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    for k in out[True]:
        assert np.array_equal(out[True][k], out[False][k]), k


@pytest.mark.parametrize("overlap", [True, False])
def test_config5_one_launch_step_bit_identical(overlap, monkeypatch):
    """The replayed step closed by one launch (midagma_mlp_step, ABI 9: the tail's dw sums, fc1's
    weight gradient, Adam over the four parameters, the next step's fc1 terms) against the separate
    launches (MIDAGMA_NO_MLP_STEP=1): after 200 Adam steps with checkpoints every 50 every
    parameter is bit-identical, with the log-det on its side stream and on one stream."""
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    d, n = 200, 1000
    X, _, _ = make_dataset(d, n, seed=2)
    if overlap:
        monkeypatch.delenv("MIDAGMA_NO_OVERLAP", raising=False)
    else:
        monkeypatch.setenv("MIDAGMA_NO_OVERLAP", "1")
    out = {}
    for one in (True, False):
        if one:
            monkeypatch.delenv("MIDAGMA_NO_MLP_STEP", raising=False)
        else:
            monkeypatch.setenv("MIDAGMA_NO_MLP_STEP", "1")
        torch.manual_seed(11)
        model = DagmaMLP(dims=[d, 10, 1], bias=True).to("cuda:0")
        with torch.no_grad():
            model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * d))
        dn = DagmaNonlinear(model, device=0)
        dn.X = torch.from_numpy(X).to("cuda:0")
        dn.checkpoint = 50
        assert dn.minimize(200, 2e-4, 0.02, 0.005, 0.1, 1.0)
        assert all(p.grad is None for p in model.parameters())
        out[one] = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    for k in out[True]:
        assert np.array_equal(out[True][k], out[False][k]), k


def test_config5_skipped_fast_objective_bit_identical(monkeypatch):
    """A fast (LdFast) step's scalar objective, which the loop never reads (nonlinear.py:214-217),
    is skipped and the Adam table's step counter it advanced is advanced by the LdFast step's end
    instead (midagma_ldfast_set_counter, ABI 10): against the objective kept on every step
    (MIDAGMA_FAST_OBJECTIVE=1), after 200 Adam steps with checkpoints every 50 every parameter is
    bit-identical."""
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    d, n = 200, 1000
    X, _, _ = make_dataset(d, n, seed=3)
    monkeypatch.delenv("MIDAGMA_NO_OVERLAP", raising=False)
    monkeypatch.delenv("MIDAGMA_NO_LDFAST", raising=False)
    out = {}
    for keep in (False, True):
        if keep:
            monkeypatch.setenv("MIDAGMA_FAST_OBJECTIVE", "1")
        else:
            monkeypatch.delenv("MIDAGMA_FAST_OBJECTIVE", raising=False)
        torch.manual_seed(13)
        model = DagmaMLP(dims=[d, 10, 1], bias=True).to("cuda:0")
        with torch.no_grad():
            model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * d))
        dn = DagmaNonlinear(model, device=0)
        dn.X = torch.from_numpy(X).to("cuda:0")
        dn.checkpoint = 50
        assert dn.minimize(200, 2e-4, 0.02, 0.005, 0.1, 1.0)
        steps, gj = dn._ld.stats()
        assert steps >= 200 and gj < steps  # the fast path ran (the skip applies to its steps)
        out[keep] = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    for k in out[True]:
        assert np.array_equal(out[True][k], out[False][k]), k


def test_config5_ldfast_path_matches_oracle(parity):
    """The h log-det's warm-started fast path (midagma_ldfast, nonlinear.LdFast): between the
    checkpoint steps (every 100 here; each runs the Gauss-Jordan chain) the product-form series
    from the last two steps' inverses, certified entrywise >= 0.  300 steps at dims [200, 10, 1]:
    the fast path carries almost every step, and every parameter stays within 1e-9 of the
    oracle's (torch CPU, slogdet) run; against the all-exact run (MIDAGMA_NO_LDFAST) to 1e-12."""
    import os
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    from oracle.mlp_oracle import OracleMLP, load_params, nonlinear_minimize
    d, n, K = 200, 1000, 300
    X, _, _ = make_dataset(d, n, seed=2)
    gen = torch.Generator().manual_seed(9)
    ref = OracleMLP([d, 10, 1])
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(torch.randn(p.shape, generator=gen, dtype=torch.float64) * 0.05)
        ref.fc1.weight.mul_(0.3 / np.sqrt(10 * d) / 0.05)
    p0 = {k: v.detach().numpy().copy() for k, v in ref.state_dict().items() if k in KEYS}
    out = {}
    for exact_only in (False, True):
        if exact_only:
            os.environ["MIDAGMA_NO_LDFAST"] = "1"
        try:
            model = DagmaMLP(dims=[d, 10, 1], bias=True).to("cuda:0")
            load_params(model, p0)
            dn = DagmaNonlinear(model, device=0)
            dn.X = torch.from_numpy(X).to("cuda:0")
            dn.checkpoint = 100
            assert dn.minimize(K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
            if not exact_only:
                steps, exact = dn._ld.stats()
                assert steps == K and exact <= 10, (steps, exact)   # 3 checkpoints + the last step
            out[exact_only] = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items() if k in KEYS}
        finally:
            os.environ.pop("MIDAGMA_NO_LDFAST", None)
    ok, it = nonlinear_minimize(ref, torch.from_numpy(X), K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1, checkpoint=100)
    assert ok and it == K
    rd = ref.state_dict()
    dev = max(np.abs(out[False][k] - rd[k].numpy()).max() / max(1.0, np.abs(rd[k].numpy()).max()) for k in KEYS)
    parity("config5", dev, 1e-9, f"max|dparam|/max(1,|p|) K={K} (fast log-det path)")
    assert dev <= 1e-9
    for k in KEYS:
        assert np.abs(out[False][k] - out[True][k]).max() <= 1e-12 * max(1.0, np.abs(out[True][k]).max()), k


def test_config5_rate_after_a_data_mode_solver():
    """Regression: a fork / join across a high-priority stream (the data-mode solver's forked
    inverse had one until round 3) left every later two-stream workload of the process ~5x
    slower: the config-5 step fell from ~7.5k to 1.3-2.2k steps/s when the MLP ran after a
    config-4 solver in one process.  In a fresh process: a data-mode solver
    (run and closed), then the bench's config-5 leg; its timed rate must stay near a fresh
    process's (healthy 6.7-7.6k across boxes, degraded 1.3-2.2k)."""
    import re
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "probe_after_data.py"), "solver_small"],
                       capture_output=True, text=True, timeout=240)
    m = re.search(r"config5 leg: (\d+) steps/s", r.stdout)
    assert r.returncode == 0 and m, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    # the rate itself is reported, not gated: a throughput floor in the correctness tier would fail
    # on a loaded box whatever the code does (the bench's config-5 leg is where the rate is judged)
    print(f"config5 leg after a data-mode solver: {m.group(1)} steps/s (healthy 6.7-8k, degraded 1.3-2.2k)")
