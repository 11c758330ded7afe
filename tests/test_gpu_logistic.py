"""GPU parity of the logistic score path (reference linear.py:245-246, 89-92) on both forms of
the sigmoid GEMM (csrc/gemm.hip):

- the one-pass 128-tile kernel (`gemm_pipe_kernel<*, B_PLAIN, EPI_SIGMOID>`), which the size rule
  picks for every grid of >= 2048 tiles (n = 1e6, and every logistic shard of that size) and for
  grids whose last round of 512 resident tiles is full;
- the serial K split (`EPI_SIGMOID_SPLIT`), the size rule's choice for small grids (d = 1000,
  n = 1e4), whose per-tile hand-off must stay paired when the inverse forked beside the GEMM
  hands its slot back mid-launch (ST_NEED_GJ).

Tolerances: the score (loss and gradient) against numpy to 1e-10 relative; trajectories with
binary X against the reference algorithm (the CPU oracle) within 2x the reference's own
summation-order envelope (the 64-row blocked oracle), as in test_gpu_parity's d = 100 case;
trajectories with continuous X and lambda1 = 0 (no L1 kink, so no chaotic entries) to 1e-9.
"""
import numpy as np
import pytest
from scipy.special import expit

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle.dagma_oracle import LinearOracle, score  # noqa: E402


@pytest.fixture(scope="module")
def hip():
    from midagma_amd import _lib
    from midagma_amd.solver import device_count
    _lib.load()
    assert device_count() >= 1, "no ROCm device visible"
    return _lib


class _BlockedOracle(LinearOracle):
    """The oracle with X^T sigmoid(XW) summed in row blocks (64 rows; 1024 at n > 65536, where
    64-row products would take minutes): a summation order as valid as OpenBLAS's, which
    measures the reference's own order sensitivity."""

    def score_grad(self, W, mu):
        S = expit(self.X @ W)
        Z = np.zeros((self.d, self.d))
        blk = 64 if self.n <= 65536 else 1024
        for b in range(0, self.n, blk):
            Z += self.X[b:b + blk].T @ S[b:b + blk]
        return (mu / self.n) * Z - mu * self.cov


def _logistic_solver(X, form=None):
    from midagma_amd.solver import HipSolver
    n, d = X.shape
    s = HipSolver(d, "logistic", "data", device=0)
    if form is not None:
        s.debug_sig_split(form)
    s.set_cov(X.T @ X / n)
    s.set_data(X, n_global=n)
    return s


def _binary(n, d, seed, p=0.3):
    rng = np.random.default_rng(seed)
    return (rng.uniform(size=(n, d)) < p).astype(np.float64)


def _check_score(sol, X, W):
    n = X.shape[0]
    sol.score_partial(W)
    loss, G = sol.score_finish()
    Z = X @ W
    ref_loss = (np.logaddexp(0.0, Z) - X * Z).sum() / n
    ref_G = X.T @ expit(Z) / n - X.T @ X / n
    assert abs(loss - ref_loss) <= 1e-10 * abs(ref_loss)
    assert np.abs(G - ref_G).max() <= 1e-10 * np.abs(ref_G).max()
    return loss, G


def _envelope_bound(W, X, K, lam, lr=3e-4):
    """W after K GPU steps against the oracle's K steps (the reference algorithm), within 2x
    the reference's own summation-order envelope."""
    d = X.shape[1]
    o = LinearOracle("logistic")
    o.prepare(X.copy(), lam, 1000)
    ref, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, lr, tol=-1.0)
    assert tr.iters == K
    ob = _BlockedOracle("logistic")
    ob.prepare(X.copy(), lam, 1000)
    Wb, _ = ob.minimize(np.zeros((d, d)), 1.0, K, 1.0, lr, tol=-1.0)
    env = np.abs(Wb - ref)
    diff = np.abs(W - ref)
    assert diff.max() <= max(1e-9, 2 * env.max()), (diff.max(), env.max())
    assert (diff > 1e-9).sum() <= 1.5 * (env > 1e-9).sum() + 10
    l_gpu, _ = score("logistic", W, o.cov, o.X)
    l_ref, _ = score("logistic", ref, o.cov, o.X)
    l_blk, _ = score("logistic", Wb, o.cov, o.X)
    assert abs(l_gpu - l_ref) <= max(1e-12 * abs(l_ref), 2 * abs(l_blk - l_ref))
    return float(diff.max()), float(env.max())


@pytest.mark.parametrize("d,n", [(1000, 262144), (100, 65536)])
def test_sigmoid_one_pass_kernel(hip, d, n):
    """The one-pass sigmoid GEMM: d = 1000, n = 262144 (2048 x 8 = 16384 tiles, the n = 1e6
    leg's kernel and grid shape class) and d = 100, n = 65536 (D = 128, 512 tiles: a full last
    round).  The size rule must pick the one-pass form; the score against numpy; 5 Adam steps
    from W = 0 against the reference algorithm."""
    X = _binary(n, d, seed=d)
    sol = _logistic_solver(X)
    assert sol.debug_sig_split() == 1  # the one-pass kernel, not the serial split
    rng = np.random.default_rng(1)
    W = rng.normal(scale=0.02, size=(d, d))
    np.fill_diagonal(W, 0.0)
    _check_score(sol, X, W)
    K = 5
    Wg = np.zeros((d, d))
    res = sol.minimize(Wg, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.05)
    sol.close()
    assert res.success and res.iters == K
    _envelope_bound(Wg, X, K, 0.05)


def test_sigmoid_split_kernel_score(hip):
    """The serial K split at d = 1000, n = 1e4 (79 x 8 = 632 tiles: the size rule's split case),
    forced off and on through the test hook: both forms against numpy, and against each other
    within 1e-12 of max|G| (the halves change the sum order of the pre-activations only)."""
    X = _binary(10000, 1000, seed=3)
    rng = np.random.default_rng(4)
    W = rng.normal(scale=0.02, size=(1000, 1000))
    np.fill_diagonal(W, 0.0)
    out = {}
    for form in (1, 2, 0):
        sol = _logistic_solver(X, form)
        out[form] = (sol.debug_sig_split(),) + _check_score(sol, X, W)
        sol.close()
    assert out[1][0] == 1 and out[2][0] == 2 and out[0][0] == 2  # the rule splits this grid
    scale = np.abs(out[1][2]).max()
    assert np.abs(out[2][2] - out[1][2]).max() <= 1e-12 * scale
    assert abs(out[2][1] - out[1][1]) <= 1e-12 * abs(out[1][1])


@pytest.mark.parametrize("form", [2, 1])
def test_sigmoid_forms_through_forced_handbacks(hip, form):
    """the split GEMM's per-tile hand-off over a multi-slot minimize in which the
    fast inverse, forked beside the GEMMs, hands slots back mid-launch.  After every 10 slots the
    stored warm starts are zeroed (test hook), so the next fast slot's first product-form pass
    sets ST_NEED_GJ while the sigmoid GEMM runs; a flag left set by such a launch would make a
    later launch add a stale partial.  Continuous X and lambda1 = 0 keep the trajectory free of
    L1-kink chaos, so both forms must match the reference algorithm's 200 steps to 1e-9, with
    every hand-back re-run (iterations equal); lr = 1e-4 keeps W inside the domain (|W| <= 0.02)."""
    d, n, K = 1000, 10000, 200
    rng = np.random.default_rng(7)
    X = rng.normal(size=(n, d)) * 0.5
    sol = _logistic_solver(X, form)
    assert sol.debug_sig_split() == form
    W = np.zeros((d, d))
    sol.begin(W, 1.0, K, 1.0, 1e-4, tol=-1.0, lambda1=0.0, checkpoint=50)
    for _ in range(200):
        sol.run_slots(10)
        r = sol.poll()
        if r.status != 0:
            break
        sol.debug_spoil_warm()
    res = sol.end(W)
    hb = sol.debug_handbacks()
    sol.close()
    assert res.iters == K and res.success
    assert hb >= 10, hb  # the hook really forced hand-backs
    o = LinearOracle("logistic")
    o.prepare(X.copy(), 0.0, 50)
    ref, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 1e-4, tol=-1.0)
    assert tr.iters == K
    assert np.abs(W - ref).max() <= 1e-9
    assert abs(res.obj_last - tr.checkpoints[-1][1]) <= 1e-10 * abs(tr.checkpoints[-1][1])
