"""dtype=np.float32 (linear.py:29) through DagmaLinear.fit on the CPU: the product's Python path
(the solver told W is float32 before every minimize call, W handed back in the caller's type)
over a CPU double of the solver that runs the oracle's float32 loop with the GPU's inverse model
(a float64 inverse rounded to float32, LinearOracle(inv64=True)), against the reference's own
float32 fit (tests/golden/fit_f32_d20.npz) and its float32 perturbation envelope
(fit_f32_d20_envelope.npz).  The GPU form of this check is
tests/test_gpu_parity.py::test_full_fit_float32_dtype."""
import numpy as np

from midagma_amd import _lib


class _HostCovSolver:
    """CPU double of HipSolver for a cov-mode fit with the host product X^T X / n."""

    def __init__(self, d, loss, mode, device=0):
        assert loss == "l2" and mode == "cov"
        self.d = d
        self.w32 = False

    def set_w_float32(self, on):
        self.w32 = bool(on)

    def set_cov(self, cov):
        self.cov = np.array(cov, dtype=np.float64)

    def set_masks(self, mask_inc, mask_exc):
        assert mask_inc is None and mask_exc is None

    def minimize(self, W, mu, max_iter, s, lr, tol, b1, b2, lambda1, checkpoint, want_checkpoints=False):
        from midagma_amd.solver import MinimizeResult
        from oracle.dagma_oracle import LinearOracle
        assert W.dtype == np.float64  # the ABI passes float64 (holding float32 values in a float32 fit)
        dt = np.float32 if self.w32 else np.float64
        o = LinearOracle("l2", dtype=dt, inv64=True)
        o.cov, o.d, o.n, o.eye = self.cov, self.d, None, np.eye(self.d).astype(dt)
        o.lambda1, o.checkpoint, o.inc, o.exc, o.X = lambda1, checkpoint, None, None, None
        Wn, tr = o.minimize(W.astype(dt), mu, max_iter, s, lr, tol, b1, b2)
        W[...] = Wn
        return MinimizeResult(iters=tr.iters, success=tr.success, status=_lib.ST_DONE if tr.success else _lib.ST_FAILED,
                              halvings=tr.halvings, early_stop=tr.early_stop, lr_final=tr.lr_final, slots=tr.iters,
                              obj_last=0.0, score_last=0.0, h_last=0.0)

    def h_value(self, W, s=1.0, grad=True):
        from oracle.dagma_oracle import h_logdet
        return h_logdet(np.asarray(W, dtype=np.float64), s)

    def score_value(self, W):
        from oracle.dagma_oracle import score
        return score("l2", np.asarray(W, dtype=np.float64), self.cov)


def test_float32_fit_matches_reference_float32_fit(golden):
    from midagma_amd import DagmaLinear
    f = golden("fit_f32_d20.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2", dtype=np.float32, solver_factory=_HostCovSolver)
    W = m.fit(X, lambda1=0.03, T=3, s=[1.0, .9, .8], warm_iter=4000, max_iter=5000, gram="host")
    assert W.dtype == np.float32
    env = golden("fit_f32_d20_envelope.npz")
    env_w = float(np.abs(env["W"] - f["W_f32"]).max())
    assert np.array_equal(W != 0, f["W_f32"] != 0)
    assert np.abs(W - f["W_f32"]).max() <= env_w


def test_float32_default_fit_stage_counts(golden):
    """The default float32 fit through the product's Python path over the CPU double (the GPU's
    inverse model; the float32 checkpoint objective as numpy computes it): each stage's successful
    call stops inside the range of the reference's float32 fit and its float32-noise replicas
    (fit_f32_d20_default.npz)."""
    from midagma_amd import DagmaLinear
    f = golden("fit_f32_d20_default.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2", dtype=np.float32, solver_factory=_HostCovSolver)
    m.fit(X, lambda1=0.03, gram="host")
    ok = [e["iters"] for e in m.minimize_log if e["success"]]
    ref = [int(c[5]) for c in f["calls"] if c[4] == 1]
    env = f["env_stage_iters"]
    assert len(ok) == 5
    # stages 1-3 (mu = 1, 0.1, 0.01); at mu = 1e-3 the reference's own float32 getri leaves
    # negative entries in inv(sI - W o W), so its unperturbed fit goes out of domain and retries
    # up to s = 1 (its float32-noise replicas do not): a float32 LAPACK artifact the float64
    # inverse rounded to float32 does not have
    for i, it in enumerate(ok[:3]):
        assert min(ref[i], env[:, i].min()) <= it <= max(ref[i], env[:, i].max()), (i, ok)
