"""Edge sizes of the GPU inner loop against the oracle: tiny d (1, 2, 3), the padding and
path boundaries (D = round_up(d, 64) up to 192, round_up(d, 128) above; the two-level
blocked inverse from D >= 256 with B2 = 256 or 128), and data mode with a row count that is
not a multiple of the 128-row GEMM tile."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402


def _case(d, n, seed=3):
    if d <= 3:
        rng = np.random.default_rng(seed)
        X = rng.standard_normal((n, d))
        if d > 1:
            X[:, 1] += 0.8 * X[:, 0]
        return X
    X, _, _ = make_dataset(d, n, seed=seed)
    return X


@pytest.mark.parametrize("d", [1, 2, 3, 63, 65, 191, 192, 193, 255, 257, 384])
def test_cov_minimize_edge_sizes(d):
    from midagma_amd.solver import HipSolver
    X = _case(d, max(60, 2 * d + 10))
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 10)
    K = 45
    s = HipSolver(d, "l2", "cov", device=0)
    s.set_cov(o.cov)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=10, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == K
    assert np.abs(W - Wr).max() <= 1e-9
    assert [c.iter for c in res.checkpoints] == [r["iter"] for r in tr.records]
    for c, r in zip(res.checkpoints, tr.records):
        assert abs(c.obj - r["obj_total"]) <= 1e-10 * abs(r["obj_total"]) + 1e-14
    s.close()


@pytest.mark.parametrize("d,n", [(2, 77), (20, 1001), (130, 300)])
def test_data_mode_ragged_rows(d, n):
    """Data mode with n not a multiple of 128: the padded rows are zero and drop out."""
    from midagma_amd.solver import HipSolver
    X = _case(d, n)
    X = X - X.mean(axis=0, keepdims=True)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 10)
    s = HipSolver(d, "l2", "data", device=0)
    s.set_data(X, n_global=n)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, 30, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=10)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 30, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters
    assert np.abs(W - Wr).max() <= 1e-9
    s.close()


def test_dagma_linear_fit_tiny():
    from midagma_amd import DagmaLinear
    X = _case(2, 200)
    W = DagmaLinear("l2").fit(X, lambda1=0.02, T=2, warm_iter=500, max_iter=800)
    assert W.shape == (2, 2) and np.isfinite(W).all() and W[0, 0] == 0 and W[1, 1] == 0


def test_nonfinite_inputs_raise_value_error():
    """scipy's check_finite (linear.py:226): non-finite W / cov / X -> ValueError."""
    from midagma_amd.solver import HipSolver
    X = _case(6, 80)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 10)
    s = HipSolver(6, "l2", "cov", device=0)
    bad = o.cov.copy()
    bad[1, 2] = np.inf
    with pytest.raises(ValueError):
        s.set_cov(bad)
    s.set_cov(o.cov)
    W = np.zeros((6, 6))
    W[0, 4] = np.nan
    with pytest.raises(ValueError):
        s.minimize(W, 1.0, 5, 1.0, 3e-4, lambda1=0.03)
    with pytest.raises(ValueError):
        s.h_value(W, 1.0)
    s.close()
    sd = HipSolver(6, "l2", "data", device=0)
    Xb = X - X.mean(axis=0, keepdims=True)
    Xb[7, 3] = np.nan
    with pytest.raises(ValueError):
        sd.set_data(Xb, n_global=80)
    with pytest.raises(ValueError):
        sd.set_data(torch.from_numpy(Xb).cuda(), n_global=80)   # device-pointer path
    sd.close()


def test_singular_vs_nonfinite_during_minimize():
    """A finite singular sI - W o W -> LinAlgError (LAPACK getrf info > 0); W that turns
    non-finite inside the loop (non-finite data) -> ValueError, as sla.inv's check_finite."""
    from midagma_amd.solver import HipSolver
    X = _case(2, 60)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 10)
    s = HipSolver(2, "l2", "cov", device=0)
    s.set_cov(o.cov)
    W = np.array([[0.0, 1.0], [1.0, 0.0]])
    with pytest.raises(np.linalg.LinAlgError):
        s.minimize(W, 1.0, 5, 1.0, 3e-4, lambda1=0.03)
    s.close()
    # data mode with a huge entry: G overflows to inf, Adam makes W nan after step 1
    Xh = X - X.mean(axis=0, keepdims=True)
    Xh[3, 0] = 1e200
    sd = HipSolver(2, "l2", "data", device=0)
    sd.set_data(Xh, n_global=60)
    W = np.zeros((2, 2))
    with pytest.raises(ValueError):
        sd.minimize(W, 1.0, 5, 1.0, 3e-4, lambda1=0.03)
    sd.close()


def test_ldfast_enqueue_refuses_a_different_d():
    """A warm-started log-det handle is sized for its d (ring, work buffers): an A of another d
    is refused with ValueError instead of being read out of bounds (ABI 7)."""
    import ctypes as C
    import torch
    from midagma_amd import _lib
    L = _lib.load()
    h = C.c_void_p()
    _lib.check(L.midagma_ldfast_create(C.byref(h), 50), None, "ldfast_create")
    try:
        A = torch.zeros(60, 60, dtype=torch.float64, device="cuda:0")
        hd = torch.zeros((), dtype=torch.float64, device="cuda:0")
        Mt = torch.zeros(60, 60, dtype=torch.float64, device="cuda:0")
        rc = L.midagma_ldfast_enqueue(h, C.c_void_p(A.data_ptr()), 60, 60, 1.0, C.c_void_p(hd.data_ptr()),
                                      C.c_void_p(Mt.data_ptr()), 60, None, 1, -1)
        assert rc == _lib.E_ARG
        with pytest.raises(ValueError):
            _lib.check(rc, None, "ldfast_enqueue")
    finally:
        L.midagma_ldfast_destroy(h)


def test_ldfast_gate_open_fallback_equals_chain():
    """A warm-started log-det step whose certificate fails (A jumps far from the warm start) opens
    the device gate and runs the one-workgroup Gauss-Jordan fallback (gj_inverse_1wg_kernel): its
    h and (sI - A)^-T equal the launch-per-step chain's of an exact step bit for bit; a closed gate
    leaves the fast inverse, within 1e-12 of the exact one, and the last exact h."""
    import ctypes as C
    import torch
    from midagma_amd import _lib
    L = _lib.load()
    d = 200
    rng = np.random.default_rng(4)
    A1 = rng.uniform(0.0, 0.5 / d, size=(d, d))
    A2 = rng.uniform(0.0, 1.2 / d, size=(d, d))  # far from A1 (rho(R) ~ 0.5): the series hands back
    dev = "cuda:0"
    f64 = dict(dtype=torch.float64, device=dev)

    def vp(t):
        return C.c_void_p(t.data_ptr())

    def new():
        h = C.c_void_p()
        _lib.check(L.midagma_ldfast_create(C.byref(h), d), None, "ldfast_create")
        return h

    def step(h, A, exact):
        At = torch.from_numpy(A).to(dev)
        hv, Mt = torch.zeros((), **f64), torch.zeros(d, d, **f64)
        _lib.check(L.midagma_ldfast_enqueue(h, vp(At), d, d, 1.0, vp(hv), vp(Mt), d, None, 1 if exact else 0, -1),
                   None, "ldfast_enqueue")
        torch.cuda.synchronize()
        return float(hv.item()), Mt.cpu().numpy()

    h = new()
    try:
        h0, _ = step(h, A1, True)
        step(h, A1 * (1 + 1e-6), False)          # converges: the gate stays closed
        h_fast, M_fast = step(h, A1 * (1 + 2e-6), False)
        a, b = C.c_int64(), C.c_int64()
        _lib.check(L.midagma_ldfast_stats(h, C.byref(a), C.byref(b)), None, "ldfast_stats")
        exact_before = b.value
        h_open, M_open = step(h, A2, False)      # the certificate fails: the fallback runs
        _lib.check(L.midagma_ldfast_stats(h, C.byref(a), C.byref(b)), None, "ldfast_stats")
        assert b.value == exact_before + 1, (exact_before, b.value)
    finally:
        L.midagma_ldfast_destroy(h)
    ref = new()
    try:
        h_ex, M_ex = step(ref, A2, True)
        h_ex1, M_ex1 = step(ref, A1 * (1 + 2e-6), True)
    finally:
        L.midagma_ldfast_destroy(ref)
    assert h_open == h_ex and np.array_equal(M_open, M_ex)
    assert h_fast == h0                          # a certified fast step keeps the last exact h
    assert np.abs(M_fast - M_ex1).max() <= 1e-12 * np.abs(M_ex1).max()


@pytest.mark.gpu
def test_ldfast_counter_advanced_by_fast_steps_only():
    """midagma_ldfast_set_counter (ABI 10): every fast step enqueued while a counter is set adds 1
    to it in its end launch, whether its gate stayed shut or opened; exact steps, and fast steps
    after set_counter(NULL), leave it alone (DagmaNonlinear's skipped objective keeps only this
    side effect, nonlinear.py:214-217)."""
    import ctypes as C
    import torch
    from midagma_amd import _lib
    L = _lib.load()
    d = 200
    rng = np.random.default_rng(5)
    A1 = rng.uniform(0.0, 0.5 / d, size=(d, d))
    A2 = rng.uniform(0.0, 1.2 / d, size=(d, d))  # far: the certificate fails, the gate opens
    dev = "cuda:0"
    f64 = dict(dtype=torch.float64, device=dev)
    ctr = torch.full((1,), 7, dtype=torch.int64, device=dev)
    h = C.c_void_p()
    _lib.check(L.midagma_ldfast_create(C.byref(h), d), None, "ldfast_create")

    def step(A, exact):
        At = torch.from_numpy(A).to(dev)
        hv, Mt = torch.zeros((), **f64), torch.zeros(d, d, **f64)
        _lib.check(L.midagma_ldfast_enqueue(h, C.c_void_p(At.data_ptr()), d, d, 1.0, C.c_void_p(hv.data_ptr()),
                                            C.c_void_p(Mt.data_ptr()), d, None, 1 if exact else 0, -1),
                   None, "ldfast_enqueue")
        torch.cuda.synchronize()
        return int(ctr.item())

    try:
        _lib.check(L.midagma_ldfast_set_counter(h, C.c_void_p(ctr.data_ptr())), None, "ldfast_set_counter")
        assert step(A1, True) == 7                    # exact: its objective advances the counter
        assert step(A1 * (1 + 1e-6), False) == 8      # fast, gate shut
        assert step(A1 * (1 + 2e-6), False) == 9
        assert step(A2, False) == 10                  # fast, gate opened (the chain ran)
        _lib.check(L.midagma_ldfast_set_counter(h, None), None, "ldfast_set_counter")
        assert step(A2 * (1 + 1e-6), False) == 10
        a, b = C.c_int64(), C.c_int64()
        _lib.check(L.midagma_ldfast_stats(h, C.byref(a), C.byref(b)), None, "ldfast_stats")
        assert a.value == 5
    finally:
        L.midagma_ldfast_destroy(h)
