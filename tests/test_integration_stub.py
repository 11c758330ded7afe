"""INTEGRATION.md Option B -- the ctypes stub a maintainer would add to the reference's
dagma/linear.py -- executed as written (the library path substituted).

CPU: the stub's return-code mapping (-3 -> ValueError as scipy's check_finite, -2 ->
LinAlgError as sla.inv on a singular matrix, other codes -> RuntimeError), through the real
library (a NaN cov given to midagma_set_cov is refused before any device call).
GPU: the stub's minimize on a reference-shaped object equals midagma_amd's own solver, and a
NaN W raises ValueError (linear.py:226, sla.inv(..., check_finite=True))."""
import os
import re
import types

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_namespace():
    from midagma_amd import _lib
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"```python\n(# --- dagma/linear.py \(reference\).*?)```", text, re.S)
    assert m, "Option B block not found in INTEGRATION.md"
    code = m.group(1).replace('"/path/to/midagma_amd/libmidagma_hip.so"', repr(_lib.LIB_PATH))
    import midagma_amd._lib  # noqa: F401  (torch first, as the library's loader does)
    _lib.load()
    ns = {}
    exec(compile(code, "INTEGRATION.md[Option B]", "exec"), ns)
    return ns


def test_stub_error_mapping_cpu():
    ns = _stub_namespace()
    check = ns["_check"]
    assert check(0, None) == 0
    with pytest.raises(ValueError):
        check(-3, None)
    with pytest.raises(np.linalg.LinAlgError):
        check(-2, None)
    for rc in (-1, -4):
        with pytest.raises(RuntimeError):
            check(rc, None)
    # a real -3 from the library: midagma_set_cov refuses a NULL solver / non-finite input
    # before touching a device
    L, dp = ns["_L"], ns["_dp"]
    cov = np.full((4, 4), np.nan)
    with pytest.raises(ValueError):
        check(L.midagma_set_cov(None, cov.ctypes.data_as(dp), 4), None)


def _ref_object(cov, lambda1=0.03, checkpoint=1000):
    d = cov.shape[0]
    return types.SimpleNamespace(d=d, cov=cov, lambda1=lambda1, checkpoint=checkpoint, inc_r=None, inc_c=None,
                                 exc_r=None, exc_c=None)


@pytest.mark.gpu
def test_stub_minimize_gpu():
    pytest.importorskip("torch")
    from midagma_amd.simulate import make_dataset
    from midagma_amd.solver import HipSolver
    from oracle.dagma_oracle import LinearOracle
    ns = _stub_namespace()
    X, _, _ = make_dataset(20, 1000, seed=0)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    obj = _ref_object(o.cov)
    W = np.zeros((20, 20))
    W, ok = ns["minimize"](obj, W, 1.0, 300, 1.0, 3e-4, tol=-1.0)
    s = HipSolver(20)
    s.set_cov(o.cov)
    W2 = np.zeros((20, 20))
    s.minimize(W2, 1.0, 300, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    s.close()
    assert ok and np.array_equal(W, W2)
    # a float32 W: the stub turns on the float32 arithmetic (ABI 8), as HipSolver.set_w_float32 does
    W32 = np.zeros((20, 20), dtype=np.float32)
    W32, ok32 = ns["minimize"](obj, W32, 1.0, 300, 1.0, 3e-4, tol=-1.0)
    s = HipSolver(20)
    s.set_cov(o.cov)
    s.set_w_float32(True)
    W3 = np.zeros((20, 20))
    s.minimize(W3, 1.0, 300, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    s.close()
    assert ok32 and W32.dtype == np.float32 and np.array_equal(W32.astype(np.float64), W3)
    Wn = np.zeros((20, 20))
    Wn[3, 4] = np.nan
    with pytest.raises(ValueError):
        ns["minimize"](obj, Wn, 1.0, 10, 1.0, 3e-4)
    # the handle survives the refused call
    W3 = np.zeros((20, 20))
    W3, ok = ns["minimize"](obj, W3, 1.0, 300, 1.0, 3e-4, tol=-1.0)
    assert ok and np.array_equal(W3, W2)
