"""Error mapping of the boundary: what the reference raises, and that the ctypes
layer maps the C ABI's codes onto the same exception types.  CPU tier: no device calls.

The reference reaches LAPACK through scipy.linalg.inv(s*I - W*W) (linear.py:226) with
check_finite=True: a non-finite W raises ValueError, a finite singular matrix LinAlgError."""
import numpy as np
import pytest

from oracle.dagma_oracle import LinearOracle


def _oracle(d=6):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((50, d))
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 1000)
    return o


def test_reference_nonfinite_W_is_value_error():
    o = _oracle()
    W = np.zeros((6, 6))
    W[2, 3] = np.nan
    with pytest.raises(ValueError):
        o.minimize(W, 1.0, 5, 1.0, 3e-4)
    W[2, 3] = np.inf
    with pytest.raises(ValueError):
        o.minimize(W, 1.0, 5, 1.0, 3e-4)


def test_reference_singular_is_linalg_error():
    o = _oracle(2)
    W = np.array([[0.0, 1.0], [1.0, 0.0]])  # s I - W o W = [[1, -1], [-1, 1]]
    with pytest.raises(np.linalg.LinAlgError):
        o.minimize(W, 1.0, 5, 1.0, 3e-4)


def test_abi_codes_map_to_reference_exceptions(monkeypatch):
    from midagma_amd import _lib
    monkeypatch.setattr(_lib, "last_error", lambda handle=None: "msg")
    with pytest.raises(ValueError):
        _lib.check(_lib.E_ARG, None, "x")
    with pytest.raises(np.linalg.LinAlgError):
        _lib.check(_lib.E_SINGULAR, None, "x")
    with pytest.raises(_lib.HipSolverError):
        _lib.check(_lib.E_HIP, None, "x")
    assert _lib.check(0) == 0


def test_dtype_choices():
    """dtype (linear.py:29): float64 and float32 are accepted (the loop computes in float64, W is
    handed back in dtype); anything else is refused at construction, before any device call."""
    from midagma_amd import DagmaLinear
    assert DagmaLinear("l2", dtype=np.float32).dtype is np.float32
    assert DagmaLinear("l2", dtype=np.dtype("float64")).dtype is np.float64
    for bad in (np.float16, np.int64):
        with pytest.raises(ValueError):
            DagmaLinear("l2", dtype=bad)
