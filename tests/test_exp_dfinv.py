"""The one-launch (dataflow) blocked inverse of the cov-mode fast slot (experiments/dfinv.hip, an
experiment enabled by MIDAGMA_EXP_DF=1: measured slower) against
the launch-per-phase blocked inverse it replaces (csrc/blockinv.hip, MIDAGMA_EXP_DF=0) and the
oracle: the same tile products in the same order, so W, the iteration counts and the
checkpoint records are bit-identical; both match the oracle (LAPACK inverse) to 1e-9.
linear.py:224-332 (the loop), :226 (the inverse)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.experiment

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402


@pytest.fixture(scope="module")
def hip():
    from midagma_amd import _lib
    from midagma_amd.solver import device_count
    _lib.load()
    assert device_count() >= 1, "no ROCm device visible"
    return _lib


@pytest.fixture(autouse=True)
def _no_lookahead(monkeypatch):
    """The one-launch inverse repeats the per-block residual launch's arithmetic; the
    launch-per-phase path it is compared with bit for bit runs that form too
    (MIDAGMA_EXP_RESID_LA=0; the default look-ahead residual rounds differently)."""
    monkeypatch.setenv("MIDAGMA_EXP_RESID_LA", "0")


def _solver(d, cov, df):
    from midagma_amd.solver import HipSolver
    old = os.environ.get("MIDAGMA_EXP_DF")
    os.environ["MIDAGMA_EXP_DF"] = "1" if df else "0"
    try:
        s = HipSolver(d, "l2", "cov", device=0)
    finally:
        if old is None:
            del os.environ["MIDAGMA_EXP_DF"]
        else:
            os.environ["MIDAGMA_EXP_DF"] = old
    s.set_cov(cov)
    return s


def _run(d, cov, df, K, lr, ck):
    s = _solver(d, cov, df)
    W = np.zeros((d, d))
    res = s.minimize(W, 1.0, K, 1.0, lr, tol=-1.0, lambda1=0.03, checkpoint=ck, want_checkpoints=True)
    s.close()
    return W, res


@pytest.mark.parametrize("d", [700, 1000])
def test_df_inverse_bit_identical_to_launch_per_phase(hip, d):
    """d=700 -> D=768 (3 outer blocks), 1000 -> 1024 (4).  (D = 512 runs one 512-wide block,
    which the one-launch inverse does not take; 1408 is not a multiple of 256.)"""
    X, _, _ = make_dataset(d, 2 * d, seed=d + 1)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    K, ck = 130, 40
    W1, r1 = _run(d, o.cov, True, K, 3e-4, ck)
    W0, r0 = _run(d, o.cov, False, K, 3e-4, ck)
    assert r1.iters == r0.iters == K and r1.success and r0.success
    assert np.array_equal(W1, W0), float(np.abs(W1 - W0).max())
    # every CkptRec field but `elapsed` (wall clock, index 15)
    strip = lambda cs: [tuple(c[:15]) + tuple(c[16:]) for c in cs]  # noqa: E731
    assert strip(r1.checkpoints) == strip(r0.checkpoints)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert tr.iters == K
    assert np.abs(W1 - Wr).max() <= 1e-9


def test_df_inverse_line_search(hip):
    """lr large enough that the domain line search halves (linear.py:230-241): the fast slot's
    domain flags come from the one-launch inverse's last outer step; halvings, lr and W match
    the launch-per-phase path bit for bit and the oracle to 1e-8."""
    d = 700
    X, _, _ = make_dataset(d, 2 * d, seed=11)
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 1000)
    o.checkpoint = 20
    W1, r1 = _run(d, o.cov, True, 60, 0.3, 20)
    W0, r0 = _run(d, o.cov, False, 60, 0.3, 20)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 60, 1.0, 0.3, tol=-1.0)
    assert (r1.iters, r1.success, r1.halvings, r1.lr_final) == (r0.iters, r0.success, r0.halvings, r0.lr_final)
    assert (r1.iters, r1.success, r1.halvings) == (tr.iters, tr.success, tr.halvings)
    assert np.array_equal(W1, W0)
    assert np.abs(W1 - Wr).max() <= 1e-8
