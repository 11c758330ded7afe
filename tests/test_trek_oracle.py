"""The PST trek-regularizer oracle (oracle/trek_oracle.py) against fixtures from the reference's
own `notreks.trek_value_grad` (tests/golden/trek_pst.npz).  CPU only."""
import numpy as np
import pytest

from oracle.trek_oracle import pst_value_grad


@pytest.mark.parametrize("d", [8, 20])
@pytest.mark.parametrize("seq", ["exp", "inv", "log", "binom"])
@pytest.mark.parametrize("agg", ["mean", "sum", "max", "lse"])
def test_pst_oracle_matches_reference(golden, d, seq, agg):
    f = golden("trek_pst.npz")
    W, pairs = f[f"W_d{d}"], f[f"pairs_d{d}"]
    v, g = pst_value_grad(W, pairs, seq, K_log=12 if seq == "log" else None, agg=agg)
    v_ref, g_ref = float(f[f"val_{seq}_{agg}_d{d}"]), f[f"grad_{seq}_{agg}_d{d}"]
    assert abs(v - v_ref) <= 1e-13 * max(1.0, abs(v_ref))
    assert np.abs(g - g_ref).max() <= 1e-12 * max(1.0, np.abs(g_ref).max())


def test_pst_empty_pairs():
    v, g = pst_value_grad(np.ones((3, 3)) * 0.1, np.zeros((0, 2), dtype=np.int64))
    assert v == 0.0 and not g.any()


# --- TCC (tests/golden/trek_tcc.npz: the reference's trek_value_grad and minimize) -----------

@pytest.mark.parametrize("d", [8, 20])
@pytest.mark.parametrize("case", ["dense", "tiny", "dag"])
@pytest.mark.parametrize("w", [1.0, 2.0])
def test_tcc_oracle_matches_reference(golden, d, case, w):
    from oracle.trek_oracle import tcc_value_grad
    f = golden("trek_tcc.npz")
    W, pairs = f[f"W_{case}_d{d}"], f[f"pairs_d{d}"]
    v, g = tcc_value_grad(W, pairs, w=w)
    v_ref, g_ref = float(f[f"val_{case}_w{w:g}_d{d}"]), f[f"grad_{case}_w{w:g}_d{d}"]
    assert abs(v - v_ref) <= 1e-13 * abs(v_ref)
    assert np.abs(g - g_ref).max() <= 1e-13 * np.abs(g_ref).max()


def test_tcc_empty_pairs():
    from oracle.trek_oracle import tcc_value_grad
    v, g = tcc_value_grad(np.ones((3, 3)) * 0.1, np.zeros((0, 2), dtype=np.int64))
    assert v == 0.0 and not g.any()


@pytest.mark.parametrize("mode", ["opt", "log"])
@pytest.mark.parametrize("K", [1, 10, 90])
def test_tcc_minimize_oracle_matches_reference(golden, mode, K):
    """The loop with TCC (linear.py:251-258): the oracle's W against the reference's W."""
    from oracle.dagma_oracle import LinearOracle
    f = golden("trek_tcc.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"]
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 40)
    o.trek = dict(kind="tcc", pairs=f["pairs_d20"], mode=mode, weight=0.2)
    W, tr = o.minimize(np.zeros((20, 20)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert tr.iters == int(f[f"traj_{mode}_it_K{K}"])
    assert np.abs(W - f[f"traj_{mode}_W_K{K}"]).max() <= 1e-12
