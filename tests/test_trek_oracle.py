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
