"""The nonlinear oracle (oracle/mlp_oracle.py) against the reference's own DagmaNonlinear
trajectories (tests/golden/mlp_traj.npz).  CPU only."""
import numpy as np
import pytest
import torch

from oracle.mlp_oracle import OracleMLP, load_params, nonlinear_fit, nonlinear_minimize

KEYS = ["fc1.weight", "fc1.bias", "fc2.0.weight", "fc2.0.bias"]


def _model(f):
    m = OracleMLP([20, 10, 1])
    load_params(m, {k: f[f"p0_{k}"] for k in KEYS})
    return m


@pytest.mark.parametrize("K", [1, 10, 100])
def test_nonlinear_minimize_oracle_matches_reference(golden, K):
    f = golden("mlp_traj.npz")
    X = torch.from_numpy(golden("data_d20_n1000_seed0.npz")["X"])
    m = _model(f)
    ok, _ = nonlinear_minimize(m, X, K, 2e-4, 0.02, 0.005, 0.1, 1.0)
    assert ok == bool(f[f"ok_K{K}"])
    sd = m.state_dict()
    for k in KEYS:
        ref = f[f"K{K}_{k}"]
        assert np.abs(sd[k].numpy() - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max()), k


def test_nonlinear_fit_oracle_matches_reference(golden):
    f = golden("mlp_traj.npz")
    X = torch.from_numpy(golden("data_d20_n1000_seed0.npz")["X"])
    m = _model(f)
    W = nonlinear_fit(m, X, T=2, warm_iter=300, max_iter=500)
    np.testing.assert_allclose(W, f["fit_W"], rtol=0, atol=1e-10)
