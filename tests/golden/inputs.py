"""Seeded inputs shared by make_golden.py and the tests (no reference import here)."""
import numpy as np


def mlp_fc1(d, m1):
    """fc1 weights of the DagmaMLP h_func fixtures (make_golden.gen_mlp)."""
    rng = np.random.default_rng(1000 + d)
    return rng.standard_normal((d * m1, d)) * (0.3 / np.sqrt(d * m1))


def mlp_params(d, m1):
    """All DagmaMLP([d, m1, 1]) parameters for the nonlinear minimize fixtures
    (make_golden.gen_mlp_traj): fc1 from mlp_fc1, zero fc1 bias, LocallyConnected fc2 uniform
    in +-1/sqrt(m1) as its reset_parameters draws (locally_connected.py:48-53)."""
    rng = np.random.default_rng(2000 + d)
    b = 1.0 / np.sqrt(m1)
    return {"fc1.weight": mlp_fc1(d, m1), "fc1.bias": np.zeros(d * m1),
            "fc2.0.weight": rng.uniform(-b, b, (d, m1, 1)), "fc2.0.bias": rng.uniform(-b, b, (d, 1))}
