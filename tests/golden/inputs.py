"""Seeded inputs shared by make_golden.py and the tests (no reference import here)."""
import numpy as np


def mlp_fc1(d, m1):
    """fc1 weights of the DagmaMLP h_func fixtures (make_golden.gen_mlp)."""
    rng = np.random.default_rng(1000 + d)
    return rng.standard_normal((d * m1, d)) * (0.3 / np.sqrt(d * m1))
