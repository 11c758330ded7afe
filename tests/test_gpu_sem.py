"""GPU linear-SEM generator (csrc/sem.hip, midagma_sem_linear) vs the CPU oracle
(oracle/sem_oracle.py) on identical seeds, plus size-independent properties at scale.

Tolerances: uniform / logistic / poisson are bit-exact (integer Philox stream, exact f64
arithmetic, comparisons); gauss / exp / gumbel go through log / sincos, where the device
library and glibc may differ by an ulp: rtol 1e-13 relative to max |X| of the column."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from midagma_amd import utils  # noqa: E402
from oracle import sem_oracle as so  # noqa: E402


def _W(d, seed, scale=1.0, graph="ER"):
    utils.set_random_seed(seed)
    B = utils.simulate_dag(d, d, graph)
    return utils.simulate_parameter(B) * scale


@pytest.mark.parametrize("sem", ["gauss", "exp", "gumbel", "uniform", "logistic", "poisson"])
@pytest.mark.parametrize("d,n", [(20, 3001), (64, 1000)])
def test_sem_matches_oracle(sem, d, n):
    W = _W(d, 7, scale=0.1 if sem == "poisson" else 1.0)
    scale = np.linspace(0.5, 1.5, d)
    X = utils.simulate_linear_sem_gpu(W, n, sem, noise_scale=scale, seed=1234, device=0).cpu().numpy()
    R = so.sem_linear(W, 0, n, sem, noise_scale=scale, seed=1234)
    if sem in ("uniform", "logistic", "poisson"):
        np.testing.assert_array_equal(X, R)
    else:
        tol = 1e-13 * np.maximum(np.abs(R).max(0), 1.0)
        assert np.all(np.abs(X - R) <= tol), np.abs(X - R).max()


def test_sem_poisson_large_rates_exact():
    """lam = exp(1.5 x0) up to ~e^10: the PTRS branch (lam >= 10) against the oracle."""
    W = np.array([[0.0, 1.5], [0.0, 0.0]])
    X = utils.simulate_linear_sem_gpu(W, 3000, "poisson", seed=21, device=0).cpu().numpy()
    R = so.sem_linear(W, 0, 3000, "poisson", seed=21)
    assert (np.exp(1.5 * R[:, 0]) >= 10).sum() > 100
    np.testing.assert_array_equal(X, R)


def test_sem_rows_independent_of_split_and_slabs():
    W = _W(50, 3)
    n = 5001
    full = utils.simulate_linear_sem_gpu(W, n, "gauss", seed=9, device=0)
    a = utils.simulate_linear_sem_gpu(W, n, "gauss", seed=9, device=0, row0=0, n_rows=1777)
    b = utils.simulate_linear_sem_gpu(W, n, "gauss", seed=9, device=0, row0=1777, n_rows=n - 1777)
    assert torch.equal(full, torch.cat([a, b]))
    os.environ["MIDAGMA_SEM_SLAB_MB"] = "1"   # 2621-row slabs: several slabs per call
    try:
        c = utils.simulate_linear_sem_gpu(W, n, "gauss", seed=9, device=0, row0=3, n_rows=n - 3)
    finally:
        del os.environ["MIDAGMA_SEM_SLAB_MB"]
    assert torch.equal(full[3:], c)


def test_sem_edge_cases():
    # no edges, a single node, a chain deeper than one level per node, empty rows
    Z = utils.simulate_linear_sem_gpu(np.zeros((5, 5)), 101, "uniform", seed=2, device=0).cpu().numpy()
    np.testing.assert_array_equal(Z, so.sem_linear(np.zeros((5, 5)), 0, 101, "uniform", seed=2))
    one = utils.simulate_linear_sem_gpu(np.zeros((1, 1)), 7, "gauss", seed=2, device=0).cpu().numpy()
    np.testing.assert_allclose(one, so.sem_linear(np.zeros((1, 1)), 0, 7, "gauss", seed=2), rtol=1e-13)
    d = 40
    chain = np.diag(np.full(d - 1, 0.9), 1)
    X = utils.simulate_linear_sem_gpu(chain, 257, "gauss", seed=4, device=0).cpu().numpy()
    R = so.sem_linear(chain, 0, 257, "gauss", seed=4)
    np.testing.assert_allclose(X, R, rtol=0, atol=1e-12 * np.abs(R).max())
    e = utils.simulate_linear_sem_gpu(chain, 10, "gauss", seed=4, device=0, row0=10, n_rows=0)
    assert e.shape == (0, d)
    cyc = chain.copy()
    cyc[d - 1, 0] = 1.0
    with pytest.raises(ValueError):
        utils.simulate_linear_sem_gpu(cyc, 10, "gauss", seed=4, device=0)


def test_sem_large_residual_is_the_noise():
    """d=1000, n=2e5 (bench-sized graph): E = X (I - W) has iid N(0, 1) columns."""
    d, n = 1000, 200000
    W = _W(d, 0)
    X = utils.simulate_linear_sem_gpu(W, n, "gauss", seed=77, device=0)
    E = X @ (torch.eye(d, dtype=torch.float64, device=X.device) - torch.from_numpy(W).to(X.device))
    mean = E.mean(0).abs().max().item()
    std = E.std(0)
    assert mean < 6.0 / np.sqrt(n)
    assert (std - 1.0).abs().max().item() < 6.0 * np.sqrt(0.5 / n)
    C = (E[:, :64].T @ E[:, :64]) / n - torch.eye(64, dtype=torch.float64, device=X.device)
    assert C.abs().max().item() < 6.0 / np.sqrt(n)
    # spot rows against the oracle
    R = so.sem_linear(W, 123456, 4, "gauss", seed=77)
    np.testing.assert_allclose(X[123456:123460].cpu().numpy(), R, rtol=0, atol=1e-11 * np.abs(R).max())
