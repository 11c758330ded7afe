"""Synthetic linear-SEM data for DAGMA (numpy only, igraph-free).

The reference draws its DAGs and data with `dagma.utils` (`utils.py:21-172`),
which needs `igraph`; that module is absent in this image.  This generator
keeps the reference's *distribution* and conventions, with a seeded
`numpy.random.Generator` instead of the global numpy/igraph RNG:

* ER DAG with exactly ``s0`` undirected edges, oriented acyclically by a
  random node order (`utils.py:58-62`: Erdos_Renyi(n=d, m=s0) -> random
  acyclic orientation -> random permutation);
* edge weights drawn uniformly from ``(-2,-0.5) U (0.5,2)`` (`utils.py:73-96`);
* ``x_j = X[:, pa(j)] @ W[pa(j), j] + z_j`` with N(0, 1) noise, nodes
  visited in topological order (`utils.py:99-172`, ``sem_type='gauss'``);
  ``sem_type='logistic'`` draws ``x_j ~ Bernoulli(sigmoid(.))``.

``W[i, j]`` is the weight of edge i -> j, as in the reference.
"""
from __future__ import annotations

import numpy as np

__all__ = ["simulate_er_dag", "simulate_weights", "simulate_linear_sem", "make_dataset",
           "is_dag", "count_accuracy"]


def simulate_er_dag(d: int, s0: int, rng: np.random.Generator) -> np.ndarray:
    """Binary adjacency B (d x d) of a random DAG with exactly min(s0, d(d-1)/2) edges."""
    n_pairs = d * (d - 1) // 2
    m = min(int(s0), n_pairs)
    # edge between topological positions (a, b), a < b, picked uniformly without replacement
    flat = rng.choice(n_pairs, size=m, replace=False)
    # unrank flat index -> (row, col) of the strict upper triangle in row-major order
    rows, cols = np.triu_indices(d, k=1)
    B_ordered = np.zeros((d, d))
    B_ordered[rows[flat], cols[flat]] = 1.0
    perm = rng.permutation(d)  # node label of topological position
    B = np.zeros((d, d))
    B[np.ix_(perm, perm)] = B_ordered
    return B


def simulate_weights(B: np.ndarray, rng: np.random.Generator,
                     w_ranges=((-2.0, -0.5), (0.5, 2.0))) -> np.ndarray:
    """Weighted adjacency: each edge weight uniform in one of the disjoint ranges."""
    which = rng.integers(len(w_ranges), size=B.shape)
    W = np.zeros(B.shape)
    for i, (lo, hi) in enumerate(w_ranges):
        U = rng.uniform(lo, hi, size=B.shape)
        W += B * (which == i) * U
    return W


def _topological_order(W: np.ndarray) -> np.ndarray:
    d = W.shape[0]
    adj = W != 0
    indeg = adj.sum(axis=0).astype(np.int64)
    order, frontier = [], [j for j in range(d) if indeg[j] == 0]
    while frontier:
        j = frontier.pop()
        order.append(j)
        for c in np.flatnonzero(adj[j]):
            indeg[c] -= 1
            if indeg[c] == 0:
                frontier.append(int(c))
    if len(order) != d:
        raise ValueError("W must be a DAG")
    return np.asarray(order)


def is_dag(W: np.ndarray) -> bool:
    try:
        _topological_order(np.asarray(W))
        return True
    except ValueError:
        return False


def simulate_linear_sem(W: np.ndarray, n: int, rng: np.random.Generator,
                        sem_type: str = "gauss", noise_scale: float = 1.0) -> np.ndarray:
    d = W.shape[0]
    X = np.zeros((n, d))
    for j in _topological_order(W):
        pa = np.flatnonzero(W[:, j])
        lin = X[:, pa] @ W[pa, j]
        if sem_type == "gauss":
            X[:, j] = lin + rng.normal(scale=noise_scale, size=n)
        elif sem_type == "logistic":
            X[:, j] = rng.binomial(1, 1.0 / (1.0 + np.exp(-lin))).astype(np.float64)
        else:
            raise ValueError(f"unknown sem type {sem_type!r}")
    return X


def make_dataset(d: int, n: int, seed: int = 0, s0: int | None = None, sem_type: str = "gauss"):
    """(X, W_true, B_true) for an ER(s0=d) linear SEM; deterministic in ``seed``."""
    rng = np.random.default_rng(seed)
    B = simulate_er_dag(d, d if s0 is None else s0, rng)
    W = simulate_weights(B, rng)
    X = simulate_linear_sem(W, n, rng, sem_type=sem_type)
    return X, W, B


def count_accuracy(B_true: np.ndarray, B_est: np.ndarray) -> dict:
    """SHD / TPR / FDR / FPR / nnz of a DAG estimate (reference `utils.py:245-310`, DAG case)."""
    B_true = np.asarray(B_true) != 0
    B_est = np.asarray(B_est) != 0
    d = B_true.shape[0]
    pred = set(np.flatnonzero(B_est).tolist())
    cond = set(np.flatnonzero(B_true).tolist())
    cond_rev = set(np.flatnonzero(B_true.T).tolist())
    true_pos = pred & cond
    false_pos = pred - (cond | cond_rev)
    reverse = (pred - cond) & cond_rev
    cond_neg = 0.5 * d * (d - 1) - len(cond)
    lower = lambda M: set(np.flatnonzero(np.tril(M.astype(int) + M.T.astype(int))).tolist())
    pl, cl = lower(B_est), lower(B_true)
    shd = len(pl - cl) + len(cl - pl) + len(reverse)
    return {"fdr": (len(reverse) + len(false_pos)) / max(len(pred), 1),
            "tpr": len(true_pos) / max(len(cond), 1),
            "fpr": (len(reverse) + len(false_pos)) / max(cond_neg, 1),
            "shd": shd, "nnz": len(pred)}
