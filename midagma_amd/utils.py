"""`dagma.utils` without igraph (reference: /root/reference/src/dagma/utils.py:1-310), plus the
GPU linear-SEM generator (csrc/sem.hip).

Same names, arguments and errors as the reference:

    set_random_seed, is_dag, simulate_dag, simulate_parameter, simulate_linear_sem,
    simulate_nonlinear_sem, count_accuracy

igraph is absent from this image, so its three roles are restated:

* `is_dag` / topological order: Kahn's algorithm with a FIFO of sources in ascending id and
  out-neighbours in ascending id -- igraph's `topological_sorting` (the order in which the
  reference visits nodes, hence consumes numpy draws);
* parents: ascending in-neighbour ids (igraph's `neighbors(j, mode=IN)`);
* random graphs (Erdos_Renyi G(n, m), Barabasi psumtree, Random_Bipartite G(n1, n2, m)):
  the same distributions, drawn from Python's `random` module -- the generator python-igraph
  uses by default, and the one `set_random_seed` seeds.  igraph's internal sampling order is
  not reproduced, so the graph of a given seed differs from the reference's; every numpy draw
  (`np.random.permutation` of the node order, `simulate_parameter`, the SEM noise) is made in
  the reference's order, so given the same B the weights and samples are the reference's.

`simulate_linear_sem_gpu` is the GPU path for large data: the same
structural equations evaluated level by level on the device, noise from a counter-based
Philox stream (a row's values do not depend on how rows are sharded).
"""
from __future__ import annotations

import ctypes as C
import random
import typing
from collections import deque

import numpy as np
from scipy.special import expit as sigmoid

__all__ = ["set_random_seed", "is_dag", "topological_sort", "simulate_dag", "simulate_parameter",
           "simulate_linear_sem", "simulate_nonlinear_sem", "count_accuracy", "simulate_linear_sem_gpu",
           "SEM_TYPES"]

SEM_TYPES = {"gauss": 0, "exp": 1, "gumbel": 2, "uniform": 3, "logistic": 4, "poisson": 5}


def set_random_seed(seed: int):
    """utils.py:8-10: seeds Python's `random` (the graph generator) and numpy's global stream."""
    random.seed(seed)
    np.random.seed(seed)


def topological_sort(W: np.ndarray) -> typing.Optional[typing.List[int]]:
    """igraph `topological_sorting()` of the graph with an edge i -> j per nonzero W[i, j], or
    None when it has a cycle (self-loops included)."""
    A = np.asarray(W) != 0
    d = A.shape[0]
    indeg = A.sum(axis=0).astype(np.int64)
    q = deque(j for j in range(d) if indeg[j] == 0)
    order = []
    while q:
        j = q.popleft()
        order.append(j)
        for c in np.flatnonzero(A[j]):
            indeg[c] -= 1
            if indeg[c] == 0:
                q.append(int(c))
    return order if len(order) == d else None


def is_dag(W: np.ndarray) -> bool:
    """utils.py:13-18."""
    return topological_sort(W) is not None


def _parents(W: np.ndarray, j: int) -> np.ndarray:
    return np.flatnonzero(np.asarray(W)[:, j] != 0)


# --- random graphs (utils.py:21-70) --------------------------------------------------------

def _erdos_renyi_gnm(d: int, m: int) -> np.ndarray:
    """Undirected G(n, m) without loops or multi-edges: m distinct pairs, uniformly."""
    n_pairs = d * (d - 1) // 2
    if m > n_pairs:
        raise ValueError("Too many edges requested compared to the number of vertices")
    B = np.zeros((d, d))
    if m == 0:
        return B
    rows, cols = np.triu_indices(d, k=1)
    pick = np.asarray(random.sample(range(n_pairs), m), dtype=np.int64)
    B[rows[pick], cols[pick]] = 1.0
    B[cols[pick], rows[pick]] = 1.0
    return B


def _barabasi(d: int, m: int) -> np.ndarray:
    """Directed preferential attachment (igraph Barabasi, psumtree, power 1, zero appeal 1,
    no multi-edges): vertex i cites min(m, i) distinct older vertices, each drawn with
    probability proportional to in-degree + 1; edges point from the new vertex to the cited."""
    B = np.zeros((d, d))
    indeg = np.zeros(d)
    for i in range(1, d):
        k = min(m, i)
        if k >= i:
            chosen = list(range(i))
        else:
            weight = indeg[:i] + 1.0
            chosen = []
            for _ in range(k):
                cum = np.cumsum(weight)
                to = int(np.searchsorted(cum, random.random() * cum[-1], side="right"))
                to = min(to, i - 1)
                chosen.append(to)
                weight[to] = 0.0
        for to in chosen:
            B[i, to] = 1.0
            indeg[to] += 1.0
    return B


def _random_bipartite(top: int, bottom: int, m: int) -> np.ndarray:
    """G(n1, n2, m), directed top -> bottom (ids 0..top-1 then top..top+bottom-1)."""
    if m > top * bottom:
        raise ValueError("Too many edges requested compared to the number of vertices")
    d = top + bottom
    B = np.zeros((d, d))
    if m:
        pick = np.asarray(random.sample(range(top * bottom), m), dtype=np.int64)
        B[pick // bottom, top + pick % bottom] = 1.0
    return B


def simulate_dag(d: int, s0: int, graph_type: str) -> np.ndarray:
    """utils.py:21-70: (d, d) binary adjacency of a random DAG with about s0 edges."""
    def _random_permutation(M):
        P = np.random.permutation(np.eye(M.shape[0]))
        return P.T @ M @ P

    def _random_acyclic_orientation(B_und):
        return np.tril(_random_permutation(B_und), k=-1)

    if graph_type == "ER":
        B = _random_acyclic_orientation(_erdos_renyi_gnm(d, s0))
    elif graph_type == "SF":
        B = _barabasi(d, int(round(s0 / d)))
    elif graph_type == "BP":
        top = int(0.2 * d)
        B = _random_bipartite(top, d - top, s0)
    elif graph_type == "Fully":
        B = np.triu(np.ones((d, d)), 1)
    else:
        raise ValueError("unknown graph type")
    B_perm = _random_permutation(B)
    assert is_dag(B_perm)
    return B_perm


def simulate_parameter(B: np.ndarray,
                       w_ranges: typing.List[typing.Tuple[float, float]] = ((-2.0, -0.5), (0.5, 2.0)),
                       ) -> np.ndarray:
    """utils.py:73-96 (numpy draws in the reference's order)."""
    W = np.zeros(B.shape)
    S = np.random.randint(len(w_ranges), size=B.shape)
    for i, (low, high) in enumerate(w_ranges):
        U = np.random.uniform(low=low, high=high, size=B.shape)
        W += B * (S == i) * U
    return W


def _scale_vec(noise_scale, d):
    if noise_scale is None:
        return np.ones(d)
    if np.isscalar(noise_scale):
        return noise_scale * np.ones(d)
    if len(noise_scale) != d:
        raise ValueError("noise scale must be a scalar or have length d")
    return noise_scale


def simulate_linear_sem(W: np.ndarray, n: int, sem_type: str,
                        noise_scale: typing.Optional[typing.Union[float, typing.List[float]]] = None,
                        ) -> np.ndarray:
    """utils.py:99-172 on the CPU: x_j = X[:, pa(j)] @ W[pa(j), j] + z_j in topological order."""
    def _single(X, w, scale):
        if sem_type == "gauss":
            return X @ w + np.random.normal(scale=scale, size=n)
        if sem_type == "exp":
            return X @ w + np.random.exponential(scale=scale, size=n)
        if sem_type == "gumbel":
            return X @ w + np.random.gumbel(scale=scale, size=n)
        if sem_type == "uniform":
            return X @ w + np.random.uniform(low=-scale, high=scale, size=n)
        if sem_type == "logistic":
            return np.random.binomial(1, sigmoid(X @ w)) * 1.0
        if sem_type == "poisson":
            return np.random.poisson(np.exp(X @ w)) * 1.0
        raise ValueError("unknown sem type")

    d = W.shape[0]
    scale_vec = _scale_vec(noise_scale, d)
    order = topological_sort(W)
    if order is None:
        raise ValueError("W must be a DAG")
    if np.isinf(n):
        if sem_type == "gauss":
            return np.sqrt(d) * np.diag(scale_vec) @ np.linalg.inv(np.eye(d) - W)
        raise ValueError("population risk not available")
    X = np.zeros([n, d])
    for j in order:
        pa = _parents(W, j)
        X[:, j] = _single(X[:, pa], W[pa, j], scale_vec[j])
    return X


def simulate_nonlinear_sem(B: np.ndarray, n: int, sem_type: str,
                           noise_scale: typing.Optional[typing.Union[float, typing.List[float]]] = None,
                           ) -> np.ndarray:
    """utils.py:175-242: mlp / mim / gp / gp-add structural equations (numpy global stream)."""
    def _single(X, scale):
        z = np.random.normal(scale=scale, size=n)
        pa_size = X.shape[1]
        if pa_size == 0:
            return z
        if sem_type == "mlp":
            hidden = 100
            W1 = np.random.uniform(low=0.5, high=2.0, size=[pa_size, hidden])
            W1[np.random.rand(*W1.shape) < 0.5] *= -1
            W2 = np.random.uniform(low=0.5, high=2.0, size=hidden)
            W2[np.random.rand(hidden) < 0.5] *= -1
            return sigmoid(X @ W1) @ W2 + z
        if sem_type == "mim":
            ws = []
            for _ in range(3):
                w = np.random.uniform(low=0.5, high=2.0, size=pa_size)
                w[np.random.rand(pa_size) < 0.5] *= -1
                ws.append(w)
            return np.tanh(X @ ws[0]) + np.cos(X @ ws[1]) + np.sin(X @ ws[2]) + z
        if sem_type == "gp":
            from sklearn.gaussian_process import GaussianProcessRegressor
            return GaussianProcessRegressor().sample_y(X, random_state=None).flatten() + z
        if sem_type == "gp-add":
            from sklearn.gaussian_process import GaussianProcessRegressor
            gp = GaussianProcessRegressor()
            return sum([gp.sample_y(X[:, i, None], random_state=None).flatten() for i in range(X.shape[1])]) + z
        raise ValueError("unknown sem type")

    d = B.shape[0]
    scale_vec = noise_scale if noise_scale else np.ones(d)
    order = topological_sort(B)
    assert order is not None and len(order) == d
    X = np.zeros([n, d])
    for j in order:
        X[:, j] = _single(X[:, _parents(B, j)], scale_vec[j])
    return X


def count_accuracy(B_true: np.ndarray, B_est: np.ndarray) -> dict:
    """utils.py:245-310: fdr / tpr / fpr / shd / nnz of a DAG (or CPDAG, -1 = undirected) estimate."""
    if (B_est == -1).any():
        if not ((B_est == 0) | (B_est == 1) | (B_est == -1)).all():
            raise ValueError("B_est should take value in {0,1,-1}")
        if ((B_est == -1) & (B_est.T == -1)).any():
            raise ValueError("undirected edge should only appear once")
    else:
        if not ((B_est == 0) | (B_est == 1)).all():
            raise ValueError("B_est should take value in {0,1}")
        if not is_dag(B_est):
            raise ValueError("B_est should be a DAG")
    d = B_true.shape[0]
    pred_und = np.flatnonzero(B_est == -1)
    pred = np.flatnonzero(B_est == 1)
    cond = np.flatnonzero(B_true)
    cond_reversed = np.flatnonzero(B_true.T)
    cond_skeleton = np.concatenate([cond, cond_reversed])
    true_pos = np.intersect1d(pred, cond, assume_unique=True)
    true_pos_und = np.intersect1d(pred_und, cond_skeleton, assume_unique=True)
    true_pos = np.concatenate([true_pos, true_pos_und])
    false_pos = np.setdiff1d(pred, cond_skeleton, assume_unique=True)
    false_pos_und = np.setdiff1d(pred_und, cond_skeleton, assume_unique=True)
    false_pos = np.concatenate([false_pos, false_pos_und])
    extra = np.setdiff1d(pred, cond, assume_unique=True)
    reverse = np.intersect1d(extra, cond_reversed, assume_unique=True)
    pred_size = len(pred) + len(pred_und)
    cond_neg_size = 0.5 * d * (d - 1) - len(cond)
    fdr = float(len(reverse) + len(false_pos)) / max(pred_size, 1)
    tpr = float(len(true_pos)) / max(len(cond), 1)
    fpr = float(len(reverse) + len(false_pos)) / max(cond_neg_size, 1)
    pred_lower = np.flatnonzero(np.tril(B_est + B_est.T))
    cond_lower = np.flatnonzero(np.tril(B_true + B_true.T))
    extra_lower = np.setdiff1d(pred_lower, cond_lower, assume_unique=True)
    missing_lower = np.setdiff1d(cond_lower, pred_lower, assume_unique=True)
    shd = len(extra_lower) + len(missing_lower) + len(reverse)
    return {"fdr": fdr, "tpr": tpr, "fpr": fpr, "shd": shd, "nnz": pred_size}


# --- GPU generator (csrc/sem.hip) ----------------------------------------------------------

def simulate_linear_sem_gpu(W: np.ndarray, n: int, sem_type: str = "gauss",
                            noise_scale: typing.Optional[typing.Union[float, typing.List[float]]] = None, *,
                            seed: typing.Optional[int] = None, device=None, row0: int = 0,
                            n_rows: typing.Optional[int] = None, out=None):
    """Rows [row0, row0 + n_rows) (default: all n) of a linear SEM sample matrix, generated on
    the GPU into a float64 torch tensor (or `out`, a C-contiguous float64 CUDA tensor).

    Same structural equations as `simulate_linear_sem`; the noise is Philox4x32-10 keyed by
    `seed` (default: drawn from numpy's global stream, so `set_random_seed` fixes it) with
    counter (row // 2, node, draw).  Shards that pass their own `row0`/`n_rows` therefore see
    exactly the rows of the unsharded matrix.  Runs on the current stream of `device`."""
    import torch

    from . import _lib
    W = np.ascontiguousarray(W, dtype=np.float64)
    d = W.shape[0]
    if sem_type not in SEM_TYPES:
        raise ValueError("unknown sem type")
    if np.isinf(n):
        raise ValueError("population risk: use simulate_linear_sem")
    n_rows = int(n) - row0 if n_rows is None else int(n_rows)
    if row0 < 0 or n_rows < 0 or row0 + n_rows > n:
        raise ValueError("rows out of range")
    scale = np.ascontiguousarray(_scale_vec(noise_scale, d), dtype=np.float64)
    if seed is None:
        seed = int(np.random.randint(0, 2 ** 62, dtype=np.int64))
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    if out is None:
        out = torch.empty((n_rows, d), dtype=torch.float64, device=dev)
    elif (out.dtype != torch.float64 or not out.is_cuda or not out.is_contiguous() or tuple(out.shape) != (n_rows, d)):
        raise ValueError("out must be a contiguous float64 CUDA tensor of shape (n_rows, d)")
    lib = _lib.lib()
    with torch.cuda.device(out.device):
        stream = torch.cuda.current_stream(out.device).cuda_stream
        _lib.check(lib.midagma_sem_linear(_lib.dptr(W), d, row0, n_rows, SEM_TYPES[sem_type], _lib.dptr(scale),
                                          C.c_uint64(seed & (2 ** 64 - 1)), C.c_void_p(out.data_ptr()), d,
                                          C.c_void_p(stream) if stream else None), None, "sem_linear")
    return out
