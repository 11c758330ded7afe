"""CPU oracle for the PST trek regularizer -- TEST INFRASTRUCTURE ONLY.

Restates `pst`/`pst_mat`/`trek_value_grad` of the reference
(`/root/reference/src/notreks/notreks.py`, the PST branch) with torch on the CPU, float64,
gradients by autograd as the reference takes them:

    W2 = W * W;  F = expm(W2) | (I - W2 + eps I)^-1 | I + sum_{k<=K} W2^k / k | (I + W2)^d
    H = F^T F;   value = agg(H[rows, cols]);  grad = d value / d W

Only tests/ may import it; the GPU path (midagma_amd, csrc/trek.hip) never does.
Pinned against fixtures produced by the reference itself (tests/golden/make_golden.py,
`trek_pst.npz`).
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["pst_value_grad"]


def _f_of_w2(W2: torch.Tensor, seq: str, K_log, eps_inv: float) -> torch.Tensor:
    d = W2.shape[0]
    eye = torch.eye(d, dtype=W2.dtype)
    if seq == "exp":                                            # notreks pst_mat, exp branch
        return torch.matrix_exp(W2)
    if seq == "inv":                                            # (I - W2 + eps I)^-1 by solve
        A = eye - W2
        if eps_inv > 0:
            A = A + eps_inv * eye
        return torch.linalg.solve(A, eye)
    if seq == "log":                                            # I + sum_{k=1..K} W2^k / k
        K = 2 * d if K_log is None else int(K_log)
        out, Wk = eye.clone(), W2.clone()
        for k in range(1, K + 1):
            out = out + Wk / float(k)
            Wk = Wk @ W2
        return out
    if seq == "binom":                                          # (I + W2)^d, repeated products
        A = eye + W2
        out = A
        for _ in range(d - 1):
            out = out @ A
        return out
    raise ValueError(seq)


def pst_value_grad(W: np.ndarray, pairs, seq: str = "exp", *, K_log=None, eps_inv: float = 1e-8,
                   agg: str = "mean", grad: bool = True):
    """(value, dvalue/dW) of the PST penalty; (0, 0) for an empty pair list."""
    P = np.asarray(pairs, dtype=np.int64)
    if P.size == 0:
        return 0.0, np.zeros_like(W)
    Wt = torch.as_tensor(np.asarray(W, dtype=np.float64)).clone().requires_grad_(grad)
    F = _f_of_w2(Wt * Wt, seq.lower().strip(), K_log, eps_inv)
    H = F.transpose(0, 1) @ F
    vals = H[torch.as_tensor(P[:, 0]), torch.as_tensor(P[:, 1])]
    agg = agg.lower().strip()
    if agg == "mean":
        v = vals.mean()
    elif agg == "sum":
        v = vals.sum()
    elif agg == "max":
        v = vals.max()
    elif agg == "lse":
        v = torch.logsumexp(vals, dim=0)
    else:
        raise ValueError(agg)
    if not grad:
        return float(v.detach()), None
    v.backward()
    return float(v.detach()), Wt.grad.detach().numpy().copy()


def _positive(x: np.ndarray) -> np.ndarray:
    """notreks `_make_positive_vector`: real part, sign such that the sum is positive."""
    x = np.real(x).astype(np.float64)
    return -x if x.sum() < 0 else x


def tcc_value_grad(W: np.ndarray, pairs, *, w: float = 1.0, eps: float = 1e-12, grad: bool = True):
    """(value, d value / d W) of the TCC penalty as the minimize loop takes it: notreks
    `trek_value_grad` calls `trek_cycle_coupling_value_gradW` with its defaults, i.e. the
    spectral penalty, version 'approx_trek_graph', Perron pairs by `numpy.linalg.eig`
    (notreks.py:156-238, 291-395, 667-706):

        W2 = W o W,  A = [[W2, w S], [I, W2^T]],  B = [[W2, 0], [I, W2^T]]
        rho_A, u, v = Perron root and left / right vectors of A (unit, positive sum)
        G_A = u v^T / (u^T v + eps)
        value = (rho_A - u^T B u / (u^T u + eps)) / m
        grad  = 2 W o ((G_A[:d,:d] + G_A[d:,d:]^T) - (u1 u1^T + u2 u2^T) / (u^T u + eps)) / m
    """
    P = np.asarray(pairs, dtype=np.int64)
    W = np.asarray(W, dtype=np.float64)
    if P.size == 0:
        return 0.0, np.zeros_like(W)
    d = W.shape[0]
    W2 = W * W
    S = np.zeros((d, d))
    S[P[:, 0], P[:, 1]] = 1.0
    eye = np.eye(d)
    A = np.block([[W2, float(w) * S], [eye, W2.T]])
    B = np.block([[W2, np.zeros((d, d))], [eye, W2.T]])
    vals, vecs = np.linalg.eig(A)
    idx = np.argmax(vals.real)
    rho = float(vals[idx].real)
    v = _positive(vecs[:, idx])
    valsT, vecsT = np.linalg.eig(A.T)
    u = _positive(vecsT[:, np.argmax(valsT.real)])
    G_A = np.outer(u, v) / ((u * v).sum() + eps)
    GW2_A = G_A[:d, :d] + G_A[d:, d:].T
    rho_lb = (u * (B @ u)).sum() / ((u * u).sum() + eps)
    den = (u @ u) + eps
    u1, u2 = u[:d], u[d:]
    GW2_lb = (np.outer(u1, u1) + np.outer(u2, u2)) / den
    m = int(P.shape[0])
    value = (rho - rho_lb) / m
    if not grad:
        return float(value), None
    return float(value), (2.0 * W * GW2_A - 2.0 * W * GW2_lb) / m
