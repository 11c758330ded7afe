"""CPU oracle for the GPU linear-SEM generator -- TEST INFRASTRUCTURE ONLY.

Restates, in numpy, what `midagma_sem_linear` (csrc/sem.hip) computes: the reference's
structural equations (`/root/reference/src/dagma/utils.py:99-172`, `simulate_linear_sem`)

    x_j = X[:, pa(j)] @ W[pa(j), j] + z_j            (gauss / exp / gumbel / uniform)
    x_j ~ Bernoulli(sigmoid(X[:, pa(j)] @ W[pa(j), j]))   (logistic)
    x_j ~ Poisson(exp(X[:, pa(j)] @ W[pa(j), j]))         (poisson)

nodes in topological order, with the noise drawn from a counter-based generator instead of
numpy's global stream (a GPU cannot replay numpy's Mersenne Twister):

* Philox4x32-10 (Salmon et al., SC'11, "Parallel random numbers: as easy as 1, 2, 3";
  the Random123 library's `philox4x32_10`), key = (seed lo, seed hi),
  counter = (pair lo, pair hi, node, draw) with pair = global row // 2, so a row's values do
  not depend on how the rows are split into calls or shards.  Pinned by the Random123
  known-answer vectors in tests/test_sem_oracle.py.
* one Philox block -> two uniforms u = (k + 1/2) 2^-52 from its two 64-bit halves
  (k = top 52 bits), u in (0, 1);  even rows take the first, odd rows the second:
    gauss   : Box-Muller, r = sqrt(-2 ln u1), z = scale * r cos(2 pi u2) (even) / r sin(2 pi u2) (odd)
    exp     : z = -scale ln u            gumbel: z = -scale ln(-ln u)
    uniform : z = -scale + (2 scale) u   logistic: x = 1 if u < 1 / (1 + exp(-acc)) else 0
    poisson : its own counter words (draw >= 2^30), 2 uniforms per block, numpy's two
              samplers (multiplication for lam < 10, PTRS (Hormann 1993) above)
* the parent sum runs over parents in ascending index with separate multiply and add
  (acc = acc + w * x), as the kernel does with -ffp-contract=off.

Integer / uniform / logistic / poisson paths match the kernel bit for bit; paths through
log / cos / sin / exp match to libm-vs-device ulps (tolerances written in the tests).
The parents / sums are the reference's equations; only the noise stream is this
generator's own (documented in DESIGN.md).
"""
from __future__ import annotations

import math

import numpy as np

__all__ = ["philox4x32_10", "uniforms", "topological_levels", "sem_linear", "SEM_TYPES"]

SEM_TYPES = {"gauss": 0, "exp": 1, "gumbel": 2, "uniform": 3, "logistic": 4, "poisson": 5}

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)
POISSON_DRAW0 = 1 << 30


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32 with 10 rounds on arrays of uint32 words (broadcast); returns 4 uint32 arrays."""
    c = [np.asarray(x, dtype=np.uint64) & _MASK for x in (c0, c1, c2, c3)]
    k0 = np.asarray(k0, dtype=np.uint64) & _MASK
    k1 = np.asarray(k1, dtype=np.uint64) & _MASK
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & _MASK
            k1 = (k1 + _W1) & _MASK
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return [x.astype(np.uint32) for x in c]


def _u52(hi, lo):
    k = ((hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)) >> np.uint64(12)
    return (k.astype(np.float64) + 0.5) * 2.0 ** -52


def uniforms(seed: int, pair, node, draw):
    """The two uniforms of the Philox block at counter (pair, node, draw), key = seed."""
    pair = np.asarray(pair, dtype=np.uint64)
    x = philox4x32_10(pair & _MASK, pair >> np.uint64(32), node, draw, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return _u52(x[0], x[1]), _u52(x[2], x[3])


def topological_levels(W: np.ndarray):
    """Nodes grouped by longest-path depth (Kahn by levels); ValueError if W is not a DAG."""
    A = np.asarray(W) != 0
    d = A.shape[0]
    indeg = A.sum(axis=0).astype(np.int64)
    level = [j for j in range(d) if indeg[j] == 0]
    levels, seen = [], 0
    while level:
        levels.append(level)
        seen += len(level)
        nxt = []
        for j in level:
            for c in np.flatnonzero(A[j]):
                indeg[c] -= 1
                if indeg[c] == 0:
                    nxt.append(int(c))
        level = sorted(nxt)
    if seen != d:
        raise ValueError("W must be a DAG")
    return levels


def _poisson(lam: float, seed: int, pair: int, node: int, odd: int) -> float:
    """numpy's Poisson samplers, driven by this row's own Philox blocks."""
    state = {"draw": POISSON_DRAW0 + (odd << 29), "buf": []}

    def u():
        if not state["buf"]:
            a, b = uniforms(seed, np.uint64(pair), node, state["draw"])
            state["buf"] = [float(b), float(a)]
            state["draw"] += 1
        return state["buf"].pop()

    if lam <= 0.0:
        return 0.0
    if lam < 10.0:
        enlam = math.exp(-lam)
        x, prod = 0, 1.0
        for _ in range(100000):
            prod = prod * u()
            if prod > enlam:
                x += 1
            else:
                return float(x)
        return float(x)
    slam = math.sqrt(lam)
    loglam = math.log(lam)
    b = 0.931 + 2.53 * slam
    a = -0.059 + 0.02483 * b
    invalpha = 1.1239 + 1.1328 / (b - 3.4)
    vr = 0.9277 - 3.6224 / (b - 2.0)
    k = 0.0
    for _ in range(4096):
        U = u() - 0.5
        V = u()
        us = 0.5 - abs(U)
        k = math.floor((2.0 * a / us + b) * U + lam + 0.43)
        if us >= 0.07 and V <= vr:
            return float(k)
        if k < 0.0 or (us < 0.013 and V > us):
            continue
        if (math.log(V) + math.log(invalpha) - math.log(a / (us * us) + b)) <= (-lam + k * loglam - math.lgamma(k + 1.0)):
            return float(k)
    return float(max(k, 0.0))


def sem_linear(W: np.ndarray, row0: int, n_rows: int, sem_type: str = "gauss", noise_scale=None,
               seed: int = 0) -> np.ndarray:
    """Rows [row0, row0 + n_rows) of the linear SEM sample matrix (n_rows x d)."""
    W = np.asarray(W, dtype=np.float64)
    d = W.shape[0]
    st = SEM_TYPES[sem_type]
    scale = np.ones(d) if noise_scale is None else np.broadcast_to(np.asarray(noise_scale, np.float64), (d,))
    rows = np.arange(row0, row0 + n_rows, dtype=np.int64)
    pair = (rows >> 1).astype(np.uint64)
    odd = (rows & 1).astype(bool)
    X = np.zeros((n_rows, d))
    for level in topological_levels(W):
        for j in level:
            acc = np.zeros(n_rows)
            for p in np.flatnonzero(W[:, j]):
                acc = acc + W[p, j] * X[:, p]
            s = scale[j]
            if st == 5:
                X[:, j] = [_poisson(math.exp(a), seed, int(pr), j, int(o)) for a, pr, o in zip(acc, pair, odd)]
                continue
            u1, u2 = uniforms(seed, pair, j, 0)
            if st == 0:
                r = np.sqrt(-2.0 * np.log(u1))
                t = 2.0 * np.pi * u2
                z = np.where(odd, r * np.sin(t), r * np.cos(t))
                X[:, j] = acc + s * z
                continue
            u = np.where(odd, u2, u1)
            if st == 1:
                X[:, j] = acc + (-s) * np.log(u)
            elif st == 2:
                X[:, j] = acc + (-s) * np.log(-np.log(u))
            elif st == 3:
                X[:, j] = acc + (-s + (2.0 * s) * u)
            elif st == 4:
                p = 1.0 / (1.0 + np.exp(-acc))
                X[:, j] = (u < p).astype(np.float64)
    return X
