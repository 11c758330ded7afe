"""How many Noda steps does the TCC kernel take per Adam step? (development tool, CPU only)

Replays csrc/tcc.hip's Noda iteration (Collatz-Wielandt start, warm start rule, the 1e-13 /
1e-14 stop rules, TCC_NODA_MAX) in numpy on every W of the oracle's minimize trajectory with
TCC on (tools/probe_perf.py trek_case's setup: make_dataset(d, 2d), 30 % of the upper pairs,
weight 0.1, mu 1, s 1, lr 3e-4) and prints the distribution of inverses per step.

    python tools/probe_noda.py [d] [K]
"""
import os
import sys
from collections import Counter

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402

NODA_MAX = 24


class Noda:
    def __init__(self):
        self.prev = None
        self.warm_ok = False
        self.counts = []

    def run(self, W, pairs, w=1.0):
        d = W.shape[0]
        W2 = W * W
        S = np.zeros((d, d))
        S[pairs[:, 0], pairs[:, 1]] = 1.0
        A = np.block([[W2, w * S], [np.eye(d), W2.T]])
        n = 2 * d
        if self.warm_ok and self.prev.min() > 1e-8 * self.prev.max():
            x = self.prev.copy()
        else:
            x = np.ones(n)
        sig = np.max(A @ x / x)
        inv = 0
        conv = False
        for _ in range(NODA_MAX):
            y = np.linalg.solve(sig * np.eye(n) - A, x)
            inv += 1
            if not np.all(y > 0) or not np.all(np.isfinite(y)):
                break
            r = x / y
            x = y / np.linalg.norm(y)
            up, lo = sig - r.min(), sig - r.max()
            stop = not (up - lo > 1e-13 * abs(up)) or not (sig - up > 1e-14 * abs(up))
            sig = up
            if stop:
                conv = True
                break
        inv += 1  # the final inverse
        M = np.linalg.inv(sig * (1 + 1e-14) * np.eye(n) - A)
        for _ in range(2):
            x = M @ x
            x = x / np.linalg.norm(x) * (1 if x.sum() > 0 else -1)
        self.prev = x
        rho_ok = np.isfinite(x).all()
        self.warm_ok = conv and rho_ok
        self.counts.append(inv)


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    rng = np.random.default_rng(0)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 40)
    o.trek = dict(kind="tcc", pairs=pairs, mode="opt", weight=0.1)
    nd = Noda()
    orig = o._trek

    def hooked(W, want_grad):
        nd.run(W, pairs)
        return orig(W, want_grad)

    o._trek = hooked
    o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    c = Counter(nd.counts)
    print(f"d={d} K={K}: inverses per step mean {np.mean(nd.counts):.2f}, histogram {sorted(c.items())}")
    for a in range(0, K, K // 10):
        print(f"  steps {a}-{a + K // 10}: mean {np.mean(nd.counts[a:a + K // 10]):.2f}")


if __name__ == "__main__":
    main()
