"""Development probe (CPU, oracle): residual of the fast inverse's warm start over a default fit.

Every 50th Adam step of LinearOracle.fit(d, n = 10 d), compares ||I - A_t X0||_inf (max row sum)
for X0 = inv(A_{t-1}) (the previous slot's inverse) and X0 = 2 inv(A_{t-1}) - inv(A_{t-2}) (the
linear extrapolation the fast blocked inverse uses), per stage s.  Usage: python tests/probes/probe_extrap.py 100
"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.abspath(__file__).rsplit('/tests/', 1)[0])
from oracle.dagma_oracle import LinearOracle
from midagma_amd.simulate import make_dataset
d = int(sys.argv[1]); n = 10 * d
X, _, _ = make_dataset(d, n, seed=0)
class O(LinearOracle):
    hist = []; stats = []
    def _inv(self, W, s):
        self.k = getattr(self, "k", 0) + 1
        A = s * np.eye(d) - W * W
        M = np.linalg.inv(A) if self.k % 50 in (48, 49, 0) else None
        h = self.hist
        if self.k % 50 == 0 and len(h) >= 2 and h[-1][1] == s and h[-2][1] == s:
            P1, P2 = h[-1][0], h[-2][0]
            r1 = np.abs(np.eye(d) - A @ P1).sum(1).max()
            r2 = np.abs(np.eye(d) - A @ (2 * P1 - P2)).sum(1).max()
            self.stats.append((s, r1, r2))
        if M is not None: h.append((M, s)); del h[:-2]
        else: h.clear()
        return super()._inv(W, s)
o = O("l2")
o.fit(X.copy(), lambda1=0.03)
S = np.array(O.stats)
for sv in sorted(set(S[:, 0]), reverse=True):
    m = S[:, 0] == sv
    l1, l2 = np.log10(S[m, 1]), np.log10(S[m, 2])
    print(f"s={sv}: n={m.sum()} log10 rho plain p25/50/75 {np.percentile(l1,[25,50,75]).round(2)}  extrap {np.percentile(l2,[25,50,75]).round(2)}  frac<=1e-4 plain {np.mean(S[m,1]<=1e-4):.2f} extrap {np.mean(S[m,2]<=1e-4):.2f}")
