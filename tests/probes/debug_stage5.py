"""Compare GPU vs oracle checkpoints for the last stage of the d=20 fit (development tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch  # noqa
from threadpoolctl import threadpool_limits
from oracle.dagma_oracle import LinearOracle, objective
from midagma_amd.solver import HipSolver
X = np.load('tests/golden/data_d20_n1000_seed0.npz')['X']
with threadpool_limits(1):
    o = LinearOracle('l2'); o.fit(X.copy(), lambda1=0.03)
    W4 = None
    # re-run to capture W before each stage
    o2 = LinearOracle('l2'); o2.prepare(X.copy(), 0.03, 1000)
    W = np.zeros((20, 20)); mu = 1.0
    starts = []
    for i, s in enumerate([1.0, .9, .8, .7, .6]):
        starts.append((W.copy(), mu, s))
        W, tr = o2.minimize(W.copy(), mu, 30000 if i < 4 else 60000, s, 3e-4)
        mu *= 0.1
sol = HipSolver(20); sol.set_cov(o2.cov)
for i, (W0, mu, s) in enumerate(starts):
    Wg = W0.copy()
    res = sol.minimize(Wg, mu, 30000 if i < 4 else 60000, s, 3e-4, tol=1e-6, lambda1=0.03, want_checkpoints=True)
    Wo, tr = o2.minimize(W0.copy(), mu, 30000 if i < 4 else 60000, s, 3e-4)
    print(f"stage {i} mu={mu} s={s}: gpu iters {res.iters} early {res.early_stop}; oracle iters {tr.iters}; max|dW|={np.abs(Wg-Wo).max():.3e}")
    for a, b in zip(res.checkpoints[:4], tr.checkpoints[:4]):
        print("   gpu", a[:4], "\n   ora", b)
        # oracle objective at the oracle's W is b; evaluate the oracle objective at GPU W? not stored
