"""Development probe (CPU, oracle): could a WHOLE-matrix warm start replace the blocked inverse's
per-block product form at d = 1000?  Runs the oracle's minimize (linear.py:224-277) on config 2's
data and, at every step, measures rho = ||I - A_k X0||_inf for the linear extrapolation
X0 = 2 M_(k-1) - M_(k-2) of the last two inverses.  The product form X0 (I + R)(I + R^2)... needs
rho^(2^p) <= 1e-16, so rho decides how many whole-matrix D^3 GEMMs a step costs.

    python tools/probe_rho_whole.py s1 400       # stage 1 from W = 0
    python tools/probe_rho_whole.py k2000 400    # from the oracle's W after 2000 steps (traj_d1000.npz)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import scipy.linalg as spla  # noqa: E402

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402


def main():
    which, steps = sys.argv[1], int(sys.argv[2])
    d = 1000
    X, _, _ = make_dataset(d, 10000, seed=0)
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 1000)
    eye = np.eye(d)
    hist, rhos = [], []

    def inv(W, s):
        A = s * eye - W * W
        M = spla.inv(A)
        if len(hist) >= 2:
            rhos.append(np.abs(eye - A @ (2 * hist[-1] - hist[-2])).sum(1).max())
        hist.append(M)
        del hist[:-2]
        return M + 1e-16

    o._inv = inv
    if which == "s1":
        W0 = np.zeros((d, d))
    else:
        W0 = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                  "traj_d1000.npz"))["W_K2000"].copy()
    t = time.time()
    o.minimize(W0, 1.0, steps, 1.0, 3e-4, tol=-1)
    r = np.array(rhos)
    q = np.quantile(r, [0.5, 0.9, 0.99, 1.0])
    print(f"{which}: {len(r)} steps, rho quantiles (50/90/99/100%) {q}, rho^3 at the median {q[0] ** 3:.1e}, "
          f"share with rho^4 > 1e-16: {(r ** 4 > 1e-16).mean():.3f}  ({time.time() - t:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
