"""Small-d cov-mode Adam steps/s on the persistent workgroup (csrc/small.hip; diagnostic).

Runs each d from W = 0 for K slots (lambda1 = 0.03, checkpoint every 1000, tol < 0) on the
library MIDAGMA_LIB names (default: the product build) and prints steps/s, best of 3.

    python tools/probe_small.py [K] [d ...]
"""
import os
import sys
import time

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from midagma_amd import _lib  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402
from midagma_amd.solver import HipSolver  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    ds = [int(a) for a in sys.argv[2:]] or [10, 16, 20, 32, 48, 64]
    _lib.load()
    lib = os.path.basename(os.environ.get("MIDAGMA_LIB", "libmidagma_hip.so"))
    for d in ds:
        X, _, _ = make_dataset(d, 1000, seed=0)
        X -= X.mean(0)
        s = HipSolver(d, "l2", "cov")
        s.set_cov(X.T @ X / X.shape[0])
        s.minimize(np.zeros((d, d)), 1.0, 200, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
        best = 0.0
        for _ in range(3):
            W = np.zeros((d, d))
            t = time.perf_counter()
            r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=1000)
            dt = time.perf_counter() - t
            best = max(best, r.iters / dt)
        print(f"{lib} d={d}: {best:9.0f} steps/s  iters {r.iters}  |W| {np.abs(W).sum():.12e}", flush=True)
        s.close()


if __name__ == "__main__":
    main()
