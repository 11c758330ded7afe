"""Probe (experiments build): the cov slot with the score GEMM forked beside the blocked inverse and
confined to the first MIDAGMA_EXP_GEMM_SES shader engines of each XCD (launch_gemm_cupart), set by
the environment of this process (knobs are read once).  Prints steps/s at each d and a hash of W
after 300 steps from W = 0 (the tile bodies are the product's: W must be bit-identical)."""
import hashlib
import os
import sys
import time

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
os.environ.setdefault("MIDAGMA_LIB", os.path.join(_REPO, "midagma_amd", "libmidagma_hip_exp.so"))
import numpy as np
import torch  # noqa: F401

from midagma_amd.simulate import make_dataset
from midagma_amd.solver import HipSolver

tag = " ".join(f"{k[12:]}={os.environ[k]}" for k in sorted(os.environ) if k.startswith("MIDAGMA_EXP_")) or "product"
for d in [int(x) for x in sys.argv[1:]] or [1000]:
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    X -= X.mean(0)
    cov = X.T @ X / X.shape[0]
    s = HipSolver(d, "l2", "cov")
    s.set_cov(cov)
    W = np.zeros((d, d))
    s.minimize(W, 1.0, 300, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
    h = hashlib.sha256(W.tobytes()).hexdigest()[:16]
    K = 2000 if d <= 1000 else 400
    s.begin(np.zeros((d, d)), 1.0, K + 1100, 1.0, 3e-4, tol=-1.0)
    s.run_slots(20)
    s.sync()
    t0 = time.perf_counter()
    s.run_slots(K)
    s.sync()
    dt = time.perf_counter() - t0
    s.close()
    print(f"{tag} d={d}: {K / dt:.1f} steps/s ({dt / K * 1e6:.1f} us/step)  W(300) sha {h}", flush=True)
