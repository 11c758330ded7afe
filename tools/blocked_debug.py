"""Diagnostic: per-outer-block residual bounds of the fast blocked inverse after a few slots."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401
from midagma_amd import _lib
from midagma_amd.simulate import make_dataset
from midagma_amd.solver import HipSolver

d = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
steps = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["2", "20", "200"])]
X, _, _ = make_dataset(d, max(2 * d, 2000), seed=0)
X -= X.mean(0)
s = HipSolver(d)
s.set_cov(X.T @ X / X.shape[0])
s.begin(np.zeros((d, d)), 1.0, 100000, 1.0, 3e-4, tol=-1.0)
L = _lib.lib()
f = L.midagma_debug_blocked
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int64]
buf = (C.c_double * 4096)()
done = 0
for k in steps:
    s.run_slots(k - done)
    s.sync()
    done = k
    n = f(s.h, buf, 4096)
    r = s.poll()
    a = np.array(buf[: n * 6]).reshape(n, 6) if n > 0 else None
    print(f"after {k} slots: iters={r.iters} status={r.status}")
    if a is not None:
        for g in range(n):
            print(f"  block {g}: done={int(a[g, 0])} rho=" + " ".join(f"{v:.2e}" for v in a[g, 1:]))
