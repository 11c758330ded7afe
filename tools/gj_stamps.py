"""Diagnostic: per-step cycle breakdown of the GJ diagonal-owner workgroup (stamps build)."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MIDAGMA_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                         "midagma_amd", "libmidagma_hip_stamps.so")
import numpy as np
import torch  # noqa
from midagma_amd import _lib
from midagma_amd.simulate import make_dataset
from midagma_amd.solver import HipSolver
d = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
X, _, _ = make_dataset(d, 2 * d, seed=0)
X -= X.mean(0)
s = HipSolver(d)
s.set_cov(X.T @ X / X.shape[0])
s.begin(np.zeros((d, d)), 1.0, 100, 1.0, 3e-4, tol=-1.0)
s.run_slots(20)
s.sync()
buf = (C.c_ulonglong * (256 * 16))()
_lib.lib().midagma_debug_stamps(buf)
a = np.array(buf, dtype=np.float64).reshape(256, 16)
K = s.D // 32
print("step: load->T, T->C.T, C.T->inv start, inversion | X0 load, NS it0 half, per-iter rest, iters")
for k in range(0, K - 1, max(1, (K - 1) // 10)):
    t = a[k]
    it = max(int(t[7]), 1)
    print(k, int(t[1] - t[0]), int(t[2] - t[1]), int(t[3] - t[2]), int(t[4] - t[3]), "|",
          int(t[5] - t[3]), int(t[6] - t[5]), int((t[4] - t[6]) / it), it)
