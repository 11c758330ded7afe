"""Which f64 MFMA C/D layout is right? (h at d=20 vs the oracle)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch  # noqa
from midagma_amd.solver import HipSolver
from oracle.dagma_oracle import h_logdet
rng = np.random.default_rng(0)
for d in (20, 100):
    W = rng.uniform(-1, 1, (d, d)) * 0.05
    s = HipSolver(d)
    h, G = s.h_value(W, 1.0)
    hr, Gr = h_logdet(W, 1.0)
    print(os.environ.get("MIDAGMA_LIB", "default"), d, "h err", abs(h - hr), "G err", np.abs(G - Gr).max(), flush=True)
