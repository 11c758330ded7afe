"""Time the GPU SEM generator: X (n x d) of an ER(s0=d) linear-Gaussian SEM, cold and warm.

    python tools/probe_sem.py [--d 1000] [--n 1000000] [--reps 3] [--sem gauss]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--d", type=int, default=1000)
    p.add_argument("--n", type=int, default=1000000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--sem", default="gauss")
    a = p.parse_args()
    import torch
    from midagma_amd.simulate import simulate_er_dag, simulate_weights
    from midagma_amd.utils import simulate_linear_sem_gpu
    from oracle.sem_oracle import topological_levels
    rng = np.random.default_rng(0)
    W = simulate_weights(simulate_er_dag(a.d, a.d, rng), rng)
    lv = topological_levels(W)
    print(f"d={a.d} n={a.n} levels={len(lv)} sizes={[len(x) for x in lv][:12]} nnz={int((W != 0).sum())}", flush=True)
    X = torch.empty((a.n, a.d), dtype=torch.float64, device="cuda")
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        simulate_linear_sem_gpu(W, a.n, a.sem, seed=5, device=0, out=X)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        print(f"rep {r}: {t * 1e3:.2f} ms  output {8.0 * a.n * a.d / t / 1e9:.0f} GB/s", flush=True)
    # reference point: torch randn + dense GEMM with (I - W)^-1 (what bench used before)
    Binv = torch.from_numpy(np.linalg.inv(np.eye(a.d) - W)).cuda()
    for r in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        E = torch.randn(a.n, a.d, dtype=torch.float64, device="cuda")
        Y = E @ Binv
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        del E, Y
        print(f"torch randn+GEMM rep {r}: {t * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
