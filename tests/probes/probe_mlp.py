"""Config 5: DagmaNonlinear Adam steps/s at dims [d, 10, 1], n=1000 on the GPU (and the CPU
oracle at a few thread counts with --cpu).

    python tools/probe_mlp.py [--d 200] [--steps 300] [--cpu]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--d", type=int, default=200)
    p.add_argument("--n", type=int, default=1000)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--cpu", action="store_true")
    a = p.parse_args()
    import torch
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    from midagma_amd.simulate import make_dataset
    X, _, _ = make_dataset(a.d, a.n, seed=0)
    torch.manual_seed(0)
    model = DagmaMLP(dims=[a.d, 10, 1]).to("cuda:0")
    with torch.no_grad():
        model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * a.d))
    dn = DagmaNonlinear(model, device=0)
    dn.X = torch.from_numpy(X).to("cuda:0")
    dn.checkpoint = 10 ** 9
    dn.minimize(20, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dn.minimize(a.steps, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"gpu d={a.d} n={a.n}: {a.steps / dt:.1f} steps/s ({dt / a.steps * 1e3:.3f} ms/step)", flush=True)
    if a.cpu:
        from oracle.mlp_oracle import OracleMLP, load_params, nonlinear_minimize
        for th in (1, 4, 8, 16):
            torch.set_num_threads(th)
            m = OracleMLP([a.d, 10, 1])
            load_params(m, {k: v.detach().cpu().numpy() for k, v in model.state_dict().items() if k != "I"})
            Xc = torch.from_numpy(X)
            nonlinear_minimize(m, Xc, 3, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
            K = 30
            t0 = time.perf_counter()
            nonlinear_minimize(m, Xc, K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
            dt = time.perf_counter() - t0
            print(f"cpu oracle d={a.d} threads={th}: {K / dt:.1f} steps/s ({dt / K * 1e3:.2f} ms/step)", flush=True)


if __name__ == "__main__":
    main()
