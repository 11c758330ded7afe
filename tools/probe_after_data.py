"""Config 5 step rate in the same process right after bench.py's config-4 data leg (development
tool): isolates whether the data leg leaves state that slows the MLP leg, and whether a slow MLP
leg is host-bound (process CPU time per step) or device-bound.

    python tools/probe_after_data.py [data steps] [first]   (first: one MLP leg before the data leg)
"""
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def mlp_leg(args):
    c0, t0 = time.process_time(), time.perf_counter()
    r = bench.bench_mlp(args, 0, with_cpu=False)
    c1, t1 = time.process_time(), time.perf_counter()
    print(f"config5 leg: {r['value']:.0f} steps/s (timed call); whole leg {t1 - t0:.2f} s wall, "
          f"{c1 - c0:.2f} s process CPU", flush=True)


def pre(kind):
    """One piece of the data leg alone, before the MLP leg's first use."""
    import numpy as np
    import torch
    from midagma_amd.solver import HipSolver
    if kind in ("xprio", "xprio_graph"):  # fork / join between a high-priority stream and the current one
        hi = torch.cuda.Stream(priority=-1)
        cur = torch.cuda.current_stream()
        a = torch.ones(1 << 20, device="cuda:0")

        def body():
            hi.wait_stream(cur)
            with torch.cuda.stream(hi):
                a.mul_(1.0)
            cur.wait_stream(hi)
            a.add_(0.0)
        if kind == "xprio":
            for _ in range(50):
                body()
        else:
            g = torch.cuda.CUDAGraph()
            body()
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                body()
            for _ in range(50):
                g.replay()
        torch.cuda.synchronize()
    elif kind == "data_leg":  # the bench's data leg at the shard size of MIDAGMA_N (default 1e6)
        args = types.SimpleNamespace(d=1000, n=int(os.environ.get("MIDAGMA_N", "1000000")), seed=0, steps=10,
                                     warmup=1, profile_reps=3)
        r = bench.bench_data(args, 1, 0, 0)
        print(f"   data leg n={args.n}: {r['value']:.2f} steps/s ({r['ms_per_step']:.3f} ms)", flush=True)
    elif kind == "prio":  # a high-priority stream, used and destroyed
        st = torch.cuda.Stream(priority=-1)
        with torch.cuda.stream(st):
            torch.ones(1000, device="cuda:0").sum()
        torch.cuda.synchronize()
        del st
    elif kind == "shard":
        X, n_k, t = bench.make_shard(1000, 1_000_000, 1, 0, 0, torch.device("cuda", 0))
        del X
        torch.cuda.empty_cache()
    elif kind.startswith("solver"):
        n = 1_000_000 if kind == "solver_big" else 100_000
        X = torch.randn(n, 1000, dtype=torch.float64, device="cuda:0")
        s = HipSolver(1000, "l2", "data")
        s.set_data(X, n_global=n)
        del X
        torch.cuda.empty_cache()
        s.begin(np.zeros((1000, 1000)), 1.0, 20, 1.0, 3e-4, tol=-1.0)
        s.run_slots(6)
        s.sync()
        s.close()
    torch.cuda.synchronize()
    print(f"-- after {kind}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and not sys.argv[1].isdigit():
        pre(sys.argv[1])
        if len(sys.argv) > 2 and sys.argv[2].startswith("prio"):
            # the MLP log-det's side stream at a given torch priority (torch.cuda.Stream range)
            import torch
            import midagma_amd.nonlinear as nl
            pr = int(sys.argv[2][4:])
            nl._SIDE[0] = torch.cuda.Stream(device=0, priority=pr)
            print(f"   MLP side stream priority {pr} (range {torch.cuda.Stream.priority_range()})", flush=True)
        mlp_leg(types.SimpleNamespace(seed=0, mlp_steps=2000))
        sys.exit(0)
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    args = types.SimpleNamespace(d=1000, n=1_000_000, seed=0, steps=K, warmup=1, profile_reps=3, mlp_steps=2000)
    if len(sys.argv) > 2 and sys.argv[2] == "first":
        mlp_leg(args)
    r = bench.bench_data(args, 1, 0, 0)
    print(f"data leg: {r['value']:.2f} steps/s", flush=True)
    for _ in range(2):
        mlp_leg(args)
