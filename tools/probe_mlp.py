"""Config 5 step-time variants (development tool): DagmaNonlinear.minimize at dims [200, 10, 1],
n = 1000, with the log-det on a side stream or not (MIDAGMA_NO_OVERLAP) and with the warm-started
fast log-det or every step exact (MIDAGMA_NO_LDFAST); prints steps/s and the fast path's share.

    python tools/probe_mlp.py [K]
    python tools/probe_mlp.py K fused  # fc1 and the tail fused on the MFMA (ABI 7) against the ABI-6 sequence
    python tools/probe_mlp.py K pre    # the fast variant after each of the bench's earlier legs' solvers
                                       # (cov d=1000, cov d=5000, data d=1000 n=1e5) in the same process
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402


def run(K, overlap, fast):
    for k in ("MIDAGMA_NO_OVERLAP", "MIDAGMA_NO_LDFAST"):
        os.environ.pop(k, None)
    if not overlap:
        os.environ["MIDAGMA_NO_OVERLAP"] = "1"
    if not fast:
        os.environ["MIDAGMA_NO_LDFAST"] = "1"
    d, n = 200, 1000
    X, _, _ = make_dataset(d, n, seed=0)
    torch.manual_seed(0)
    model = DagmaMLP(dims=[d, 10, 1]).to("cuda:0")
    with torch.no_grad():
        model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * d))
    dn = DagmaNonlinear(model, device=0)
    dn.X = torch.from_numpy(X).to("cuda:0")
    dn.checkpoint = 10 ** 9
    dn.minimize(20, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dn.minimize(K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = dn._ld.stats() if fast and getattr(dn, "_ld", None) is not None else None
    print(f"overlap={int(overlap)} ldfast={int(fast)}: {K / dt:.0f} steps/s ({dt / K * 1e6:.1f} us/step)"
          f"{'' if st is None else f'  steps {st[0]}, Gauss-Jordan {st[1]}'}", flush=True)


def pre_leg(kind):
    """One of the bench's earlier solvers, run and closed in this process."""
    from midagma_amd.solver import HipSolver
    if kind.startswith("cov"):
        d = int(kind[3:])
        X, _, _ = make_dataset(d, 2 * d, seed=0)
        X -= X.mean(0)
        s = HipSolver(d, "l2", "cov")
        s.set_cov(X.T @ X / X.shape[0])
        K = 2000 if d <= 1000 else 20
    else:
        d, n = 1000, 100_000
        X = np.random.default_rng(0).standard_normal((n, d))
        s = HipSolver(d, "l2", "data")
        s.set_data(X, n_global=n)
        K = 20
    s.begin(np.zeros((d, d)), 1.0, K + 10, 1.0, 3e-4, tol=-1.0)
    s.run_slots(K)
    s.sync()
    s.close()
    torch.cuda.synchronize()
    print(f"-- after {kind}:", flush=True)


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    if len(sys.argv) > 2 and sys.argv[2] == "queues":
        # the log-det side stream created after 0..7 other streams (HIP maps streams onto
        # GPU_MAX_HW_QUEUES hardware queues round-robin)
        import midagma_amd.nonlinear as nl
        keep = []
        for extra in range(8):
            nl._SIDE.clear()
            print(f"-- side stream created after {extra} extra streams:", flush=True)
            run(K, True, True)
            keep.append(torch.cuda.Stream())
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "ramp":
        # the same run repeated, then after a 2 s MFMA burn, with the engine clock read around each
        # run: is the first solver's slowness the process's first work or the clock it starts at?
        import subprocess

        def clocks(tag):
            try:
                r = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=20)
                ln = [x.strip() for x in r.stdout.splitlines() if "sclk" in x or "fclk" in x or "mclk" in x]
                print(f"   clocks {tag}: {' | '.join(ln[:3])}", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"   clocks {tag}: n/a ({e})", flush=True)
        for rep in range(4):
            clocks(f"before run {rep}")
            run(K, True, True)
        a = torch.randn(8192, 8192, dtype=torch.float64, device="cuda:0")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            a = a @ a * 1e-4
            torch.cuda.synchronize()
        print("-- after a 2 s DGEMM burn:", flush=True)
        for rep in range(2):
            clocks(f"after burn run {rep}")
            run(K, True, True)
        time.sleep(5)
        print("-- after 5 s idle:", flush=True)
        clocks("after idle")
        run(K, True, True)
        run(K, False, True)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "fused":  # fc1 + tail on the MFMA (ABI 7) or the ABI-6 sequence
        import midagma_amd.nonlinear as nl
        for rep in range(2):
            for f in (True, False):
                nl.FUSED_TAIL = f
                print(f"-- FUSED_TAIL={f}", flush=True)
                run(K, True, True)
                run(K, False, True)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "linsplit":  # split-K count of dZ^T X
        import midagma_amd.nonlinear as nl
        for rep in range(2):
            for ks in (4, 8, 2):
                nl.LIN_SPLIT = ks
                print(f"-- LIN_SPLIT={ks}", flush=True)
                run(K, True, True)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "serial":  # one stream (the log-det in sequence)
        run(K, False, True)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "fast":
        run(K, True, True)
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "pre":
        run(K, True, True)
        for kind in ("cov1000", "cov5000", "data"):
            pre_leg(kind)
            run(K, True, True)
            run(K, False, True)
        sys.exit(0)
    for overlap in (True, False):
        for fast in (True, False):
            run(K, overlap, fast)
