"""In-library RCCL all-reduce (ABI 7) against the plain single-process slots, world size 1
(development tool): steps/s of run_slots with and without the solver's
communicator (the all-reduce captured in the slot graph) and of the host-driven protocol
(step_partial -> dist.all_reduce -> step_finish), at logistic d=1000 n=1e4 and at the config-4
per-rank shard of 8 GPUs (l2, d=1000, n=125k).

    python tools/probe_comm.py [K]
"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from midagma_amd.solver import HipSolver  # noqa: E402


def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def make(loss, d, n, lib):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, d))
    if loss == "logistic":
        X = (X > 0).astype(np.float64)
    else:
        X -= X.mean(0)
    s = HipSolver(d, loss, "data", device=0)
    s.set_data(X, n_global=n)
    s.set_cov(np.eye(d) if loss == "l2" else X.T @ X / n)
    if lib:
        s.attach_comm(None)
    return s


def timed(s, K, host):
    d = s.d
    s.begin(np.zeros((d, d)), 1.0, K + 40, 1.0, 3e-4, tol=-1.0)
    if host:
        zt, ctx = s.torch_zbuf()

        def steps(k):
            for _ in range(k):
                s.step_partial()
                with ctx():
                    dist.all_reduce(zt)
                s.step_finish()
    else:
        def steps(k):
            s.run_slots(k)
    steps(10)
    s.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(K)
    s.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    W = np.zeros((d, d))
    r = s.end(W)
    return K / dt, W, r.iters


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    for loss, d, n, k in (("logistic", 1000, 10_000, K), ("l2", 1000, 125_000, max(20, K // 4))):
        out = {}
        for rep in range(2):
            for kind in ("plain", "library", "host"):
                s = make(loss, d, n, kind == "library")
                v, W, it = timed(s, k, kind == "host")
                s.close()
                out.setdefault(kind, []).append(v)
                if rep == 0:
                    out[kind + "_W"] = W
        same = {k: bool(np.array_equal(out[k + "_W"], out["plain_W"])) for k in ("library", "host")}
        same["host_max_dW"] = float(np.abs(out["host_W"] - out["plain_W"]).max())
        line = ", ".join(f"{kk} {np.mean(out[kk]):.1f} ({' / '.join(f'{x:.1f}' for x in out[kk])})"
                         for kk in ("plain", "library", "host"))
        print(f"{loss} d={d} n={n} K={k}: steps/s {line}; library/plain {np.mean(out['library']) / np.mean(out['plain']):.4f}"
              f", host/plain {np.mean(out['host']) / np.mean(out['plain']):.4f}; W bit-identical: {same}", flush=True)
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
