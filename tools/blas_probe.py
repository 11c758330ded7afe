"""Development probe: fp64 GEMM timings of the config-5 fc1 shapes (torch/rocBLAS), including
a chunked (split-K by bmm) weight gradient."""
import time

import torch

torch.set_default_dtype(torch.float64)
X = torch.randn(1000, 200, device="cuda")
G = torch.randn(1000, 2000, device="cuda")


def timed(f, reps=200):
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


print(f"dW = G^T X            {timed(lambda: G.t() @ X):.1f} us", flush=True)
print(f"dW^T = X^T G          {timed(lambda: X.t() @ G):.1f} us", flush=True)
for c in (2, 4, 5, 8, 10, 20):
    r = 1000 // c
    Gc, Xc = G.view(c, r, 2000), X.view(c, r, 200)
    print(f"chunked c={c:2d} bmm+sum {timed(lambda: torch.bmm(Gc.transpose(1, 2), Xc).sum(0)):.1f} us", flush=True)
ref = G.t() @ X
for c in (5, 10):
    r = 1000 // c
    d = torch.bmm(G.view(c, r, 2000).transpose(1, 2), X.view(c, r, 200)).sum(0)
    print(c, "max rel diff", ((d - ref).abs().max() / ref.abs().max()).item())
