"""Config-5 GEMM shapes under torch's two BLAS back ends (diagnostic): fc1's X W1^T
(1000 x 200 @ 200 x 2000) and the weight gradient's 4-way batched dZ^T X, f64, timed with HIP
events (best of 5 batches of 200)."""
import torch

dev = torch.device("cuda:0")
n, d, m1, ks = 1000, 200, 10, 4
X = torch.randn(n, d, dtype=torch.float64, device=dev)
W1 = torch.randn(d * m1, d, dtype=torch.float64, device=dev)
dZ = torch.randn(n, d * m1, dtype=torch.float64, device=dev)


def t(fn, reps=200):
    best = 1e9
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


for lib in ("hipblas", "ck", "hipblaslt"):
    try:
        if lib != "default":
            torch.backends.cuda.preferred_blas_library(lib)
        else:
            torch.backends.cuda.preferred_blas_library("default")
        cur = torch.backends.cuda.preferred_blas_library()
        f = t(lambda: X @ W1.t())
        r = n // ks
        g = t(lambda: torch.bmm(dZ.view(ks, r, -1).transpose(1, 2), X.view(ks, r, -1)))
        g1 = t(lambda: dZ.t() @ X)
        # layouts the tail kernels would have to adopt: Z^T = W1 X^T with X^T stored once (X is
        # fixed over a fit), and Z = X W1t with W1^T stored (one transposed copy per step)
        XT = X.t().contiguous()
        W1t = W1.t().contiguous()
        ft = t(lambda: W1 @ XT)
        fw = t(lambda: X @ W1t)
        print(f"{lib:10s} ({cur}): fwd {f:7.2f} us  fwd Z^T=W1 X^T {ft:7.2f} us  fwd X W1t {fw:7.2f} us  "
              f"bwd bmm4 {g:7.2f} us  bwd mm {g1:7.2f} us", flush=True)
    except Exception as e:  # noqa: BLE001
        print(lib, "failed:", repr(e)[:200], flush=True)
