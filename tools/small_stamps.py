"""Phase breakdown of the small-d persistent slot loop (csrc/small.hip; diagnostic).

Loads the kstamps build (`make -C midagma_amd/csrc kstamps`), runs the default stage-1 loop at d
(default 20) from W = 0 and prints the mean shader-clock cycles per slot of each phase, converted
to microseconds with the launches' real-time span.

    python tools/small_stamps.py [d] [slots]
"""
import ctypes as C
import os
import sys
import time

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
os.environ["MIDAGMA_LIB"] = os.path.join(_REPO, "midagma_amd", "libmidagma_hip_kstamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from midagma_amd import _lib  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402
from midagma_amd.solver import HipSolver  # noqa: E402

PHASES = {0: "table read + (sI - W o W)^T", 7: "inverse: X0, R = I - S X0, |R| (barrier)",
          8: "inverse: pass 1 (Y, R^2, images, barrier)", 9: "inverse: pass 2", 1: "inverse: rest (3rd pass / GJ)",
          2: "score product", 3: "domain + ckpt sums, barrier", 4: "controller (thread 0), barrier",
          5: "G_obj + Adam + update, barrier"}


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    L = _lib.load()
    buf = (C.c_ulonglong * 16)()  # [0..11] phases, [12] slots, [13] real time
    X, _, _ = make_dataset(d, 1000, seed=0)
    X -= X.mean(0)
    s = HipSolver(d, "l2", "cov")
    s.set_cov(X.T @ X / X.shape[0])
    W = np.zeros((d, d))
    s.minimize(W, 1.0, 200, 1.0, 3e-4, tol=-1.0)  # warm (code objects, clocks)
    assert L.midagma_debug_small_stamps(buf) == 0
    W = np.zeros((d, d))
    t0 = time.perf_counter()
    r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0)
    dt = time.perf_counter() - t0
    assert L.midagma_debug_small_stamps(buf) == 0
    s.close()
    a = np.array(buf, dtype=np.float64)
    n, span = a[12], a[13] * 1e-8  # 100 MHz
    cyc = sum(a[p] for p in PHASES)
    hz = cyc / span if span > 0 else 0.0
    print(f"d={d}: {K} steps in {dt * 1e3:.1f} ms wall ({K / dt:.0f} steps/s); {int(n)} slots stamped, "
          f"{int(a[6])} on Gauss-Jordan; clock {hz / 1e9:.2f} GHz (stamped cycles / real-time span)", flush=True)
    for p, name in PHASES.items():
        print(f"  {name:34s} {a[p] / n:9.0f} cycles  {a[p] / n / hz * 1e6 if hz else 0:7.3f} us  "
              f"{100 * a[p] / cyc:5.1f} %")
    print(f"  {'slot':34s} {cyc / n:9.0f} cycles  {cyc / n / hz * 1e6 if hz else 0:7.3f} us")


if __name__ == "__main__":
    main()
