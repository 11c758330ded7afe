"""Phase breakdown of the cov slot's latency-bound launches (diagnostic).

Loads the kstamps build (`make -C midagma_amd/csrc kstamps`: csrc/kstamps.h), runs fast cov
slots at d (default 1000) and prints, per kernel kind, the mean time a workgroup spends in each
phase (wave 0's s_memtime, converted with the s_memrealtime 100 MHz span of the same workgroups)
and the mean workgroup lifetime; compare with the launch's duration in the rocprofv3 summary.

    python tools/kstamps.py [d] [slots]
"""
import ctypes as C
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
os.environ["MIDAGMA_LIB"] = os.path.join(_REPO, "midagma_amd", "libmidagma_hip_kstamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from midagma_amd import _lib  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402
from midagma_amd.solver import HipSolver  # noqa: E402

KINDS = ["nm_resid", "nm_pass", "binv_panel", "binv_trail"]
PHASES = {"nm_resid": ["operands + warm start loaded", "MFMA + split-K sum", "stores drained"],
          "nm_pass": ["rho (row partials reduced; operands in flight)", "MFMAs + split-K sums", "stores drained"],
          "binv_panel": ["tile product (chunk loads + MFMA)", "stores drained"],
          "binv_trail": ["whole tile (C0 load, chunks, MFMA, stores drained)"]}
NP = 6


def read(L):
    buf = (C.c_ulonglong * (4 * (NP + 2)))()
    assert L.midagma_debug_kstamps(buf) == 0
    return np.array(buf, dtype=np.float64).reshape(4, NP + 2)


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    L = _lib.load()
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    X -= X.mean(0)
    s = HipSolver(d, "l2", "cov")
    s.set_cov(X.T @ X / X.shape[0])
    s.begin(np.zeros((d, d)), 1.0, K + 200, 1.0, 3e-4, tol=-1.0)
    s.run_slots(50)
    s.sync()
    read(L)  # zero
    s.run_slots(K)
    s.sync()
    a = read(L)
    s.close()
    print(f"d={d}, {K} slots (fast slots with their GJ slots): mean per workgroup, wave 0's clock", flush=True)
    for k, name in enumerate(KINDS):
        n = a[k, NP]
        if n == 0:
            print(f"{name}: no samples")
            continue
        cyc = a[k, :NP]
        total_cyc = cyc.sum()
        span_us = a[k, NP + 1] / n / 100.0  # s_memrealtime: 100 MHz
        ghz = total_cyc / n / (span_us * 1e3) if span_us > 0 else float("nan")
        parts = ", ".join(f"{p}: {c / n / ghz / 1e3:.2f} us" for p, c in zip(PHASES[name], cyc) if c > 0)
        print(f"{name}: {int(n)} workgroups, lifetime {span_us:.2f} us (clock {ghz:.2f} GHz): {parts}", flush=True)


if __name__ == "__main__":
    main()
