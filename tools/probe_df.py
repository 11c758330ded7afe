"""Per-task timing of the one-launch fast-slot inverse (experiments/dfinv.hip), development tool:
python tools/probe_df.py [d] [passes] -- runs a few cov-mode slots with MIDAGMA_DF_STAMPS set,
then prints per task type the compute and wait times and the outer steps' timeline of the
last launch (100 MHz device clock).  The one-launch inverse exists in the experiments build
only (midagma_amd/libmidagma_hip_exp.so, `make -C midagma_amd/csrc exp`)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MIDAGMA_DF_STAMPS"] = "1"
os.environ.setdefault("MIDAGMA_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "midagma_amd", "libmidagma_hip_exp.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from midagma_amd import _lib  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402
from midagma_amd.solver import HipSolver  # noqa: E402

NAMES = ["resid", "pass", "U", "V", "diag", "trail"]


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    X -= X.mean(0)
    s = HipSolver(d, "l2", "cov")
    s.set_cov(X.T @ X / X.shape[0])
    s.begin(np.zeros((d, d)), 1.0, 5000, 1.0, 3e-4, tol=-1.0)
    s.run_slots(30)
    s.sync()
    L = _lib.load()
    D = (d + 127) // 128 * 128
    nwg = torch.cuda.get_device_properties(0).multi_processor_count * int(os.environ.get("MIDAGMA_EXP_DF_PER_CU", "2"))
    f = L.midagma_debug_df_plan
    f.restype = C.c_int
    f.argtypes = [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_void_p,
                  C.c_void_p, C.POINTER(C.c_int)]
    est, nt = C.c_double(), C.c_int64()
    assert f(D, passes, nwg, C.byref(est), C.byref(nt), None, None, None) == 0
    tasks = np.zeros(nt.value * 12, dtype=np.int32)
    woff = np.zeros(nwg + 1, dtype=np.int32)
    f(D, passes, nwg, None, None, tasks.ctypes.data, woff.ctypes.data, None)
    tasks = tasks.reshape(-1, 12)
    g = L.midagma_debug_df_stamps
    g.restype = C.c_int64
    g.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    st = np.zeros(3 * len(tasks), dtype=np.uint64)
    n = g(s.h, st.ctypes.data, len(st))
    assert n >= 3 * len(tasks), n
    st = st[:3 * len(tasks)].reshape(-1, 3).astype(np.float64) * 0.01  # us
    t0 = st[:, 0].min()
    st -= t0
    comp = st[:, 2] - st[:, 1]
    wait = st[:, 1] - st[:, 0]
    print(f"d={d} D={D} passes={passes} nwg={nwg}: {len(tasks)} tasks, planned {est.value:.1f} us, "
          f"launch span {st[:, 2].max():.1f} us")
    for ty in range(6):
        m = tasks[:, 0] == ty
        if m.any():
            print(f"  {NAMES[ty]:6s} n={m.sum():5d}  compute mean {comp[m].mean():6.2f} p90 {np.percentile(comp[m], 90):6.2f}"
                  f"  wait mean {wait[m].mean():6.2f} max {wait[m].max():7.2f}  first go {st[m, 1].min():7.1f}"
                  f"  last done {st[m, 2].max():7.1f}")
    K2 = D // 256
    for gg in range(K2):
        row = []
        for ty in range(6):
            m = (tasks[:, 0] == ty) & (tasks[:, 1] == gg)
            if m.any():
                row.append(f"{NAMES[ty]} {st[m, 1].min():6.1f}-{st[m, 2].max():6.1f}")
        print(f"  g={gg}: " + "  ".join(row))
    busy = comp.sum() / (nwg * st[:, 2].max())
    print(f"  busy fraction (compute / (nwg x span)) {busy:.2f}; per-workgroup task count "
          f"{np.diff(woff).min()}-{np.diff(woff).max()}")
    s.close()


if __name__ == "__main__":
    main()
