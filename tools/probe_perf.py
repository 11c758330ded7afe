"""Quick GPU timing probe (development tool): steps/s of the slot at several sizes.

Loads the experiments build (midagma_amd/libmidagma_hip_exp.so, `make -C midagma_amd/csrc exp`):
its comparisons switch MIDAGMA_EXP_* knobs, which the product library compiles to their
defaults (csrc/knobs.h).  MIDAGMA_LIB overrides."""
import os
import sys
import time

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
os.environ.setdefault("MIDAGMA_LIB", os.path.join(_REPO, "midagma_amd", "libmidagma_hip_exp.so"))
import numpy as np
import torch  # noqa: F401

from midagma_amd.simulate import make_dataset
from midagma_amd.solver import HipSolver


def cov_case(d, n, warm, K):
    X, _, _ = make_dataset(d, n, seed=0)
    X -= X.mean(0)
    cov = X.T @ X / n
    s = HipSolver(d, "l2", "cov")
    s.set_cov(cov)
    s.begin(np.zeros((d, d)), 1.0, warm + K + 1000, 1.0, 3e-4, tol=-1.0)
    s.run_slots(warm)
    s.sync()
    t0 = time.perf_counter()
    s.run_slots(K)
    s.sync()
    dt = time.perf_counter() - t0
    r = s.poll()
    print(f"cov d={d}: {K / dt:.1f} steps/s  ({dt / K * 1e3:.3f} ms/step)  iters={r.iters} status={r.status}",
          {k: round(v, 4) for k, v in s.profile_parts(5).items()}, flush=True)
    s.close()


def data_case(d, n, warm, K, loss="l2"):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, d))
    s = HipSolver(d, loss, "data")
    s.set_data(X, n_global=n)
    if loss == "logistic":
        s.set_cov(X.T @ X / n)
    s.begin(np.zeros((d, d)), 1.0, warm + K + 1000, 1.0, 3e-4, tol=-1.0)
    s.run_slots(warm)
    s.sync()
    t0 = time.perf_counter()
    s.run_slots(K)
    s.sync()
    dt = time.perf_counter() - t0
    r = s.poll()
    pp = s.profile_parts(2)
    f = 2.0 * n * d * d
    print(f"data {loss} d={d} n={n}: {K / dt:.2f} steps/s ({dt / K * 1e3:.2f} ms/step) iters={r.iters}",
          {k: round(v, 4) for k, v in pp.items()},
          f"TF xw={f / pp['gemm_xw'] / 1e9:.1f} xty={f / pp['gemm_xty'] / 1e9:.1f}", flush=True)
    s.close()


def trek_case(d, seq, K):
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    X -= X.mean(0)
    s = HipSolver(d, "l2", "cov")
    s.set_cov(X.T @ X / X.shape[0])
    rng = np.random.default_rng(0)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    if seq == "tcc":
        s.set_trek_tcc(pairs, mode="opt", weight=0.1)
    else:
        s.set_trek(pairs, seq, agg="mean", mode="opt", weight=0.1, K_log=20)
    s.begin(np.zeros((d, d)), 1.0, K + 1000, 1.0, 3e-4, tol=-1.0)
    s.run_slots(3)
    s.sync()
    i0 = s.poll().iters
    t0 = time.perf_counter()
    s.run_slots(K)
    s.sync()
    dt = time.perf_counter() - t0
    it = s.poll().iters - i0  # Adam steps: a hand-back's re-run takes a slot of its own
    print(f"cov+{'TCC' if seq == 'tcc' else 'PST-' + seq} d={d}: {it / dt:.1f} steps/s ({dt / it * 1e3:.3f} ms/step)"
          f" over {K} slots, {it} steps, hand-backs {s.debug_handbacks()}", flush=True)
    s.close()


def trek_phase(d, warm, K, fix):
    """TCC on a fit's later W: `warm` untimed steps from W = 0, then K timed steps (hand-backs of
    the timed part only)"""
    os.environ["MIDAGMA_EXP_TCC_FIX"] = fix
    X, _, _ = make_dataset(d, 2 * d, seed=0)
    X -= X.mean(0)
    s = HipSolver(d, "l2", "cov")
    s.set_cov(X.T @ X / X.shape[0])
    rng = np.random.default_rng(0)
    iu = np.array(np.triu_indices(d, 1)).T
    pairs = iu[rng.uniform(size=len(iu)) < 0.3]
    s.set_trek_tcc(pairs, mode="opt", weight=0.1)
    s.begin(np.zeros((d, d)), 1.0, warm + K + 1000, 1.0, 3e-4, tol=-1.0)
    s.run_slots(warm)
    s.sync()
    b0, i0 = s.debug_handbacks(), s.poll().iters
    t0 = time.perf_counter()
    s.run_slots(K)
    s.sync()
    dt = time.perf_counter() - t0
    it = s.poll().iters - i0  # Adam steps: a hand-back's re-run takes a slot of its own
    print(f"MIDAGMA_EXP_TCC_FIX={fix} cov+TCC d={d} after {i0} steps: {it / dt:.1f} steps/s "
          f"({dt / it * 1e3:.3f} ms/step) over {K} slots, hand-backs {s.debug_handbacks() - b0}", flush=True)
    s.close()


def fit_case(d, n):
    from midagma_amd import DagmaLinear
    X, _, _ = make_dataset(d, n, seed=0)
    m = DagmaLinear("l2")
    t0 = time.perf_counter()
    m.fit(X.copy(), lambda1=0.03)
    dt = time.perf_counter() - t0
    its = [e["iters"] for e in m.minimize_log]
    print(f"fit d={d} n={n}: {dt:.2f} s, iters {its} = {sum(its)}, {dt / sum(its) * 1e3:.3f} ms/iter", flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "small"):
        cov_case(20, 1000, 50, 20000)
        for d in (10, 32, 48, 64):
            cov_case(d, 1000, 50, 10000)
        cov_case(65, 1000, 50, 5000)
        cov_case(200, 2000, 20, 500)
    if which in ("all", "d1000"):
        cov_case(1000, 2000, 10, 2000)
    if which == "dfcmp":  # the one-launch fast-slot inverse against the launch-per-phase one
        for d, K in ((1000, 2000), (500, 2000), (1400, 1000)):
            for df in ("1", "0"):
                os.environ["MIDAGMA_EXP_DF"] = df
                print(f"MIDAGMA_EXP_DF={df}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_DF")
    if which == "fusecmp":  # the cov score GEMM inside the last trailing launch, or apart
        big = len(sys.argv) > 2 and sys.argv[2] == "big"
        for d, K in (((2000, 200), (5000, 30)) if big else ((1000, 2000), (500, 2000), (1400, 1000))):
            for f in ("1", "0"):
                os.environ["MIDAGMA_EXP_FUSE_GEMM"] = f
                print(f"MIDAGMA_EXP_FUSE_GEMM={f}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_FUSE_GEMM")
    if which == "tccfast":  # TCC (2d > 128): the fast slots' short Noda chain with hand-back, or the whole gated chain
        for d in [int(x) for x in sys.argv[2:]] or [100, 300, 1000]:
            for f in ("5", "0", "4", "3"):
                os.environ["MIDAGMA_EXP_TCC_FAST_STEPS"] = f
                print(f"MIDAGMA_EXP_TCC_FAST_STEPS={f}", end=" ")
                trek_case(d, "tcc", 300 if d <= 300 else 60)
        os.environ.pop("MIDAGMA_EXP_TCC_FAST_STEPS")
    if which == "tccfix":  # TCC (2d > 128): the fixed-shift stage first (one inverse), or Noda from the warm start
        for d in [int(x) for x in sys.argv[2:]] or [20, 64, 100, 300, 1000]:
            for f, pre, hold in (("1", "1", "8"), ("1", "1", "1"), ("0", "1", "8")) if d > 64 else (("1", "1", "8"), ("0", "1", "8")):
                os.environ["MIDAGMA_EXP_TCC_FIX"] = f
                os.environ["MIDAGMA_EXP_TCC_FIX_PRE"] = pre
                os.environ["MIDAGMA_EXP_TCC_FIX_HOLD"] = hold
                print(f"MIDAGMA_EXP_TCC_FIX={f} MIDAGMA_EXP_TCC_FIX_PRE={pre} MIDAGMA_EXP_TCC_FIX_HOLD={hold}", end=" ")
                trek_case(d, "tcc", 2000 if d <= 64 else (300 if d <= 300 else 60))
        os.environ.pop("MIDAGMA_EXP_TCC_FIX")
        os.environ.pop("MIDAGMA_EXP_TCC_FIX_PRE")
    if which == "tccphase":  # TCC after a fit's first steps: the fixed-shift stage on / off
        for d, warm, K in ((100, 2000, 300), (100, 400, 100), (300, 1000, 200), (1000, 200, 40)):
            for f, pre, hold in (("1", "1", "8"), ("1", "1", "1"), ("0", "1", "8")):
                os.environ["MIDAGMA_EXP_TCC_FIX_PRE"] = pre
                os.environ["MIDAGMA_EXP_TCC_FIX_HOLD"] = hold
                print(f"MIDAGMA_EXP_TCC_FIX_PRE={pre} MIDAGMA_EXP_TCC_FIX_HOLD={hold}", end=" ")
                trek_phase(d, warm, K, f)
        os.environ.pop("MIDAGMA_EXP_TCC_FIX")
        os.environ.pop("MIDAGMA_EXP_TCC_FIX_PRE")
    if which == "tccd1000":  # d = 1000 later in a fit: the pre-step rule (easy threshold: default, 4) and no pre-step
        for easy, pre in (("0", "1"), ("4", "1"), ("0", "0")):
            os.environ["MIDAGMA_EXP_TCC_FIX_EASY"] = easy
            os.environ["MIDAGMA_EXP_TCC_FIX_PRE"] = pre
            print(f"MIDAGMA_EXP_TCC_FIX_EASY={easy} MIDAGMA_EXP_TCC_FIX_PRE={pre}", end=" ")
            trek_phase(1000, int(sys.argv[2]) if len(sys.argv) > 2 else 1500, 60, "1")
        os.environ.pop("MIDAGMA_EXP_TCC_FIX_EASY")
        os.environ.pop("MIDAGMA_EXP_TCC_FIX_PRE")
    if which == "tccfastblk":  # d = 1000: the fixed-stage inverse's fast blocks on / off, from W = 0 and later
        for fb in ("1", "0"):
            os.environ["MIDAGMA_EXP_TCC_FASTBLK"] = fb
            print(f"MIDAGMA_EXP_TCC_FASTBLK={fb}", end=" ")
            trek_case(1000, "tcc", 60)
            print(f"MIDAGMA_EXP_TCC_FASTBLK={fb}", end=" ")
            trek_phase(1000, int(sys.argv[2]) if len(sys.argv) > 2 else 1500, 60, "1")
        os.environ.pop("MIDAGMA_EXP_TCC_FASTBLK")
    if which == "tccphase1":  # one later-phase case (a kernel trace): d [warm K]
        a = [int(x) for x in sys.argv[2:]]
        d = a[0] if a else 100
        trek_phase(d, a[1] if len(a) > 1 else 2000, a[2] if len(a) > 2 else 300, "1")
    if which == "tccbinv":  # TCC (D2 >= 512): the shifted inverses on the blocked inverse (2), or the flat Gauss-Jordan (0)
        for d in [int(x) for x in sys.argv[2:]] or [300, 500, 1000]:
            for f in ("2", "0", "2", "0"):
                os.environ["MIDAGMA_EXP_TCC_BINV"] = f
                print(f"MIDAGMA_EXP_TCC_BINV={f}", end=" ")
                trek_case(d, "tcc", 300 if d <= 300 else 60)
        os.environ.pop("MIDAGMA_EXP_TCC_BINV")
    if which == "ctlfold":  # the fast cov slot's control in the last trailing launch, or its own launch
        for d, K in ((1000, 3000), (500, 3000), (1400, 1000), (2000, 300)):
            for f in ("1", "0", "1", "0"):
                os.environ["MIDAGMA_EXP_CTL_FOLD"] = f
                print(f"MIDAGMA_EXP_CTL_FOLD={f}", end=" ")
                cov_case(d, 2 * d, 20, K)
        os.environ.pop("MIDAGMA_EXP_CTL_FOLD")
    if which == "atfold":  # build_at folded into the previous slot's update, or its own launch
        for d, K in ((1000, 3000), (500, 3000), (1400, 1000), (2000, 300)):
            for f in ("1", "0", "1", "0"):
                os.environ["MIDAGMA_EXP_AT_FOLD"] = f
                print(f"MIDAGMA_EXP_AT_FOLD={f}", end=" ")
                cov_case(d, 2 * d, 20, K)
        os.environ.pop("MIDAGMA_EXP_AT_FOLD")
    if which == "splitcmp":  # split-K count of the cov score GEMM (fused into the last trail launch or apart)
        for d, K in ((1000, 2000), (1400, 1000)):
            for sp in ("4", "8", "2"):
                for f in ("1", "0"):
                    os.environ["MIDAGMA_EXP_COV_SPLIT"] = sp
                    os.environ["MIDAGMA_EXP_FUSE_GEMM"] = f
                    print(f"MIDAGMA_EXP_COV_SPLIT={sp} MIDAGMA_EXP_FUSE_GEMM={f}", end=" ")
                    cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_COV_SPLIT")
        os.environ.pop("MIDAGMA_EXP_FUSE_GEMM")
    if which == "splitmid":  # 128-tile grids of 81..196 tiles: split-K 1..4 of the fused cov score GEMM
        for d, K in ((1150, 1000), (1400, 1000), (1700, 600)):
            for sp in ("1", "2", "3", "4"):
                os.environ["MIDAGMA_EXP_COV_SPLIT"] = sp
                print(f"MIDAGMA_EXP_COV_SPLIT={sp}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_COV_SPLIT")
    if which == "padb2":  # cov mode, d > 256 with 256 not dividing the 128-padded size: D to 256-multiples
        for d, K in ((300, 3000), (600, 3000), (1150, 1000), (1400, 1000), (1700, 600)):
            for f in ("0", "1"):
                os.environ["MIDAGMA_EXP_COV_PAD_B2"] = f
                print(f"MIDAGMA_EXP_COV_PAD_B2={f}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_COV_PAD_B2")
    if which == "covla":  # large D cov mode: the trailing-update look-ahead (MIDAGMA_EXP_COV_LA)
        ds = [int(x) for x in sys.argv[2:]] or [2000, 5000]
        for d in ds:
            for f in ("0", "1"):
                os.environ["MIDAGMA_EXP_COV_LA"] = f
                print(f"MIDAGMA_EXP_COV_LA={f}", end=" ")
                cov_case(d, 2 * d, 3, 200 if d <= 2500 else 60)
        os.environ.pop("MIDAGMA_EXP_COV_LA")
    if which == "eagerla":  # large D cov mode: eager launches (MIDAGMA_EXP_EAGER) with / without the look-ahead
        ds = [int(x) for x in sys.argv[2:]] or [2000, 3000, 5000]
        for d in ds:
            for e, la in (("0", "0"), ("1", "0"), ("1", "1")):
                os.environ["MIDAGMA_EXP_EAGER"] = e
                os.environ["MIDAGMA_EXP_COV_LA"] = la
                print(f"MIDAGMA_EXP_EAGER={e} MIDAGMA_EXP_COV_LA={la}", end=" ")
                cov_case(d, 2 * d, 3, 200 if d <= 2500 else 60)
        os.environ.pop("MIDAGMA_EXP_EAGER")
        os.environ.pop("MIDAGMA_EXP_COV_LA")
    if which == "covforkall":  # cov mode at any blocked D: score GEMM on the main stream beside the inverse
        ds = [int(x) for x in sys.argv[2:]] or [300, 1000, 1400, 2000]
        splits = os.environ.pop("PROBE_SPLITS", "").split(",") if os.environ.get("PROBE_SPLITS") else [None]
        for d in ds:
            for f in ("0", "2"):
                for sp in (splits if f == "2" else [None]):
                    os.environ["MIDAGMA_EXP_COV_FORK"] = f
                    if sp:
                        os.environ["MIDAGMA_EXP_COV_SPLIT"] = sp
                    print(f"MIDAGMA_EXP_COV_FORK={f} split={sp}", end=" ")
                    cov_case(d, 2 * d, 10, 2000 if d <= 1000 else (1000 if d <= 1500 else 300))
                    os.environ.pop("MIDAGMA_EXP_COV_SPLIT", None)
        os.environ.pop("MIDAGMA_EXP_COV_FORK")
    if which == "covds":  # cov mode at the given d (knobs read once per process: set them in the environment)
        for d in [int(x) for x in sys.argv[2:]] or [1000]:
            cov_case(d, 10 * d, 200, 4000 if d <= 1000 else (1000 if d <= 2000 else 100))
    if which == "b2_512":  # cov mode: 512-wide outer blocks where 512 divides D (run with MIDAGMA_EXP_B2_512=0 / 1)
        for d in [int(x) for x in sys.argv[2:]] or [1000, 2000]:
            print(f"MIDAGMA_EXP_B2_512={os.environ.get('MIDAGMA_EXP_B2_512', '0')}", end=" ")
            cov_case(d, 2 * d, 10, 2000 if d <= 1000 else 300)
    if which == "smallshard":  # logistic / l2 data mode at n = 1e4: the in-sequence fast inverse or the fork
        for loss in ("logistic", "l2"):
            for rows, ff in (("16384", "0"), ("0", "0"), ("16384", "1")):
                os.environ["MIDAGMA_EXP_DATA_FAST_ROWS"] = rows
                os.environ["MIDAGMA_EXP_DATA_FORK_FAST"] = ff
                print(f"MIDAGMA_EXP_DATA_FAST_ROWS={rows} FORK_FAST={ff}", end=" ")
                data_case(1000, 10000, 5, 200, loss)
        os.environ.pop("MIDAGMA_EXP_DATA_FAST_ROWS")
        os.environ.pop("MIDAGMA_EXP_DATA_FORK_FAST")
    if which == "covfork":  # large D cov mode: score GEMM beside the inverse (MIDAGMA_EXP_COV_FORK)
        ds = [int(x) for x in sys.argv[2:]] or [2000, 5000]
        for d in ds:
            for f in ("0", "1"):
                os.environ["MIDAGMA_EXP_COV_FORK"] = f
                print(f"MIDAGMA_EXP_COV_FORK={f}", end=" ")
                cov_case(d, 2 * d, 3, 200 if d <= 2500 else 60)
        os.environ.pop("MIDAGMA_EXP_COV_FORK")
    if which == "b512":  # 256 < d <= 512, cov mode (run with MIDAGMA_EXP_BINV512=0 / 1: read once per process)
        for d in (300, 400, 500):
            print(f"MIDAGMA_EXP_BINV512={os.environ.get('MIDAGMA_EXP_BINV512', '0')}", end=" ")
            cov_case(d, 2 * d, 20, 3000)
    if which == "lacmp":  # look-ahead residual experiment (block g's launches prepare block g+1's R) on / off
        for d, K in ((1000, 2000), (700, 2000), (1150, 1000), (1400, 1000)):
            for f in ("1", "0"):
                os.environ["MIDAGMA_EXP_RESID_LA"] = f
                print(f"MIDAGMA_EXP_RESID_LA={f}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_RESID_LA")
    if which == "groupcmp":  # fast slots captured per graph (MIDAGMA_EXP_FAST_GROUP, default 4)
        for d, K in ((1000, 2000), (300, 4000), (2000, 300)):
            for g in ("4", "8", "16"):
                os.environ["MIDAGMA_EXP_FAST_GROUP"] = g
                print(f"MIDAGMA_EXP_FAST_GROUP={g}", end=" ")
                cov_case(d, 2 * d, 10, K)
        os.environ.pop("MIDAGMA_EXP_FAST_GROUP")
    if which == "b128":  # 64 < d <= 128 (run with MIDAGMA_EXP_BINV128=0 / 1: read once per process)
        for d in (65, 100, 128):
            print(f"MIDAGMA_EXP_BINV128={os.environ.get('MIDAGMA_EXP_BINV128', '1')}", end=" ")
            cov_case(d, 2000, 20, 5000)
    if which == "pad256":  # 128 < d <= 192 in cov mode: D = 256 (one-block fast path) or 192 (flat GJ)
        for d in (129, 150, 192):
            for f in ("1", "0"):
                os.environ["MIDAGMA_EXP_COV_PAD256"] = f
                print(f"MIDAGMA_EXP_COV_PAD256={f}", end=" ")
                cov_case(d, 2000, 20, 3000)
        os.environ.pop("MIDAGMA_EXP_COV_PAD256")
    if which == "d1000short":  # PMC passes: few dispatches
        cov_case(1000, 2000, 10, 40)
    if which == "fit":
        fit_case(1000, 10000)
    if which == "fit20":
        fit_case(20, 1000)
    if which == "d2000":
        cov_case(2000, 4000, 5, 100)
    if which in ("all", "d5000"):
        cov_case(5000, 6000, 2, 30)
    if which == "trek":
        for seq in ("exp", "inv", "log"):
            trek_case(1000, seq, 50)
    if which == "tcc":
        for d, K in ((8, 2000), (20, 2000), (32, 2000), (100, 500), (300, 200)):
            trek_case(d, "tcc", K)
    if which == "large3":  # the large-D cov slots (run once per knob setting: the knobs are read once)
        for d, K in ((2000, 300), (3000, 100), (5000, 40)):
            cov_case(d, d + 1000, 3, K)
    if which == "tcc20":  # one size, for a kernel trace
        trek_case(20, "tcc", 2000)
    if which == "tccd":  # the given sizes (default 100), for a kernel trace
        for d in [int(x) for x in sys.argv[2:]] or [100]:
            trek_case(d, "tcc", 300 if d <= 300 else 60)
    if which == "tccnb":  # the one-workgroup TCC at each block count it fits
        for d, nbs in ((8, ("8", "16", "32")), (16, ("8", "16", "32")), (20, ("16", "32")), (32, ("16", "32")),
                       (64, ("32",))):
            for nb in nbs:
                os.environ["MIDAGMA_EXP_TCC_NB"] = nb
                print(f"MIDAGMA_EXP_TCC_NB={nb}", end=" ")
                trek_case(d, "tcc", 2000)
        os.environ.pop("MIDAGMA_EXP_TCC_NB")
    if which == "shards":  # config 4's per-rank shard at N = 1, 2, 4, 8 GPUs, timed on one GPU
        for n, K in ((1_000_000, 10), (500_000, 20), (250_000, 40), (125_000, 80)):
            data_case(1000, n, 2, K)
    if which == "data125k":
        data_case(1000, 125000, 3, 60)
    if which == "data1m":
        data_case(1000, 1000000, 2, 20)
    if which in ("all", "data"):
        data_case(1000, 100000, 2, 10)
    if which == "data250":
        data_case(1000, 250000, 2, 20)
