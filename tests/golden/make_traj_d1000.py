"""Fixture for the d=1000 long-horizon trajectory check (tests/test_gpu_parity.py::test_trajectory_d1000).

BASELINE config 2 data (d=1000, n=1e4, ER(s0=d) Gaussian SEM of midagma_amd.simulate.make_dataset,
seed 0, lambda1=0.03, cov precomputed as in linear.py:428).  The oracle (oracle/dagma_oracle.py,
the numpy/scipy restatement of linear.py:165-333, bit-exact to the reference's own outputs at
d=20 and d=100) runs minimize(W=0, mu=1, s=1, lr=3e-4, tol=-1) at ONE BLAS thread and keeps W
after K = 1000 and 2000 steps.  The envelope is SURVEY.md 8(c)'s: the same run with 1e-16
relative noise injected into every inverse (`inv_hook`), under several noise seeds; env_K is the
largest max|W_noisy - W| over those seeds.

    python tests/golden/make_traj_d1000.py            # clean run + 3 noisy seeds, in parallel
    python tests/golden/make_traj_d1000.py --seed 5   # one worker (used by the above)
"""
import argparse
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
HERE = os.path.join(REPO, "tests", "golden")
KS = (1000, 2000)
NOISE_SEEDS = (101, 202, 303)


def run(seed):
    from midagma_amd.simulate import make_dataset
    from oracle.dagma_oracle import LinearOracle
    X, _, _ = make_dataset(1000, 10000, seed=0)
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 1000)
    if seed >= 0:
        rng = np.random.default_rng(seed)
        o.inv_hook = lambda M: M * (1.0 + 1e-16 * rng.standard_normal(M.shape))
    t0 = time.time()
    _, tr = o.minimize(np.zeros((1000, 1000)), 1.0, max(KS), 1.0, 3e-4, tol=-1.0, snap_at=KS)
    return {K: tr.snaps[K] for K in KS}, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=None, help="-1: clean run; >= 0: noisy seed")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.seed is not None:
        snaps, wall = run(a.seed)
        np.savez(a.out, **{f"W_K{K}": snaps[K] for K in KS})
        print(json.dumps({"seed": a.seed, "wall_s": wall}), flush=True)
        return
    tmp = "/tmp/traj_d1000"
    os.makedirs(tmp, exist_ok=True)
    seeds = (-1,) + NOISE_SEEDS
    procs = [subprocess.Popen([sys.executable, __file__, "--seed", str(s), "--out", f"{tmp}/s{s}.npz"])
             for s in seeds]
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("worker failed")
    ref = np.load(f"{tmp}/s-1.npz")
    out = {"Ks": np.array(KS), "noise_seeds": np.array(NOISE_SEEDS)}
    for K in KS:
        out[f"W_K{K}"] = ref[f"W_K{K}"]
        env = max(float(np.abs(np.load(f"{tmp}/s{s}.npz")[f"W_K{K}"] - ref[f"W_K{K}"]).max())
                  for s in NOISE_SEEDS)
        out[f"env_K{K}"] = np.array(env)
        print(f"K={K}: envelope {env:.3e}", flush=True)
    np.savez_compressed(os.path.join(HERE, "traj_d1000.npz"), **out)


if __name__ == "__main__":
    main()
