"""Noise envelope of the d=1000 default fit (tests/test_gpu_parity.py::test_full_fit_d1000_matches_reference_algorithm).

fit_d1000_ref.npz (make_fit_d1000.py) is the oracle's default DagmaLinear('l2').fit on BASELINE
config 2.  This script reruns that fit with 1e-16 relative noise injected into every inverse
(the reference's own sensitivity, the "perturbed-oracle envelope"), one process
per noise seed at one BLAS thread (~2 h each), and stores for each seed what the fixture holds:
per-stage iteration counts, h_final, score_final and the thresholded W as (row, col, value).

    python tests/golden/make_fit_d1000_envelope.py          # all seeds in parallel
    python tests/golden/make_fit_d1000_envelope.py --seed 7 --out /tmp/x.npz
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
SEEDS = (7, 11, 13)


def run(seed, out):
    from midagma_amd.simulate import make_dataset
    from oracle.dagma_oracle import LinearOracle
    X, _, _ = make_dataset(1000, 10000, seed=0)
    o = LinearOracle("l2")
    rng = np.random.default_rng(seed)
    o.inv_hook = lambda M: M * (1.0 + 1e-16 * rng.standard_normal(M.shape))
    t0 = time.time()
    W = o.fit(X.copy(), lambda1=0.03)
    rows, cols = np.nonzero(W)
    stages = np.array([[i, tr.iters, int(tr.success)] for (i, _mu, _s, _lr, tr) in o.stages], dtype=np.int64)
    np.savez_compressed(out, stages=stages, h_final=o.h_final, score_final=o.score_final,
                        rows=rows.astype(np.int32), cols=cols.astype(np.int32), vals=W[rows, cols])
    print(json.dumps({"seed": seed, "wall_s": time.time() - t0, "stages": stages.tolist()}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.seed is not None:
        run(a.seed, a.out)
        return
    tmp = "/tmp/fit_d1000_env"
    os.makedirs(tmp, exist_ok=True)
    procs = [subprocess.Popen([sys.executable, __file__, "--seed", str(s), "--out", f"{tmp}/s{s}.npz"])
             for s in SEEDS]
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("worker failed")
    out = {"seeds": np.array(SEEDS)}
    for s in SEEDS:
        z = np.load(f"{tmp}/s{s}.npz")
        for k in z.files:
            out[f"s{s}_{k}"] = z[k]
    np.savez_compressed(os.path.join(HERE, "fit_d1000_envelope.npz"), **out)


if __name__ == "__main__":
    main()
