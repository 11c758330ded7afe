"""Fixture for the d=1000 full-fit check (tests/test_gpu_parity.py::test_full_fit_d1000_matches_reference_algorithm).

The oracle (oracle/dagma_oracle.py, the numpy/scipy restatement of linear.py pinned bit-exact
to the reference's own outputs at d=20 and d=100) runs the default DagmaLinear('l2').fit on
BASELINE config 2 (d=1000, n=1e4, ER(s0=d) Gaussian SEM of midagma_amd.simulate.make_dataset,
seed 0, lambda1=0.03).  One run took 2.5 h on 6 BLAS threads of the build container, so the
fixture keeps only what the check needs: the per-stage iteration counts, h_final and
score_final, and the thresholded W as (row, col, value) triples.

    OMP_NUM_THREADS=6 OPENBLAS_NUM_THREADS=6 python tests/golden/make_fit_d1000.py
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle  # noqa: E402


def main(out=os.path.join(REPO, "tests", "golden", "fit_d1000_ref.npz")):
    X, _, _ = make_dataset(1000, 10000, seed=0)
    o = LinearOracle("l2")
    t0 = time.time()
    W = o.fit(X.copy(), lambda1=0.03)
    rows, cols = np.nonzero(W)
    stages = np.array([[i, tr.iters, int(tr.success)] for (i, _mu, _s, _lr, tr) in o.stages], dtype=np.int64)
    np.savez_compressed(out, stages=stages, h_final=o.h_final, score_final=o.score_final,
                        rows=rows.astype(np.int32), cols=cols.astype(np.int32), vals=W[rows, cols])
    print(json.dumps({"wall_s": time.time() - t0, "stages": stages.tolist()}))


if __name__ == "__main__":
    main()
