"""Multi-rank data mode through the real HIP path: two ranks share cuda:0 (the GPU box
has one device) and all-reduce the per-step score partial with gloo on the CUDA tensor
bound as the solver's zbuf -- the same code path RCCL takes on an 8-GPU node.  The
result must equal the single-process GPU data-mode fit and stay replicated."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, X, loss, K, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from midagma_amd import DagmaLinear
        m = DagmaLinear(loss, score_mode="data", device=0)
        m.X, m.lambda1, m.checkpoint = X.copy(), 0.03, 1000
        m.n, m.d = X.shape
        m.exc_r = m.exc_c = m.inc_r = m.inc_c = None
        if loss == "l2":
            m.X -= m.X.mean(axis=0, keepdims=True)
        m.cov = m.X.T @ m.X / float(m.n)
        m._setup_solver()
        W, ok = m.minimize(np.zeros((m.d, m.d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
        sc, _ = m._score(W)
        out_q.put((rank, W, ok, sc))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("loss", ["l2", "logistic"])
def test_two_ranks_match_single_process(loss):
    from midagma_amd.simulate import make_dataset
    from midagma_amd.solver import HipSolver
    X, _, _ = make_dataset(30, 1500, seed=4, sem_type="gauss" if loss == "l2" else "logistic")
    K, world = 120, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, X, loss, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(outs[0][1], outs[1][1]), "replicas diverged"
    assert outs[0][2] and outs[0][3] == outs[1][3]
    # single process, same data, data mode on the GPU
    Xs = X.copy()
    if loss == "l2":
        Xs -= Xs.mean(axis=0, keepdims=True)
    s = HipSolver(30, loss, "data", device=0)
    s.set_data(Xs, n_global=Xs.shape[0])
    s.set_cov(Xs.T @ Xs / float(Xs.shape[0]))
    W = np.zeros((30, 30))
    r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    assert r.iters == K
    dW = np.abs(outs[0][1] - W)
    if loss == "l2":
        assert dW.max() <= 1e-9
    else:
        # binary X: exactly-zero gradient entries take their L1 branch from rounding (see
        # test_gpu_parity.test_logistic_data_mode); the rank-split sum is another valid order
        assert dW.max() <= 1e-3 and (dW > 1e-9).mean() <= 0.05


_NCCL_CHILD = r"""
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from midagma_amd import DagmaLinear
from midagma_amd.simulate import make_dataset
X, _, _ = make_dataset(64, 3000, seed=5)
kw = dict(lambda1=0.03, T=2, warm_iter=600, max_iter=800)
m0 = DagmaLinear("l2", score_mode="data", device=0)
W0 = m0.fit(X.copy(), **kw)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
m1 = DagmaLinear("l2", score_mode="data", device=0, force_allreduce=True, comm="host")
W1 = m1.fit(X.copy(), **kw)
m2 = DagmaLinear("l2", score_mode="data", device=0, force_allreduce=True, comm="host")
W2 = m2.fit(X.copy(), n_global=X.shape[0], **kw)
# the in-library communicator (ABI 7): the all-reduce captured in the slot graphs, the loop on the device
m3 = DagmaLinear("l2", score_mode="data", device=0, force_allreduce=True)
W3 = m3.fit(X.copy(), **kw)
from midagma_amd.solver import HipSolver
Xc = X - X.mean(axis=0, keepdims=True)
res = {}
for lib_comm in (False, True):
    for loss in ("l2", "logistic"):
        Xl = Xc if loss == "l2" else (X > 0).astype(np.float64)
        s = HipSolver(64, loss, "data", device=0)
        s.set_data(Xl, n_global=Xl.shape[0])
        s.set_cov(Xl.T @ Xl / float(Xl.shape[0]))
        if lib_comm:
            s.attach_comm(None)
            assert s.comm_ranks == 1
        Wk = np.zeros((64, 64))
        r = s.minimize(Wk, 1.0, 300, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
        s.score_partial(Wk)
        if lib_comm:
            s.comm_allreduce_zbuf()
        res[(lib_comm, loss)] = (Wk, r.iters, s.score_finish()[0])
        s.close()
out = dict(it0=[e["iters"] for e in m0.minimize_log], it1=[e["iters"] for e in m1.minimize_log],
           bit_identical=bool(np.array_equal(W1, W0)), h=[m0.h_final, m1.h_final], sc=[m0.score_final, m1.score_final],
           allreduce_path=m1._allreduce is not None and m2._allreduce is not None,
           cov_rel=float(np.abs(m2.cov - m0.cov).max() / np.abs(m0.cov).max()),
           dW2=float(np.abs(W2 - W0).max()), support2=bool(np.array_equal(W2 != 0, W0 != 0)),
           inlib=bool(m3._inlib and m3._allreduce is None and m3._solver.comm_ranks == 1),
           it3=[e["iters"] for e in m3.minimize_log], lib_fit_identical=bool(np.array_equal(W3, W0)),
           sc3=m3.score_final,
           lib_solver_identical={loss: bool(np.array_equal(res[(True, loss)][0], res[(False, loss)][0])
                                            and res[(True, loss)][1:] == res[(False, loss)][1:])
                                 for loss in ("l2", "logistic")})
print(json.dumps(out), flush=True)
for m in (m0, m1, m2, m3):
    m._solver.close()
torch.cuda.synchronize()
dist.destroy_process_group()
print("DESTROYED", flush=True)
"""


def test_nccl_one_rank_allreduce_path_bit_identical():
    """The RCCL code paths at world size 1.  Host-driven (comm='host'): DagmaLinear(score_mode='data', force_allreduce=True)
    under a one-rank 'nccl' process group runs every step as step_partial -> dist.all_reduce of
    the torch-owned score buffer on the solver's stream (ExternalStream) -> step_finish.  A
    one-rank sum is the identity, so W must equal the single-process run bit for bit.  The
    sharded form fit(X, n_global=n) (device Gram + all-reduce for cov) must agree to 1e-9.
    In-library (the default under 'nccl', ABI 7): the solver's own communicator, the all-reduce
    captured in the replayed slot graphs and the loop driven from the device: fit() and a
    HipSolver.minimize (l2 and logistic, 300 steps) equal the single-process runs bit for bit.
    Runs in a child process (its own HIP/RCCL state), which also destroys the process group."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NCCL_DEBUG="WARN")
    r = subprocess.run([sys.executable, "-c", _NCCL_CHILD, repo, str(_free_port())], capture_output=True,
                       text=True, timeout=240, env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"child rc={r.returncode}: {r.stderr[-3000:]}"
    out = json.loads(lines[-1])
    assert out["allreduce_path"]
    assert out["it1"] == out["it0"]
    assert out["bit_identical"]
    assert out["h"][0] == out["h"][1] and out["sc"][0] == out["sc"][1]
    assert out["cov_rel"] <= 1e-12
    assert out["dW2"] <= 1e-9 and out["support2"]
    # the in-library RCCL path (the default under 'nccl'): bit-identical to the single-process run
    assert out["inlib"] and out["it3"] == out["it0"] and out["lib_fit_identical"]
    assert out["sc3"] == out["sc"][0]
    assert out["lib_solver_identical"] == {"l2": True, "logistic": True}, out["lib_solver_identical"]
    assert "DESTROYED" in r.stdout and r.returncode == 0, f"destroy_process_group: rc={r.returncode} {r.stderr[-3000:]}"
