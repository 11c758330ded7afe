"""ABI 11: data mode on several devices from ONE process (`HipGroup`, `DagmaLinear(devices=[...])`).

The reference's entry is a single-process `fit(X)` (src/dagma/linear.py:335-351) and its per-step
score gradient (244-246) is a sum over the rows of X.  A device group keeps one data-mode solver per
device with a row shard each and sums the shards' partials inside every slot.
The GPU box has one device, so:
  * an EMULATED group (every member on cuda:0, the sum a fixed-order device sum inside one captured
    graph over the members' streams) checks the sharded arithmetic at ndev 1..4 against the CPU
    oracle and against the plain one-device data-mode solver; the members'
    W bits and states must agree (the library checks and raises otherwise);
  * a one-member group through the REAL path (ncclCommInitAll, the library's per-device thread,
    the all-reduce captured in the slot graphs) must equal the plain solver bit for bit.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(d, n, seed, loss="l2"):
    from midagma_amd.simulate import make_dataset
    X, _, _ = make_dataset(d, n, seed=seed, sem_type="gauss" if loss == "l2" else "logistic")
    if loss == "l2":
        X = X - X.mean(axis=0, keepdims=True)
    return np.ascontiguousarray(X)


def _plain(X, loss, K, W0=None, checkpoint=100):
    from midagma_amd.solver import HipSolver
    d = X.shape[1]
    s = HipSolver(d, loss, "data", device=0)
    s.set_data(X, n_global=X.shape[0])
    s.set_cov(X.T @ X / float(X.shape[0]))
    W = np.zeros((d, d)) if W0 is None else W0.copy()
    r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=checkpoint, want_checkpoints=True)
    s.close()
    return W, r


def _group(X, loss, K, devices, W0=None, checkpoint=100, emulate=None):
    from midagma_amd.solver import HipGroup
    d = X.shape[1]
    g = HipGroup(d, loss, devices=devices, emulate=emulate)
    g.set_data(X)
    g.set_cov(X.T @ X / float(X.shape[0]))
    W = np.zeros((d, d)) if W0 is None else W0.copy()
    r = g.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=checkpoint, want_checkpoints=True)
    return g, W, r


@pytest.mark.parametrize("ndev", [1, 2, 3, 4])
def test_emulated_group_matches_oracle(ndev, parity):
    """l2, d=64, n=3001 (ragged shards): W after 300 steps vs the oracle's restatement of
    linear.py:165-333 within 1e-9, every checkpoint's objective within 1e-9 relative."""
    from oracle.dagma_oracle import LinearOracle
    X = _data(64, 3001, seed=11)
    g, W, r = _group(X, "l2", 300, [0] * ndev, emulate=True)
    assert g.emulated and g.size == ndev and r.iters == 300 and r.success
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 100)
    W_ref, tr = o.minimize(np.zeros((64, 64)), 1.0, 300, 1.0, 3e-4, tol=-1.0)
    dW = float(np.abs(W - W_ref).max())
    assert dW <= 1e-9, dW
    objs = [c.obj for c in r.checkpoints]
    ref = [c[1] for c in tr.checkpoints]
    assert len(objs) == len(ref) == 3
    assert np.allclose(objs, ref, rtol=1e-9, atol=0)
    # the summed partial: _score through the group equals the oracle's score at W
    loss, G = g.score(W)
    from oracle.dagma_oracle import score
    l_ref, G_ref = score("l2", W, o.cov)
    assert abs(loss - l_ref) <= 1e-10 * abs(l_ref) and np.abs(G - G_ref).max() <= 1e-10 * np.abs(G_ref).max()
    g.close()
    parity("config4", dW, 1e-9, f"max|dW| emulated {ndev}-member group, d=64 K=300")


def test_emulated_group_blocked_slots_match_plain_solver():
    """d=300, n=4003 over 3 members: small shards run the blocked fast inverse (hand-backs, pivoted
    checkpoint slots), whose fast graphs the group captures over all members' streams.  W after 250
    steps within 1e-9 of the plain one-device data-mode solver and of the oracle."""
    from oracle.dagma_oracle import LinearOracle
    X = _data(300, 4003, seed=12)
    W1, r1 = _plain(X, "l2", 250)
    g, W3, r3 = _group(X, "l2", 250, [0, 0, 0])
    assert r3.iters == r1.iters == 250
    assert np.abs(W3 - W1).max() <= 1e-9
    o = LinearOracle("l2")
    o.prepare(X.copy(), 0.03, 100)
    W_ref, _ = o.minimize(np.zeros((300, 300)), 1.0, 250, 1.0, 3e-4, tol=-1.0)
    assert np.abs(W3 - W_ref).max() <= 1e-9
    # a second call on the same group (the next stage's mu, from this W) re-captures its graphs
    from midagma_amd.solver import HipSolver
    W = W3.copy()
    r = g.minimize(W, 0.1, 60, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
    s = HipSolver(300, "l2", "data", device=0)
    s.set_data(X, n_global=X.shape[0])
    s.set_cov(X.T @ X / float(X.shape[0]))
    Wp = W3.copy()
    rp = s.minimize(Wp, 0.1, 60, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100)
    assert r.iters == rp.iters == 60 and np.abs(W - Wp).max() <= 1e-9
    s.close()
    g.close()


def test_emulated_group_logistic_matches_plain_solver():
    """logistic (binary X), d=48, n=2000 over 2 members, 200 steps: the loss tail rides in the
    summed buffer; W within the rank-split tolerance of tests/test_gpu_distributed.py (exactly
    zero gradient entries of a binary X take their L1 branch from rounding)."""
    X = _data(48, 2000, seed=13, loss="logistic")
    W1, r1 = _plain(X, "logistic", 200)
    g, W2, r2 = _group(X, "logistic", 200, [0, 0])
    assert r2.iters == r1.iters == 200
    dW = np.abs(W2 - W1)
    assert dW.max() <= 1e-3 and (dW > 1e-9).mean() <= 0.05
    l1, _ = g.score(W1)
    s = _plain_score(X, W1)
    assert abs(l1 - s) <= 1e-12 * abs(s)
    g.close()


def _plain_score(X, W):
    from midagma_amd.solver import HipSolver
    s = HipSolver(X.shape[1], "logistic", "data", device=0)
    s.set_data(X, n_global=X.shape[0])
    s.set_cov(X.T @ X / float(X.shape[0]))
    s.score_partial(W)
    out = s.score_finish()[0]
    s.close()
    return out


def test_fit_devices_emulated_matches_single_device_fit():
    """DagmaLinear('l2', devices=[0, 0]).fit(X): the reference's fit() (linear.py:335-462) over an
    emulated two-member group, with an exclusion mask, against the plain one-device data-mode fit:
    the same per-stage iteration counts, W within 1e-9, the same support."""
    from midagma_amd import DagmaLinear
    X = _data(40, 2500, seed=14)
    kw = dict(lambda1=0.03, T=2, warm_iter=700, max_iter=900, exclude_edges=((0, 1), (2, 3)))
    m0 = DagmaLinear("l2", score_mode="data", device=0)
    W0 = m0.fit(X.copy(), **kw)
    m2 = DagmaLinear("l2", devices=[0, 0])
    W2 = m2.fit(X.copy(), **kw)
    assert m2._solver.emulated and m2._solver.size == 2
    assert [e["iters"] for e in m2.minimize_log] == [e["iters"] for e in m0.minimize_log]
    assert np.abs(W2 - W0).max() <= 1e-9 and np.array_equal(W2 != 0, W0 != 0)
    assert W2[0, 1] == 0 and W2[2, 3] == 0
    assert abs(m2.h_final - m0.h_final) <= 1e-9 * max(1.0, abs(m0.h_final))
    assert abs(m2.score_final - m0.score_final) <= 1e-9 * abs(m0.score_final)
    # cov formed from the members' device Gram matrices (gram='device') agrees with the host product
    m3 = DagmaLinear("l2", devices=[0, 0, 0])
    Xc = X.copy()
    m3.fit(Xc, lambda1=0.03, T=1, max_iter=10, gram="device")
    assert np.abs(m3.cov - m0.cov).max() <= 1e-12 * np.abs(m0.cov).max()
    for m in (m0, m2, m3):
        m._solver.close()


def test_group_bad_devices_raise():
    from midagma_amd.solver import HipGroup
    import torch
    n = torch.cuda.device_count()
    with pytest.raises(ValueError):
        HipGroup(16, "l2", devices=[n])          # no such device
    with pytest.raises(ValueError):
        HipGroup(16, "l2", devices=[0, 0], emulate=False)   # one RCCL rank per device
    g = HipGroup(16, "l2", devices=[0, 0])
    with pytest.raises(ValueError):
        g.set_data(np.zeros((1, 16)))            # fewer rows than members
    g.close()


_RCCL_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch  # noqa: F401
from midagma_amd.solver import HipSolver, HipGroup
from midagma_amd.simulate import make_dataset
out = {}
for loss, d, n, K in (("l2", 64, 3000, 300), ("logistic", 64, 3000, 300), ("l2", 300, 4000, 200)):
    X, _, _ = make_dataset(d, n, seed=5, sem_type="gauss" if loss == "l2" else "logistic")
    if loss == "l2":
        X = X - X.mean(axis=0, keepdims=True)
    X = np.ascontiguousarray(X)
    cov = X.T @ X / float(n)
    s = HipSolver(d, loss, "data", device=0)
    s.set_data(X, n_global=n)
    s.set_cov(cov)
    W1 = np.zeros((d, d))
    r1 = s.minimize(W1, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100, want_checkpoints=True)
    s.score_partial(W1)
    sc1 = s.score_finish()[0]
    s.close()
    g = HipGroup(d, loss, devices=[0])
    assert not g.emulated and g.comm_ranks == 1
    g.set_data(X)
    g.set_cov(cov)
    W2 = np.zeros((d, d))
    r2 = g.minimize(W2, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=100, want_checkpoints=True)
    sc2 = g.score(W1)[0]
    g.close()
    out[f"{loss}_{d}"] = dict(W=bool(np.array_equal(W1, W2)), iters=[r1.iters, r2.iters],
                              ckpt=bool([c._replace(elapsed=0.0) for c in r1.checkpoints]
                                        == [c._replace(elapsed=0.0) for c in r2.checkpoints]),
                              score=[sc1, sc2])
# DagmaLinear(devices=[0]).fit: the reference's fit over a one-member RCCL group
from midagma_amd import DagmaLinear
X, _, _ = make_dataset(40, 2500, seed=6)
kw = dict(lambda1=0.03, T=2, warm_iter=600, max_iter=800)
m0 = DagmaLinear("l2", score_mode="data", device=0)
W0 = m0.fit(X.copy(), **kw)
m1 = DagmaLinear("l2", devices=[0])
W1 = m1.fit(X.copy(), **kw)
out["fit"] = dict(W=bool(np.array_equal(W0, W1)), it0=[e["iters"] for e in m0.minimize_log],
                  it1=[e["iters"] for e in m1.minimize_log], rccl=m1._solver.comm_ranks)
m0._solver.close()
m1._solver.close()
print(json.dumps(out), flush=True)
"""


def test_one_device_rccl_group_bit_identical_to_plain_solver():
    """The real group path at one device: ncclCommInitAll, the all-reduce in the captured slot
    graphs, the agreement poll, the library's member thread.  A one-rank sum is the identity, so
    W, iterations, checkpoint records and the score equal the plain solver's bit for bit (l2 and
    logistic at d=64; the blocked fast-inverse slots at d=300), and so does fit().  In a child
    process (its own HIP / RCCL state)."""
    env = dict(os.environ, NCCL_DEBUG="WARN")
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD, REPO], capture_output=True, text=True, timeout=300,
                       env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"child rc={r.returncode}: {r.stderr[-3000:]}"
    out = json.loads(lines[-1])
    for key in ("l2_64", "logistic_64", "l2_300"):
        o = out[key]
        assert o["W"] and o["ckpt"] and o["iters"][0] == o["iters"][1], (key, o)
        assert o["score"][0] == o["score"][1], (key, o)
    f = out["fit"]
    assert f["W"] and f["it0"] == f["it1"] and f["rccl"] == 1, f
