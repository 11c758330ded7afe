"""The CPU oracle (oracle/dagma_oracle.py) reproduces the reference's own outputs.

Fixtures were produced by tests/golden/make_golden.py, which imports the
reference (fbleile/midagma) in the build container at one BLAS thread.  The
oracle must match them BIT-FOR-BIT at one BLAS thread; this pins the oracle
that every GPU parity test then uses as its checker.
"""
import numpy as np
import pytest

from oracle.dagma_oracle import LinearOracle, adam_step, AdamState, h_logdet, score, mlp_h_value

pytestmark = pytest.mark.usefixtures("one_blas_thread")


def _x20(golden):
    return golden("data_d20_n1000_seed0.npz")["X"].copy()


def _oracle(X, loss="l2", lambda1=0.03, exc=None, inc=None):
    o = LinearOracle(loss)
    o.prepare(X.copy(), lambda1, 1000, exc, inc)
    return o


def test_generator_is_stable(golden):
    from midagma_amd.simulate import make_dataset
    X, W, B = make_dataset(20, 1000, seed=0)
    g = golden("data_d20_n1000_seed0.npz")
    assert np.array_equal(X, g["X"]) and np.array_equal(W, g["W_true"])
    m = golden("data_meta.npz")
    X1, W1, _ = make_dataset(100, 2000, seed=1)
    assert X1.sum() == m["d100_sum"] and np.array_equal(X1[0], m["d100_row0"])


@pytest.mark.parametrize("d", [5, 20, 100])
@pytest.mark.parametrize("s", [1.0, 0.9, 0.6])
def test_h_matches_reference(golden, d, s):
    b = golden("blocks.npz")
    h, G = h_logdet(b[f"h_W_d{d}"], s)
    assert h == b[f"h_val_d{d}_s{s}"]
    assert np.array_equal(G, b[f"h_grad_d{d}_s{s}"])


def test_score_matches_reference(golden):
    b = golden("blocks.npz")
    W = b["score_W"]
    o = _oracle(_x20(golden))
    l, G = score("l2", W, o.cov)
    assert l == b["score_l2_loss"] and np.array_equal(G, b["score_l2_grad"])
    ol = _oracle(golden("data_meta.npz")["logit_X"], "logistic")
    l, G = score("logistic", W, ol.cov, ol.X)
    assert l == b["score_logistic_loss"] and np.array_equal(G, b["score_logistic_grad"])


def test_adam_matches_reference(golden):
    b = golden("blocks.npz")
    st = AdamState()
    for k in range(5):
        assert np.array_equal(adam_step(st, b["adam_g"][k], k + 1, 0.99, 0.999), b["adam_out"][k])


@pytest.mark.parametrize("tag,K", [("d20", 1), ("d20", 10), ("d20", 100), ("d20", 1000),
                                   ("d20", 10000), ("d100", 1), ("d100", 10), ("d100", 100),
                                   ("d100", 1000), ("logistic_d20", 100), ("logistic_d20", 1000),
                                   ("logistic_d100", 10), ("logistic_d100", 500)])
def test_minimize_trajectory_bit_exact(golden, tag, K):
    t = golden(f"traj_{tag}.npz")
    if tag == "d20":
        X, loss, l1 = _x20(golden), "l2", 0.03
    elif tag == "d100":
        from midagma_amd.simulate import make_dataset
        X, loss, l1 = make_dataset(100, 2000, seed=1)[0], "l2", 0.03
    elif tag == "logistic_d100":
        X, loss, l1 = golden("data_logistic_d100.npz")["X"].copy(), "logistic", 0.05
    else:
        X, loss, l1 = golden("data_meta.npz")["logit_X"].copy(), "logistic", 0.05
    o = _oracle(X, loss, l1)
    d = X.shape[1]
    W, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert tr.success == bool(t[f"ok_K{K}"]) and tr.iters == int(t[f"it_K{K}"])
    assert np.array_equal(W, t[f"W_K{K}"])


def test_branches_bit_exact(golden):
    b = golden("branches.npz")
    X = _x20(golden)
    o = _oracle(X)
    W, tr = o.minimize(np.zeros((20, 20)), 1.0, 60, 1.0, 0.3, tol=-1.0)
    assert tr.success and tr.iters == int(b["halve_it"]) and tr.halvings == int(b["halve_nhalvings"])
    assert np.array_equal(W, b["halve_W"])
    o = _oracle(X)
    W, tr = o.minimize(np.zeros((20, 20)), 1.0, 60, 0.9, 0.3, tol=-1.0)
    assert tr.success is False and tr.iters == int(b["ood_it"])
    assert np.array_equal(W, b["ood_W"])
    exc = tuple(map(tuple, b["mask_exc"]))
    inc = tuple(map(tuple, b["mask_inc"]))
    o = _oracle(X, exc=exc, inc=inc)
    W, tr = o.minimize(np.zeros((20, 20)), 1.0, 500, 1.0, 3e-4, tol=-1.0)
    assert np.array_equal(W, b["mask_W"])
    for r, c in exc:
        assert W[r, c] == 0.0


def test_full_fit_bit_exact(golden):
    f = golden("fit_d20.npz")
    o = LinearOracle("l2")
    W = o.fit(_x20(golden), lambda1=0.03)
    stages = np.array([(mu, s, lr, 0, tr.success, tr.iters) for (_, mu, s, lr, tr) in o.stages])
    assert np.array_equal(stages[:, [0, 2, 4, 5]], f["calls"][:, [0, 2, 4, 5]])
    assert np.array_equal(o.W_unthresholded, f["W_unthresholded"])
    assert np.array_equal(W, f["W"])
    assert o.h_final == f["h_final"] and o.score_final == f["score_final"]


@pytest.mark.parametrize("d", [20, 200])
@pytest.mark.parametrize("s", [1.0, 0.8])
def test_mlp_h_func(golden, d, s):
    """h_func value and gradient (autograd in the reference) vs the closed form."""
    from tests.golden.inputs import mlp_fc1
    g = golden("mlp_h.npz")
    w = mlp_fc1(d, 10)
    h, dA = mlp_h_value(w, d, s)
    assert abs(h - g[f"h_d{d}_s{s}"]) <= 1e-12 * max(1.0, abs(h))
    # dh/dW1[j*m+k, i] = 2 * W1[j*m+k, i] * dh/dA[i, j]
    grad = (2 * w.reshape(d, 10, d) * dA.T[:, None, :]).reshape(d * 10, d)
    np.testing.assert_allclose(grad.reshape(-1)[g[f"pick_d{d}"]], g[f"gradpick_d{d}_s{s}"],
                               rtol=1e-10, atol=1e-14)


def test_fit_d1000_envelope_fixture():
    """fit_d1000_envelope.npz (tests/golden/make_fit_d1000_envelope.py): the oracle's default
    d=1000 fit refitted with 1e-16 relative noise in every inverse, 3 seeds.  Each refit keeps the
    unperturbed fit's thresholded support; its W, h_final and score_final deviate by amounts
    that set the GPU full-fit test's tolerances (tests/test_gpu_parity.py)."""
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    f = np.load(os.path.join(here, "fit_d1000_ref.npz"))
    e = np.load(os.path.join(here, "fit_d1000_envelope.npz"))
    ref = set(zip(f["rows"].tolist(), f["cols"].tolist()))
    assert len(e["seeds"]) == 3
    for s in e["seeds"]:
        assert set(zip(e[f"s{s}_rows"].tolist(), e[f"s{s}_cols"].tolist())) == ref
        assert e[f"s{s}_stages"].shape == f["stages"].shape
        assert np.all(e[f"s{s}_stages"][:, 2] == 1)  # every stage succeeded
        assert abs(float(e[f"s{s}_h_final"]) - float(f["h_final"])) < 1e-8
        assert abs(float(e[f"s{s}_score_final"]) / float(f["score_final"]) - 1) < 1e-5


def test_float32_fit_bit_exact(golden):
    """dtype=np.float32 (linear.py:29, 408, 429): the oracle's float32 fit (Id, W and mask_exc in
    float32, so numpy rounds s*Id - W*W, the float32 inverse, M + 1e-16, 2 W o M^T and every
    in-place update of W to float32) reproduces the reference's own float32 fit bit for bit
    (fit_f32_d20.npz), and its float32 perturbation envelope (fit_f32_d20_envelope.npz: 1-ulp
    noise in every float32 inverse) keeps that fit's support."""
    f = golden("fit_f32_d20.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = LinearOracle("l2", dtype=np.float32)
    W = o.fit(X, lambda1=0.03, T=3, s=[1.0, .9, .8], warm_iter=4000, max_iter=5000)
    assert W.dtype == np.float32
    assert np.array_equal(W, f["W_f32"])
    assert float(o.h_final) == float(f["h_final_f32"]) and float(o.score_final) == float(f["score_final_f32"])
    env = golden("fit_f32_d20_envelope.npz")
    for Wn in env["W"]:
        assert np.array_equal(Wn != 0, f["W_f32"] != 0)


def test_float32_default_fit_bit_exact(golden):
    """The DEFAULT fit with dtype=np.float32 (fit_f32_d20_default.npz): its stages stop early on the
    float32 checkpoint objective -- numpy's float32 np.abs(W).sum(), lambda1 times it in float32 and
    slogdet's float32 log|det| (linear.py:113-114, 127, 328-331) -- and go out of domain and retry
    at s = 0.7 and 0.6.  The oracle reproduces every call (mu, lr, success, iterations) and W."""
    f = golden("fit_f32_d20_default.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = LinearOracle("l2", dtype=np.float32)
    W = o.fit(X, lambda1=0.03)
    calls = np.array([(mu, s, lr, 0, tr.success, tr.iters) for (_, mu, s, lr, tr) in o.stages])
    assert np.array_equal(calls[:, [0, 2, 4, 5]], f["calls"][:, [0, 2, 4, 5]])
    assert np.array_equal(W, f["W"])
    assert float(o.h_final) == float(f["h_final"]) and float(o.score_final) == float(f["score_final"])
