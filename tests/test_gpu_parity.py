"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference-generated golden fixtures.  Run on an MI355X: pytest -m gpu.

Tolerances (BASELINE.json north star: W within 1e-5 after the same iteration
count): kernels h/score rel 1e-12; trajectories W within 1e-5 at
every K where the reference's own 1e-16-perturbation envelope is < 1e-6;
full fit: same per-stage iteration counts, same support, max|dW| <= 2x the
reference's envelope, h_final/score_final within 1e-6 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from midagma_amd.simulate import make_dataset  # noqa: E402
from oracle.dagma_oracle import LinearOracle, h_logdet, score  # noqa: E402


@pytest.fixture(scope="module")
def hip():
    from midagma_amd import _lib
    from midagma_amd.solver import device_count
    _lib.load()
    assert device_count() >= 1, "no ROCm device visible"
    return _lib


def _solver(d, cov=None, loss="l2", mode="cov"):
    from midagma_amd.solver import HipSolver
    s = HipSolver(d, loss, mode, device=0)
    if cov is not None:
        s.set_cov(cov)
    return s


def _oracle(X, loss="l2", l1=0.03, exc=None, inc=None):
    o = LinearOracle(loss)
    o.prepare(X.copy(), l1, 1000, exc, inc)
    return o


def _rel(a, b):
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max()))


# --------------------------------------------------------------------------- kernels
@pytest.mark.parametrize("d", [5, 20, 64, 100, 200, 513])
@pytest.mark.parametrize("s", [1.0, 0.9, 0.6])
def test_h_matches_oracle(hip, d, s):
    rng = np.random.default_rng(d)
    W = rng.uniform(-1, 1, (d, d)) * (0.5 / np.sqrt(d))
    np.fill_diagonal(W, 0)
    sol = _solver(d)
    h, G = sol.h_value(W, s)
    h_ref, G_ref = h_logdet(W, s)
    assert abs(h - h_ref) <= 1e-12 * max(1.0, abs(h_ref)) + 1e-13
    assert _rel(G, G_ref) <= 1e-12


@pytest.mark.parametrize("d", [20, 100, 257])
def test_score_matches_oracle(hip, d):
    X, _, _ = make_dataset(d, 3 * d, seed=d)
    X = X - X.mean(0)
    cov = X.T @ X / X.shape[0]
    rng = np.random.default_rng(1)
    W = rng.normal(size=(d, d)) * 0.1
    sol = _solver(d, cov)
    l, G = sol.score_value(W)
    l_ref, G_ref = score("l2", W, cov)
    assert abs(l - l_ref) <= 1e-12 * abs(l_ref)
    assert _rel(G, G_ref) <= 1e-12


def test_golden_h_and_score(hip, golden):
    b = golden("blocks.npz")
    for d in (5, 20, 100):
        sol = _solver(d)
        for s in (1.0, 0.9, 0.6):
            h, G = sol.h_value(b[f"h_W_d{d}"], s)
            assert abs(h - b[f"h_val_d{d}_s{s}"]) <= 1e-12 * max(1, abs(float(b[f"h_val_d{d}_s{s}"])))
            assert _rel(G, b[f"h_grad_d{d}_s{s}"]) <= 1e-12
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = _oracle(X)
    sol = _solver(20, o.cov)
    l, G = sol.score_value(b["score_W"])
    assert abs(l - b["score_l2_loss"]) <= 1e-12 * abs(float(b["score_l2_loss"]))
    assert _rel(G, b["score_l2_grad"]) <= 1e-12


# --------------------------------------------------------------------------- trajectories
@pytest.mark.parametrize("K", [1, 10, 100, 1000, 10000])
def test_trajectory_d20(hip, golden, parity, K):
    """BASELINE config 1 (d=20, n=1000; the small.hip persistent workgroup): W after K steps
    against the reference's own minimize (traj_d20.npz)."""
    t = golden("traj_d20.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = _oracle(X)
    sol = _solver(20, o.cov)
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    dW = float(np.abs(W - t[f"W_K{K}"]).max())
    parity("config1", dW, 1e-9, f"max|dW| K={K}")
    assert res.success and res.iters == int(t[f"it_K{K}"])
    assert float(t[f"env_K{K}"]) < 1e-6
    assert dW <= 1e-5
    # tighter: the GPU trajectory sits at rounding distance from the reference here
    assert dW <= 1e-9


@pytest.mark.parametrize("K", [1, 10, 100, 1000])
def test_trajectory_d100(hip, golden, K):
    t = golden("traj_d100.npz")
    X = make_dataset(100, 2000, seed=1)[0]
    o = _oracle(X)
    sol = _solver(100, o.cov)
    W = np.zeros((100, 100))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    assert res.success and res.iters == K
    # the reference's own 1e-16-perturbation envelope is <= 1.5e-16 at K <= 1000
    assert float(t[f"env_K{K}"]) < 1e-12
    assert np.abs(W - t[f"W_K{K}"]).max() <= 1e-9


def test_branches(hip, golden):
    b = golden("branches.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = _oracle(X)
    sol = _solver(20, o.cov)
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, 60, 1.0, 0.3, tol=-1.0, lambda1=0.03)
    assert res.success and res.iters == int(b["halve_it"]) and res.halvings == int(b["halve_nhalvings"])
    assert np.abs(W - b["halve_W"]).max() <= 1e-5
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, 60, 0.9, 0.3, tol=-1.0, lambda1=0.03)
    assert (not res.success) and res.iters == int(b["ood_it"])
    assert np.abs(W - b["ood_W"]).max() <= 1e-5
    exc = tuple(map(tuple, b["mask_exc"]))
    inc = tuple(map(tuple, b["mask_inc"]))
    o2 = _oracle(X, exc=exc, inc=inc)
    mi, me = o2.masks(1.0)
    sol.set_masks(mi, me)
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, 500, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    assert np.abs(W - b["mask_W"]).max() <= 1e-5
    for r, c in exc:
        assert W[r, c] == 0.0


def test_full_fit_d20(hip, golden, parity):
    """Default fit (T=5, s=[1,.9,.8,.7,.6]).  Stages 1-4 must take the reference's
    iteration counts.  The last stage (mu=1e-4, s=0.6) is chaotic: from identical
    starting W, GPU and reference separate by O(lr) within 2000 steps, and whether the
    relative objective change at a checkpoint is below tol=1e-6 varies (the reference
    itself shows 2.8e-7 at its stopping checkpoint) -- so only a one-checkpoint slack
    is allowed there ('or documented when an early-stop lands differently')."""
    from midagma_amd import DagmaLinear
    f = golden("fit_d20.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2")
    W = m.fit(X, lambda1=0.03, s=[1.0, .9, .8, .7, .6])
    iters = [e["iters"] for e in m.minimize_log]
    ref_iters = [int(c[5]) for c in f["calls"]]
    assert iters[:4] == ref_iters[:4]
    assert abs(iters[4] - ref_iters[4]) <= 1000
    # noise envelopes: the reference itself, refit with 1e-16 relative noise in every inverse
    # under 9 seeds (fit_d20.npz + fit_d20_envelope.npz); tolerance = 2x the widest spread
    e = golden("fit_d20_envelope.npz")
    Wn = np.concatenate([f["W_unthresholded_noisy"][None], e["W_unthresholded"]])
    hn = np.append(e["h_final"], float(f["h_final_noisy"]))
    sn = np.append(e["score_final"], float(f["score_final_noisy"]))
    env = float(np.abs(Wn - f["W_unthresholded"][None]).max())
    env_h = float(np.abs(hn - float(f["h_final"])).max())
    env_s = float(np.abs(sn - float(f["score_final"])).max())
    parity("config1", float(np.abs(W - f["W"]).max()), max(2 * env, 1e-5), "full fit max|dW|")
    assert np.array_equal(W != 0, f["W"] != 0)
    assert np.abs(W - f["W"]).max() <= max(2 * env, 1e-5)
    assert abs(m.h_final - f["h_final"]) <= max(2 * env_h, 1e-12)
    assert abs(m.score_final - f["score_final"]) <= max(2 * env_s, 1e-9 * abs(float(f["score_final"])))


def test_full_fit_float32_dtype(hip, golden):
    """dtype=np.float32 (linear.py:29): the reference keeps W (and Id) in float32, so numpy rounds
    every operation on them to float32 (fit_f32_d20.npz: T = 3, max |dW| 1.6e-4 from its float64
    fit, identical support).  The GPU loop emulates those float32 operations around a float64
    inverse rounded to float32 (csrc/common.h).  Bar: the reference's own float32 perturbation
    envelope -- the largest deviation of its float32 fit under 1-ulp noise in every float32
    inverse over 8 seeds (fit_f32_d20_envelope.npz, 1.9e-4) -- and the identical support."""
    from midagma_amd import DagmaLinear
    f = golden("fit_f32_d20.npz")
    env = golden("fit_f32_d20_envelope.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2", dtype=np.float32)
    W = m.fit(X, lambda1=0.03, T=3, s=[1.0, .9, .8], warm_iter=4000, max_iter=5000)
    assert W.dtype == np.float32
    env_w = float(np.abs(env["W"] - f["W_f32"]).max())
    assert np.array_equal(W != 0, f["W_f32"] != 0)
    assert np.abs(W - f["W_f32"]).max() <= env_w
    # every call's iteration count (here the stages run to max_iter: no early stop at this length)
    assert [e["iters"] for e in m.minimize_log] == [int(c[5]) for c in f["calls_f32"]]


def test_float32_default_fit_stage_counts_in_envelope(hip, golden):
    """The default fit with dtype=np.float32 stops its stages early on the float32 checkpoint
    objective (linear.py:113-114, 127, 328-331): numpy's float32 L1 sum (csrc/np_sum.h, bit for bit),
    lambda1 times it in float32, log|det| rounded to float32.  Each stage's successful call must take
    a number of iterations inside the range the reference's own float32 fit and its float32-noise
    replicas span (fit_f32_d20_default.npz: stage 1 12k-16k, stage 2 7k-8k, stage 3 8k-18k)."""
    from midagma_amd import DagmaLinear
    f = golden("fit_f32_d20_default.npz")
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2", dtype=np.float32)
    W = m.fit(X, lambda1=0.03)
    assert W.dtype == np.float32
    ok = [e["iters"] for e in m.minimize_log if e["success"]]
    ref = [int(c[5]) for c in f["calls"] if c[4] == 1]
    env = f["env_stage_iters"]
    assert len(ok) == len(ref) == env.shape[1] == 5
    # stages 1-3; at mu = 1e-3 the reference's unperturbed float32 fit leaves the domain through
    # negative entries of its float32 getri inverse and retries up to s = 1, which none of its
    # float32-noise replicas does (tests/test_dtype_cpu.py)
    for i, it in enumerate(ok[:3]):
        lo, hi = min(ref[i], env[:, i].min()), max(ref[i], env[:, i].max())
        assert lo <= it <= hi, (i, it, lo, hi, ok)


@pytest.mark.parametrize("d,mode", [(20, "cov"), (48, "cov"), (100, "cov"), (300, "cov"), (64, "data")])
def test_float32_checkpoint_objective(hip, d, mode):
    """The checkpoint record of a float32 fit holds the reference's float32 objective terms: l1 is
    numpy's float32 np.abs(W).sum() of that checkpoint's W bit for bit (the small loop's thread-0
    sum at d <= 32, np_l1_kernel on the graph path), obj = mu (score + f32(f32(lambda1) l1)) + h,
    and h = -f32(log|det|) + d log s within float32 rounding of the oracle's float32 slogdet."""
    from midagma_amd.solver import HipSolver
    n = 1000
    X, _, _ = make_dataset(d, n, seed=d + 1)
    Xc = X - X.mean(axis=0, keepdims=True)
    if mode == "cov":
        sol = _solver(d, Xc.T @ Xc / n)
    else:
        sol = HipSolver(d, "l2", "data", device=0)
        sol.set_data(Xc, n_global=n)
        sol.set_cov(Xc.T @ Xc / n)
    sol.set_w_float32(True)
    W = np.zeros((d, d))
    mu, lam = 1.0, 0.03
    res = sol.minimize(W, mu, 200, 1.0, 3e-4, tol=-1.0, lambda1=lam, checkpoint=100, want_checkpoints=True)
    sol.close()
    assert res.iters == 200
    rec = res.checkpoints[-1]
    assert rec.iter == 200
    W32 = W.astype(np.float32)
    assert rec.l1 == float(np.abs(W32).sum())
    l1term = float(np.float32(lam) * np.float32(rec.l1))
    assert rec.obj == mu * (rec.score + l1term) + rec.h
    h_ref, _ = h_logdet(W32, 1.0)
    assert abs(rec.h - float(h_ref)) <= 1e-6 * max(1.0, abs(float(h_ref))) + 1e-7


@pytest.mark.parametrize("d,K,n", [(20, 1000, 1000), (100, 300, 2000), (300, 100, 1000), (1000, 40, 2000)])
def test_float32_trajectory_matches_reference_float32(hip, d, K, n):
    """dtype=np.float32 per step: K Adam steps of stage 1 from a float32 W = 0 against the
    reference's float32 arithmetic (the oracle with dtype=float32, bit-exact to the reference's
    float32 fit: test_oracle_golden.py::test_float32_fit_bit_exact).  On the CPU the float64
    inverse rounded to float32 (the GPU's model) stays within 1e-8 of the reference's float32
    getri over these horizons, while float64 W moves 3e-5 to 1.9e-4 away; bound 1e-7, and at most
    a tenth of that float32 / float64 spread.  d = 20: the persistent workgroup; 100: one 128
    outer block; 300, 1000: the blocked two-level inverse (fast and pivoted slots)."""
    X, _, _ = make_dataset(d, n, seed=d)
    ref = {}
    for dt in (np.float32, np.float64):
        o = LinearOracle("l2", dtype=dt)
        o.prepare(X.copy(), 0.03, 1000)
        Wr, tr = o.minimize(np.zeros((d, d), dtype=dt), 1.0, K, 1.0, 3e-4, tol=-1.0)
        assert tr.iters == K
        ref[dt] = Wr.astype(np.float64)
    Xc = X - X.mean(axis=0, keepdims=True)
    sol = _solver(d, Xc.T @ Xc / n)
    sol.set_w_float32(True)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03)
    sol.close()
    assert res.iters == K
    assert np.array_equal(W, W.astype(np.float32).astype(np.float64))  # float32 values throughout
    dev = float(np.abs(W - ref[np.float32]).max())
    spread = float(np.abs(ref[np.float64] - ref[np.float32]).max())
    assert dev <= min(1e-7, 0.1 * spread), (dev, spread)


def test_full_fit_d1000_matches_reference_algorithm(hip, golden, parity):
    """BASELINE config 2 end to end: the default fit at d=1000, n=1e4 (ER(s0=d) Gaussian SEM,
    seed 0) against the oracle's run of the reference algorithm (fit_d1000_ref.npz, 2.5 h of
    CPU; tests/golden/make_fit_d1000.py), with tolerances from the reference's own noise
    envelope (fit_d1000_envelope.npz, tests/golden/make_fit_d1000_envelope.py: the same fit
    with 1e-16 relative noise in every inverse, 3 seeds, ~3 h each at one BLAS thread).  The
    perturbed refits keep the identical 1007-edge support but move W on it by up to 1.9e-2,
    h_final by 1.7e-9, score_final by 3.7e-6 relative and the early-stop checkpoints of the
    stages by up to 3000 iterations (the literal 1e-5 after a full fit is below
    the reference's own reproducibility).  Bar: the identical thresholded support, W on it,
    h_final and score_final within 2x the envelope's widest deviation from the unperturbed run,
    and every stage's iteration count inside the envelope's range widened by one checkpoint."""
    from midagma_amd import DagmaLinear
    f = golden("fit_d1000_ref.npz")
    e = golden("fit_d1000_envelope.npz")
    X, _, _ = make_dataset(1000, 10000, seed=0)
    m = DagmaLinear("l2")
    W = m.fit(X, lambda1=0.03)
    iters = [e_["iters"] for e_ in m.minimize_log]
    rows, cols = np.nonzero(W)
    gr, gc, gv = f["rows"], f["cols"], f["vals"]
    ref = np.zeros((1000, 1000))
    ref[gr, gc] = gv
    env_w = env_h = env_s = 0.0
    lo = f["stages"][:, 1].astype(np.int64).copy()
    hi = lo.copy()
    for sd in e["seeds"]:
        Wp = np.zeros((1000, 1000))
        Wp[e[f"s{sd}_rows"], e[f"s{sd}_cols"]] = e[f"s{sd}_vals"]
        env_w = max(env_w, float(np.abs(Wp - ref).max()))
        env_h = max(env_h, abs(float(e[f"s{sd}_h_final"]) - float(f["h_final"])))
        env_s = max(env_s, abs(float(e[f"s{sd}_score_final"]) - float(f["score_final"])) / float(f["score_final"]))
        st = e[f"s{sd}_stages"][:, 1]
        lo, hi = np.minimum(lo, st), np.maximum(hi, st)
    dw = float(np.abs(W - ref).max())
    ds = abs(m.score_final - float(f["score_final"])) / abs(float(f["score_final"]))
    dh = abs(m.h_final - float(f["h_final"]))
    print(f"stages gpu {iters} envelope {lo.tolist()}..{hi.tolist()}; nnz {len(rows)} vs {len(gr)}; "
          f"max|dW| {dw:.3e} (env {env_w:.3e}); score rel {ds:.3e} (env {env_s:.3e}); h abs {dh:.3e} (env {env_h:.3e})")
    parity("config2", dw, 2 * env_w, "full fit max|dW|")
    assert len(iters) == len(f["stages"])
    for a, l_, h_ in zip(iters, lo, hi):
        assert l_ - 1000 <= a <= h_ + 1000
    assert set(zip(rows.tolist(), cols.tolist())) == set(zip(gr.tolist(), gc.tolist()))
    assert dw <= 2 * env_w and ds <= 2 * env_s and dh <= 2 * env_h


def test_fit_stages_from_reference_start(hip, golden):
    """Each stage restarted from the oracle's own starting W: identical iteration
    counts in all five stages, W within 1e-9 for the non-chaotic stages."""
    from midagma_amd.solver import HipSolver
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = _oracle(X)
    sol = HipSolver(20)
    sol.set_cov(o.cov)
    W, mu = np.zeros((20, 20)), 1.0
    for i, s in enumerate([1.0, .9, .8, .7, .6]):
        K = 30000 if i < 4 else 60000
        Wg = W.copy()
        res = sol.minimize(Wg, mu, K, s, 3e-4, tol=1e-6, lambda1=0.03)
        W, tr = o.minimize(W.copy(), mu, K, s, 3e-4)
        assert res.iters == tr.iters and res.early_stop == tr.early_stop
        if i < 4:
            assert np.abs(Wg - W).max() <= 1e-9
        mu *= 0.1


def test_checkpoint_early_stop_matches_oracle(hip, golden):
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = _oracle(X)
    W_ref, tr = o.minimize(np.zeros((20, 20)), 1.0, 30000, 1.0, 3e-4, tol=1e-6)
    sol = _solver(20, o.cov)
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, 30000, 1.0, 3e-4, tol=1e-6, lambda1=0.03, want_checkpoints=True)
    assert res.early_stop == tr.early_stop and res.iters == tr.iters
    for (it, obj, sc, h, *_), (it2, obj2, sc2, h2) in zip(res.checkpoints, tr.checkpoints):
        assert it == it2
        assert abs(obj - obj2) <= 1e-9 * abs(obj2)
        assert abs(h - h2) <= 1e-9 + 1e-9 * abs(h2)


@pytest.mark.parametrize("d,K,s_dom", [(20, 100, 1.0), (300, 60, 1.0), (20, 50, 0.9)])
def test_float32_line_search_branches(hip, d, K, s_dom):
    """The domain line search on a float32 W (linear.py:230-241: revert W += lr g, lr /= 2,
    re-step W -= lr g, each rounded to float32) and the out-of-domain return: lr = 0.3 gives one
    halving at d = 20 and three at d = 300 (the blocked path), and s = 0.9 leaves the domain at
    iteration 2.  Iterations, halvings, the final lr and success equal the reference's float32
    arithmetic (the oracle with dtype=float32); W within 1e-6."""
    X, _, _ = make_dataset(d, 1000, seed=0)
    o = LinearOracle("l2", dtype=np.float32)
    o.prepare(X.copy(), 0.03, 1000)
    Wr, tr = o.minimize(np.zeros((d, d), dtype=np.float32), 1.0, K, s_dom, 0.3, tol=-1.0)
    sol = _solver(d, o.cov)
    sol.set_w_float32(True)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, s_dom, 0.3, tol=-1.0, lambda1=0.03)
    sol.close()
    assert (res.iters, res.halvings, res.success) == (tr.iters, tr.halvings, tr.success)
    assert res.lr_final == tr.lr_final
    assert np.array_equal(W, W.astype(np.float32).astype(np.float64))
    assert np.abs(W - Wr.astype(np.float64)).max() <= 1e-6


@pytest.mark.parametrize("d,loss", [(100, "l2"), (300, "l2"), (64, "logistic")])
def test_float32_data_mode_matches_reference_float32(hip, d, loss):
    """dtype=np.float32 in data mode (X on the device): l2 at d = 100 (D = 128) and 300 (the
    blocked inverse forked beside the GEMMs, I - W with its float32 diagonal from build_at), and
    logistic (X W with a float32-valued W; continuous X and lambda1 = 0, so no L1-kink chaos), 60
    steps from a float32 W = 0 against the oracle's float32 arithmetic (bit-exact to the
    reference's float32 fit).  Data mode sums X^T X (I - W) in another order than cov mode, so a
    float32 rounding may flip by an ulp: bound 1e-7 (the GPU's model, a float64 inverse rounded
    to float32, is within 2e-9 on the CPU), and where float64 W is measurably away from the float32
    trajectory (d = 300: 6e-5) at most 1% of that spread."""
    K, n = 60, 2000
    if loss == "l2":
        X, _, _ = make_dataset(d, n, seed=d + 7)
        lam = 0.03
    else:
        X = np.random.default_rng(d).normal(size=(n, d)) * 0.5
        lam = 0.0
    ref = {}
    for dt in (np.float32, np.float64):
        o = LinearOracle(loss, dtype=dt)
        o.prepare(X.copy(), lam, 1000)
        Wr, tr = o.minimize(np.zeros((d, d), dtype=dt), 1.0, K, 1.0, 3e-4, tol=-1.0)
        assert tr.iters == K
        ref[dt] = Wr.astype(np.float64)
        Xd = o.X  # (centred in place for l2)
    sol = _solver(d, Xd.T @ Xd / n, loss=loss, mode="data")
    sol.set_data(np.ascontiguousarray(Xd), n_global=n)
    sol.set_w_float32(True)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=lam)
    sol.close()
    assert res.iters == K
    assert np.array_equal(W, W.astype(np.float32).astype(np.float64))
    dev = float(np.abs(W - ref[np.float32]).max())
    spread = float(np.abs(ref[np.float64] - ref[np.float32]).max())
    assert dev <= 1e-7, (dev, spread)
    if spread > 1e-6:
        assert dev <= 0.01 * spread, (dev, spread)


# --------------------------------------------------------------------------- data mode / logistic
class _BlockedOracle(LinearOracle):
    """The oracle with X^T sigmoid(XW) summed in 64-row blocks: a summation order as
    valid as OpenBLAS's, used to measure the reference's own order sensitivity."""

    def score_grad(self, W, mu):
        from scipy.special import expit
        S = expit(self.X @ W)
        Z = np.zeros((self.d, self.d))
        for c in range(0, self.n, 64):
            Z += self.X[c:c + 64].T @ S[c:c + 64]
        return (mu / self.n) * Z - mu * self.cov


@pytest.mark.parametrize("K", [1, 10, 100, 1000])
def test_logistic_data_mode(hip, golden, K):
    """Logistic (data mode).  With binary X some score-gradient entries are exactly 0
    at W = 0 (e.g. (17,14) here); their rounding sign picks the L1 subgradient branch,
    so ANY summation order moves those few entries by O(lr).  Bound: the GPU is within
    2x the reference's own order envelope, and every entry outside it matches to 1e-9."""
    t = golden("traj_logistic_d20.npz")
    X = golden("data_meta.npz")["logit_X"].copy()
    o = _oracle(X, "logistic", 0.05)
    sol = _solver(20, o.cov, loss="logistic", mode="data")
    sol.set_data(X, n_global=X.shape[0])
    W = np.zeros((20, 20))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.05)
    assert res.success and res.iters == K
    ref = t[f"W_K{K}"]
    ob = _BlockedOracle("logistic")
    ob.prepare(X.copy(), 0.05, 1000)
    Wb, _ = ob.minimize(np.zeros((20, 20)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    env = np.abs(Wb - ref)
    chaotic = env > 1e-9
    assert np.abs(W - ref).max() <= max(1e-5, 2 * env.max())
    assert np.abs(W - ref)[~chaotic].max() <= 1e-9
    assert chaotic.sum() <= 0.1 * W.size


@pytest.mark.parametrize("K", [1, 10, 100, 500])
def test_logistic_data_mode_d100(hip, golden, K):
    """Logistic at d=100, n=3000 (D=128: the 128-tile pipelined GEMM with the sigmoid epilogue)
    against the reference's own minimize (traj_logistic_d100.npz, make_golden.py
    gen_traj_logistic_d100).  Same bound as the d=20 case: within 2x the reference's
    summation-order envelope (64-row blocked X^T S), entries outside it to 1e-9."""
    t = golden("traj_logistic_d100.npz")
    X = golden("data_logistic_d100.npz")["X"].copy()
    d = X.shape[1]
    o = _oracle(X, "logistic", 0.05)
    sol = _solver(d, o.cov, loss="logistic", mode="data")
    sol.set_data(X, n_global=X.shape[0])
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.05)
    assert res.success and res.iters == K == int(t[f"it_K{K}"])
    ref = t[f"W_K{K}"]
    ob = _BlockedOracle("logistic")
    ob.prepare(X.copy(), 0.05, 1000)
    Wb, _ = ob.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    env = np.abs(Wb - ref)
    # At d=100 about a quarter of the entries sit on the L1 kink (|score gradient| < mu*lambda1):
    # they chatter around 0 with amplitude ~lr and their sign follows the last rounding bit, in
    # the reference itself as much as here (the blocked order moves ~23% of them by up to 3e-4).
    # Bound: no entry further than 2x the reference's own envelope, no more entries moved than
    # it moves (+50%), and the objective's data-fit term equal to 1e-9 relative.
    diff = np.abs(W - ref)
    assert diff.max() <= max(1e-5, 2 * env.max())
    assert (diff > 1e-9).sum() <= 1.5 * (env > 1e-9).sum() + 10
    from oracle.dagma_oracle import score
    l_gpu, _ = score("logistic", W, o.cov, o.X)
    l_ref, _ = score("logistic", ref, o.cov, o.X)
    l_blk, _ = score("logistic", Wb, o.cov, o.X)
    assert abs(l_gpu - l_ref) <= max(1e-9 * abs(l_ref), 2 * abs(l_blk - l_ref))


def test_l2_data_mode_matches_cov_mode(hip):
    X, _, _ = make_dataset(100, 3000, seed=5)
    o = _oracle(X)
    Xc = o.X  # centered
    a = _solver(100, o.cov)
    b = _solver(100, o.cov, mode="data")
    b.set_data(Xc, n_global=Xc.shape[0])
    Wa, Wb = np.zeros((100, 100)), np.zeros((100, 100))
    ra = a.minimize(Wa, 1.0, 300, 1.0, 3e-4, tol=-1.0)
    rb = b.minimize(Wb, 1.0, 300, 1.0, 3e-4, tol=-1.0)
    assert ra.iters == rb.iters == 300
    assert np.abs(Wa - Wb).max() <= 1e-9
    Wr, _ = o.minimize(np.zeros((100, 100)), 1.0, 300, 1.0, 3e-4, tol=-1.0)
    assert np.abs(Wb - Wr).max() <= 1e-9


def test_data_mode_full_size_config4(hip, parity):
    """The headline workload at its full size on one GPU (BASELINE config 4, d=1000, n=1e6):
    X from the GPU SEM generator, centered on the host as fit() does (linear.py:411); data
    mode (two n x d MFMA GEMMs per step, forked blocked inverse) against the oracle's
    reference-algorithm steps on cov = X^T X / n.  Same W after 5 Adam steps."""
    from midagma_amd.simulate import simulate_er_dag, simulate_weights
    from midagma_amd.utils import simulate_linear_sem_gpu
    d, n, K = 1000, 1_000_000, 5
    rng = np.random.default_rng(0)
    W_true = simulate_weights(simulate_er_dag(d, d, rng), rng)
    Xh = simulate_linear_sem_gpu(W_true, n, "gauss", seed=17, device=0).cpu().numpy()
    o = LinearOracle("l2")
    o.prepare(Xh, 0.03, 1000)  # centers Xh in place, cov = X^T X / n
    sol = _solver(d, mode="data")
    sol.set_data(Xh, n_global=n)
    del Xh
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0)
    o.X = None
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    parity("config4", float(np.abs(W - Wr).max()), 1e-9, f"max|dW| K={K}")
    assert res.iters == tr.iters == K and res.success
    assert np.abs(W - Wr).max() <= 1e-9
    sol.close()


def test_data_mode_score_and_gram(hip):
    X, _, _ = make_dataset(70, 1000, seed=9)
    X = X - X.mean(0)
    sol = _solver(70, mode="data")
    sol.set_data(X, n_global=X.shape[0])
    sol.data_gram()
    sol.cov_from_zbuf(X.shape[0])
    cov = X.T @ X / X.shape[0]
    rng = np.random.default_rng(2)
    W = rng.normal(size=(70, 70)) * 0.1
    sol.score_partial(W)
    l, G = sol.score_finish()
    l_ref, G_ref = score("l2", W, cov)
    assert abs(l - l_ref) <= 1e-11 * abs(l_ref) and _rel(G, G_ref) <= 1e-11


# --------------------------------------------------------------------------- large d (properties)
@pytest.mark.parametrize("d", [1000, 2000])
def test_inverse_large_d(hip, d):
    """At the bench size: GJ inverse vs LAPACK, and the Neumann-series identity."""
    import scipy.linalg as sla
    rng = np.random.default_rng(d)
    W = (rng.uniform(-1, 1, (d, d)) * (rng.uniform(size=(d, d)) < 4.0 / d)) * 0.4
    np.fill_diagonal(W, 0)
    sol = _solver(d)
    h, G = sol.h_value(W, 1.0)
    A = np.eye(d) - W * W
    M = sla.inv(A)
    assert _rel(G, 2 * W * M.T) <= 1e-11
    h_ref = -np.linalg.slogdet(A)[1]
    assert abs(h - h_ref) <= 1e-10 * max(1, abs(h_ref))


def test_minimize_d1000_short(hip):
    d = 1000
    X, _, _ = make_dataset(d, 2000, seed=11)
    o = _oracle(X)
    sol = _solver(d, o.cov)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, 3, 1.0, 3e-4, tol=-1.0)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 3, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == 3
    assert np.abs(W - Wr).max() <= 1e-10


@pytest.mark.parametrize("d", [300, 600, 1000, 1150, 1400, 2000])
def test_blocked_fast_path_trajectory(hip, d):
    """Cov mode at d > 192 runs the two-level blocked inverse: warm-started fast slots between
    Gauss-Jordan slots (first slot, every checkpoint).  d=300 -> D=512 (cov mode pads
    256 < d <= 640 to 256-multiples: B2=256, 2 outer blocks), 600 -> 768 (B2=256, 3), 1000 ->
    1024 (B2=256, 4; score GEMM split-K 4), 1150 ->
    1152 (B2=128, 9; split 3), 1400 -> 1408 (B2=128, 11; split 2), 2000 -> 2048 (B2=256, 8;
    trailing update on the 128-tile GEMM).  Same iterations, W and checkpoint objectives as
    the oracle (LAPACK inverse)."""
    X, _, _ = make_dataset(d, 2 * d, seed=d)
    o = _oracle(X)
    o.checkpoint = 40
    K = 130 if d < 2000 else 90
    sol = _solver(d, o.cov)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=40, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == K and res.success
    assert np.abs(W - Wr).max() <= 1e-9
    got = [(c[0], c[1], c[3]) for c in res.checkpoints]
    assert [g[0] for g in got] == [c[0] for c in tr.checkpoints] == list(range(40, K, 40)) + [K]
    for (it, obj, h), (_, obj_r, _, h_r) in zip(got, tr.checkpoints):
        assert abs(obj - obj_r) <= 1e-10 * abs(obj_r) and abs(h - h_r) <= 1e-9 * max(1.0, abs(h_r))


def test_blocked_path_line_search(hip):
    """The domain line search (linear.py:230-241) on the blocked-inverse path: at d=300, lr=0.3
    the reference halves lr three times in 60 steps.  The fast slots take the domain flags from
    the last outer step, a halving turns the warm start back to the plain previous inverse, and
    far warm starts hand back to the GJ slot; iterations, halvings, lr and W match the oracle."""
    d = 300
    X, _, _ = make_dataset(d, 2 * d, seed=7)
    o = _oracle(X)
    o.checkpoint = 20
    sol = _solver(d, o.cov)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, 60, 1.0, 0.3, tol=-1.0, lambda1=0.03, checkpoint=20)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 60, 1.0, 0.3, tol=-1.0)
    assert tr.halvings == 3
    assert (res.iters, res.success, res.halvings) == (tr.iters, tr.success, tr.halvings)
    assert res.lr_final == tr.lr_final
    assert np.abs(W - Wr).max() <= 1e-8


def test_large_d_split_k_score_and_trajectory(hip):
    """d=4500 -> D=4608: the cov score GEMM runs split-K 3 (1296 128-tiles, last-wave
    rounding) with the k loop trimmed to 4512, the fast slots sum the 3 slices inside
    fused_update, and the trailing update runs on the 128-tile GEMM over 18 outer blocks.
    _score at a dense W and 8 Adam steps (checkpoints every 4: GJ and fast slots) against the
    oracle (LAPACK inverse)."""
    d = 4500
    X, _, _ = make_dataset(d, 2 * d, seed=5)
    o = _oracle(X)
    o.checkpoint = 4
    sol = _solver(d, o.cov)
    rng = np.random.default_rng(2)
    Wd = rng.normal(size=(d, d)) * 0.01
    l, G = sol.score_value(Wd)
    l_ref, G_ref = score("l2", Wd, o.cov)
    assert abs(l - l_ref) <= 1e-12 * abs(l_ref)
    assert _rel(G, G_ref) <= 1e-12
    K = 8
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=4, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert res.iters == tr.iters == K and res.success
    assert np.abs(W - Wr).max() <= 1e-9
    for c, (_, obj_r, _, h_r) in zip(res.checkpoints, tr.checkpoints):
        assert abs(c[1] - obj_r) <= 1e-10 * abs(obj_r) and abs(c[3] - h_r) <= 1e-9 * max(1.0, abs(h_r))


CKPT_FIELDS = {"obj_total": "obj", "score_datafit": "score", "reg_dag_value": "h", "lr": "lr", "w_abs_sum": "l1",
               "w_norm": "w_norm", "max_abs_w": "max_abs_w", "min_abs_w_nonzero": "min_abs_w_nonzero",
               "grad_raw_norm": "grad_raw_norm", "grad_step_norm": "grad_step_norm",
               "grad_score_norm": "grad_score_norm", "grad_dag_norm": "grad_dag_norm",
               "grad_l1_norm": "grad_l1_norm", "grad_inc_norm": "grad_inc_norm"}


@pytest.mark.parametrize("d", [20, 300])
def test_checkpoint_records_match_oracle(hip, golden, d):
    """minimize.checkpoint numeric fields (linear.py:262-326) from the device records equal the
    oracle's, with include/exclude masks so every norm is non-trivial.  d=300 runs the
    blocked-inverse path (fast slots between the GJ checkpoint slots)."""
    if d == 20:
        X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    else:
        X, _, _ = make_dataset(d, 2 * d, seed=3)
    exc, inc = ((0, 1), (2, 3), (5, 4)), ((4, 5), (7, 8))
    o = _oracle(X, exc=exc, inc=inc)
    o.checkpoint = 50
    mi, me = o.masks(1.0)
    sol = _solver(d, o.cov)
    sol.set_masks(mi, me)
    W = np.zeros((d, d))
    res = sol.minimize(W, 1.0, 130, 1.0, 3e-4, tol=-1.0, lambda1=0.03, checkpoint=50, want_checkpoints=True)
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, 130, 1.0, 3e-4, tol=-1.0)
    assert np.abs(W - Wr).max() <= 1e-9
    got = res.checkpoints
    assert [c.iter for c in got] == [r["iter"] for r in tr.records] == [50, 100, 130]
    for c, r in zip(got, tr.records):
        for key, attr in CKPT_FIELDS.items():
            a, b = getattr(c, attr), r[key]
            assert abs(a - b) <= 1e-9 * max(1e-12, abs(b)), (c.iter, key, a, b)
        assert 0.0 <= c.elapsed < 60.0


def test_dagma_linear_emits_checkpoint_rows(hip, golden):
    """fit() with logging on: one reference-schema row per checkpoint of every stage."""
    from midagma_amd import DagmaLinear
    from midagma_amd.slog import LogConfig
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    m = DagmaLinear("l2", log_cfg=LogConfig(enabled=True, store_jsonl=False))
    m.fit(X, lambda1=0.03, T=2, warm_iter=300, max_iter=500, checkpoint=100)
    rows = m._slog.load(event="minimize.checkpoint")
    calls = m.minimize_log
    assert len(rows["iter"]) == sum(-(-c["iters"] // 100) for c in calls)
    assert set(rows["reg_dag_name"]) == {"dagma_logdet"} and set(rows["mu"]) == {1.0, 0.1}
    assert all(float(v) >= 0.0 for v in rows["grad_dag_norm"])


# --------------------------------------------------------------------------- DagmaMLP h_func
@pytest.mark.parametrize("d", [20, 200])
@pytest.mark.parametrize("s", [1.0, 0.8])
def test_mlp_h_func(hip, golden, d, s):
    from midagma_amd.nonlinear import DagmaMLP
    from tests.golden.inputs import mlp_fc1
    g = golden("mlp_h.npz")
    dev = torch.device("cuda", 0)
    model = DagmaMLP([d, 10, 1]).to(dev)
    with torch.no_grad():
        model.fc1.weight.copy_(torch.from_numpy(mlp_fc1(d, 10)))
    h = model.h_func(s)
    h.backward()
    assert abs(h.item() - float(g[f"h_d{d}_s{s}"])) <= 1e-12 * max(1.0, abs(float(g[f"h_d{d}_s{s}"])))
    grad = model.fc1.weight.grad.detach().cpu().numpy().reshape(-1)[g[f"pick_d{d}"]]
    np.testing.assert_allclose(grad, g[f"gradpick_d{d}_s{s}"], rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("d,n", [(300, 2000), (1000, 4000), (300, 20000)])
def test_data_mode_shard_inverse_paths(hip, d, n):
    """Data-mode shards of <= 16384 rows run the cov-mode slot structure (the warm-started fast
    blocked inverse, forked beside the GEMMs; pivoted slots at the first step, checkpoints and
    hand-backs); larger shards fork the pivoted blocked inverse beside the GEMMs (n=20000).  l2
    against the oracle's reference-algorithm steps (K=130, checkpoints every 40: iterations, W
    and the checkpoint objectives)."""
    X, _, _ = make_dataset(d, n, seed=d + 3)
    o = _oracle(X)
    o.checkpoint = 40
    K = 130
    s = _solver(d, mode="data")
    s.set_data(o.X, n_global=n)
    W = np.zeros((d, d))
    r = s.minimize(W, 1.0, K, 1.0, 3e-4, tol=-1.0, checkpoint=40, want_checkpoints=True)
    s.close()
    Wr, tr = o.minimize(np.zeros((d, d)), 1.0, K, 1.0, 3e-4, tol=-1.0)
    assert r.iters == tr.iters == K and r.success
    assert np.abs(W - Wr).max() <= 1e-9
    assert len(r.checkpoints) == len(tr.checkpoints)
    for c, (_, obj_r, _, _) in zip(r.checkpoints, tr.checkpoints):
        assert abs(c[1] - obj_r) <= 1e-10 * abs(obj_r)
