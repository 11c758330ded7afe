"""Generate the golden fixtures by running the REFERENCE in this container.

Run (build container only -- the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=1 OMP_NUM_THREADS=1 \
        python tests/golden/make_golden.py

It imports fbleile/midagma from /root/reference/src (read-only) and records
inputs + outputs of `DagmaLinear._h/_score/_adam_update/minimize/fit`
(`src/dagma/linear.py`) and `DagmaMLP.h_func` (`src/dagma/nonlinear.py:68-86`)
into small .npz files next to this script.  Inputs come from the build's own
numpy SEM generator (`midagma_amd.simulate`, seeded), because the reference's
generator needs igraph, which is not installed.

BLAS is pinned to one thread: the last bits of dgemm/dgetrf depend on the
thread count, and the oracle test demands bit-equality.
"""
from __future__ import annotations

import os
import sys

for _v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ.setdefault(_v, "1")
os.environ.setdefault("TQDM_DISABLE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/src")

from threadpoolctl import threadpool_limits  # noqa: E402

import dagma.linear as ref_linear  # noqa: E402
from dagma.linear import DagmaLinear  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402
from tests.golden.inputs import mlp_fc1  # noqa: E402


class Recorder:
    """Stand-in for the tqdm bar `minimize` calls `update` on (linear.py:329, 332)."""

    def __init__(self):
        self.units = 0
        self.big = 0

    def update(self, k=1):
        if k == 1:
            self.units += 1
        else:
            self.big += 1

    @property
    def iters(self):
        return self.units + (1 if self.big else 0)


def setup_model(X, loss="l2", lambda1=0.03, checkpoint=1000, exclude=None, include=None):
    """Replicate fit()'s data preparation (linear.py:406-429) on a fresh model."""
    m = DagmaLinear(loss_type=loss, verbose=False)
    X = X.copy()
    m.X, m.lambda1, m.checkpoint = X, lambda1, checkpoint
    m.n, m.d = X.shape
    m.Id = np.eye(m.d).astype(m.dtype)
    if loss == "l2":
        m.X -= X.mean(axis=0, keepdims=True)
    m.exc_r = m.exc_c = m.inc_r = m.inc_c = None
    if exclude is not None:
        m.exc_r, m.exc_c = zip(*exclude)
    if include is not None:
        m.inc_r, m.inc_c = zip(*include)
    m.cov = X.T @ X / float(m.n)
    return m


def run_minimize(m, W0, mu, K, s, lr, tol=-1.0):
    rec = Recorder()
    W, ok = m.minimize(W0.copy(), mu, K, s, lr, tol=tol, pbar=rec)
    return W, ok, rec.iters


def in_domain_W(d, rng, scale):
    """A random dense W inside the M-matrix domain (spectral radius of W*W < s)."""
    W = rng.uniform(-1, 1, size=(d, d)) * scale
    np.fill_diagonal(W, 0.0)
    return W


class NoisyInv:
    """scipy.linalg stand-in whose inv() adds 1e-16 relative noise (SURVEY.md 8c envelope)."""

    def __init__(self, rng):
        import scipy.linalg as sla
        self._sla, self._rng = sla, rng

    def inv(self, A):
        M = self._sla.inv(A)
        return M * (1.0 + 1e-16 * self._rng.standard_normal(M.shape))

    def __getattr__(self, k):
        return getattr(self._sla, k)


def with_noisy_inv(fn, seed=123):
    orig = ref_linear.sla
    ref_linear.sla = NoisyInv(np.random.default_rng(seed))
    try:
        return fn()
    finally:
        ref_linear.sla = orig


def gen_data():
    X, W, B = make_dataset(20, 1000, seed=0)
    np.savez_compressed(os.path.join(HERE, "data_d20_n1000_seed0.npz"), X=X, W_true=W, B_true=B)
    X1, W1, B1 = make_dataset(100, 2000, seed=1)
    Xl, Wl, Bl = make_dataset(20, 1000, seed=2, sem_type="logistic")
    np.savez_compressed(os.path.join(HERE, "data_meta.npz"),
                        d100_sum=X1.sum(), d100_row0=X1[0], d100_Wtrue=W1,
                        logit_X=Xl, logit_W_true=Wl)
    return X, X1, Xl


def gen_blocks(X20, Xl):
    rng = np.random.default_rng(7)
    out = {}
    # G1 _h
    for d, scale in ((5, 0.3), (20, 0.12), (100, 0.05)):
        W = in_domain_W(d, rng, scale)
        out[f"h_W_d{d}"] = W
        for s in (1.0, 0.9, 0.6):
            m = setup_model(np.zeros((2, d)) + np.arange(d), "l2")
            h, G = m._h(W, s)
            key = f"d{d}_s{s}"
            out[f"h_val_{key}"] = np.array(h)
            out[f"h_grad_{key}"] = G
    # G2 _score, l2 and logistic at d=20
    W = in_domain_W(20, rng, 0.1)
    out["score_W"] = W
    m = setup_model(X20, "l2")
    l, G = m._score(W)
    out["score_l2_loss"], out["score_l2_grad"] = np.array(l), G
    ml = setup_model(Xl, "logistic")
    l, G = ml._score(W)
    out["score_logistic_loss"], out["score_logistic_grad"] = np.array(l), G
    # G3 _adam_update: five steps of a fixed gradient sequence
    m.opt_m, m.opt_v = 0, 0
    gs = rng.standard_normal((5, 20, 20))
    out["adam_g"] = gs
    out["adam_out"] = np.stack([m._adam_update(gs[k], k + 1, 0.99, 0.999) for k in range(5)])
    np.savez_compressed(os.path.join(HERE, "blocks.npz"), **out)


def gen_traj(X, tag, Ks, lr=3e-4, mu=1.0, s=1.0, loss="l2", lambda1=0.03):
    """W after K steps (tol=-1: no early stop) + the 1e-16-noise envelope per K."""
    out = {"Ks": np.array(Ks)}
    d = X.shape[1]
    W0 = np.zeros((d, d))
    for K in Ks:
        m = setup_model(X, loss, lambda1=lambda1)
        W, ok, it = run_minimize(m, W0, mu, K, s, lr)
        out[f"W_K{K}"], out[f"ok_K{K}"], out[f"it_K{K}"] = W, np.array(ok), np.array(it)
        m2 = setup_model(X, loss, lambda1=lambda1)
        Wn, _, _ = with_noisy_inv(lambda: run_minimize(m2, W0, mu, K, s, lr))
        out[f"env_K{K}"] = np.array(np.abs(Wn - W).max())
    np.savez_compressed(os.path.join(HERE, f"traj_{tag}.npz"), **out)


def gen_traj_logistic_d100():
    """Logistic at d=100 (D=128: the 128-tile pipelined GEMM with the sigmoid epilogue on the
    GPU side).  Binary X from the logistic SEM (seed 9, n=3000); the reference's minimize at
    K = 1, 10, 100, 500 and the same run with 1e-16 noise in every inverse (the envelope)."""
    Xl, _, _ = make_dataset(100, 3000, seed=9, sem_type="logistic")
    np.savez_compressed(os.path.join(HERE, "data_logistic_d100.npz"), X=Xl)
    gen_traj(Xl, "logistic_d100", [1, 10, 100, 500], loss="logistic", lambda1=0.05)


def gen_branches(X):
    out = {}
    d = X.shape[1]
    W0 = np.zeros((d, d))
    # lr-halving path: large lr at s=1.0 (linear.py:234-241)
    m = setup_model(X, "l2")
    msgs = []
    m.vprint = lambda *a, **k: msgs.append(" ".join(str(x) for x in a))
    W, ok, it = run_minimize(m, W0, 1.0, 60, 1.0, 0.3)
    out["halve_W"], out["halve_ok"], out["halve_it"] = W, np.array(ok), np.array(it)
    out["halve_nhalvings"] = np.array(sum("Learning rate decreased" in x for x in msgs))
    # out-of-domain at s <= 0.9 (linear.py:231-233)
    m = setup_model(X, "l2")
    W, ok, it = run_minimize(m, W0, 1.0, 60, 0.9, 0.3)
    out["ood_W"], out["ood_ok"], out["ood_it"] = W, np.array(ok), np.array(it)
    # include / exclude edge masks (linear.py:217-222, 276)
    exc = ((0, 1), (2, 3), (5, 4))
    inc = ((1, 0), (3, 7))
    m = setup_model(X, "l2", exclude=exc, include=inc)
    W, ok, it = run_minimize(m, W0, 1.0, 500, 1.0, 3e-4)
    out["mask_W"], out["mask_exc"], out["mask_inc"] = W, np.array(exc), np.array(inc)
    np.savez_compressed(os.path.join(HERE, "branches.npz"), **out)


def gen_fit(X):
    """Full default fit at d=20 with per-stage iteration counts."""
    calls = []

    class Spy(DagmaLinear):
        def minimize(self, W, mu, max_iter, s, lr, tol=1e-6, beta_1=0.99, beta_2=0.999, pbar=None):
            rec = Recorder()
            Wr, ok = super().minimize(W, mu, max_iter, s, lr, tol, beta_1, beta_2, pbar=rec)
            calls.append((mu, s, lr, max_iter, ok, rec.iters))
            return Wr, ok

        def _h(self, W, s=1.0):
            self.last_h_W = W.copy()  # the final call (linear.py:456) sees the pre-threshold W
            return super()._h(W, s)

    def one_fit():
        calls.clear()
        m = Spy(loss_type="l2", verbose=False)
        W = m.fit(X.copy(), lambda1=0.03, s=[1.0, .9, .8, .7, .6])
        return m, W, list(calls)

    m, W, c = one_fit()
    m2, W2, c2 = with_noisy_inv(one_fit, seed=99)
    out = {"W": W, "W_unthresholded": m.last_h_W, "calls": np.array(c, dtype=np.float64),
           "h_final": np.array(m.h_final), "score_final": np.array(m.score_final),
           "W_noisy": W2, "W_unthresholded_noisy": m2.last_h_W,
           "h_final_noisy": np.array(m2.h_final), "score_final_noisy": np.array(m2.score_final),
           "calls_noisy": np.array(c2, dtype=np.float64)}
    np.savez_compressed(os.path.join(HERE, "fit_d20.npz"), **out)


def gen_fit_envelope(X, seeds=(7, 11, 13, 17, 19, 23, 29, 31)):
    """Several 1e-16-noise replicas of the default d=20 fit: the spread of the chaotic
    last stage (iteration count, h_final, score_final, W) over noise seeds."""
    rows = {"W_unthresholded": [], "h_final": [], "score_final": [], "last_iters": []}

    class Spy(DagmaLinear):
        def minimize(self, W, mu, max_iter, s, lr, tol=1e-6, beta_1=0.99, beta_2=0.999, pbar=None):
            rec = Recorder()
            Wr, ok = super().minimize(W, mu, max_iter, s, lr, tol, beta_1, beta_2, pbar=rec)
            self.last_iters = rec.iters
            return Wr, ok

        def _h(self, W, s=1.0):
            self.last_h_W = W.copy()
            return super()._h(W, s)

    def one_fit():
        m = Spy(loss_type="l2", verbose=False)
        m.fit(X.copy(), lambda1=0.03, s=[1.0, .9, .8, .7, .6])
        return m

    for sd in seeds:
        m = with_noisy_inv(one_fit, seed=sd)
        rows["W_unthresholded"].append(m.last_h_W)
        rows["h_final"].append(m.h_final)
        rows["score_final"].append(m.score_final)
        rows["last_iters"].append(m.last_iters)
    np.savez_compressed(os.path.join(HERE, "fit_d20_envelope.npz"), seeds=np.array(seeds),
                        **{k: np.array(v, dtype=np.float64) for k, v in rows.items()})


def gen_fit_f32(X):
    """A shortened fit (T = 3) with dtype=np.float32 and the same fit with float64: the reference
    keeps W in float32 through its in-place Adam updates (linear.py:275, 429), so the two runs
    differ by float32 rounding; the pair bounds the dtype=float32 drop-in."""
    out = {}
    for tag, dt in (("f32", np.float32), ("f64", np.float64)):
        calls = []
        m = _stage_spy(calls)(loss_type="l2", verbose=False, dtype=dt)
        W = m.fit(X.copy(), lambda1=0.03, T=3, s=[1.0, .9, .8], warm_iter=4000, max_iter=5000)
        out[f"W_{tag}"] = W
        out[f"h_final_{tag}"] = np.array(m.h_final)
        out[f"score_final_{tag}"] = np.array(m.score_final)
        # per minimize call: (mu, s, lr, max_iter, success, iterations) -- the float32 checkpoint
        # objective decides where each stage stops early (linear.py:113-114, 127, 328-331)
        out[f"calls_{tag}"] = np.array(calls, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "fit_f32_d20.npz"), **out)


def _stage_spy(calls):
    """DagmaLinear recording (mu, s, lr, max_iter, success, iterations) of every minimize call."""
    class Spy(DagmaLinear):
        def minimize(self, W, mu, max_iter, s, lr, tol=1e-6, beta_1=0.99, beta_2=0.999, pbar=None):
            rec = Recorder()
            Wr, ok = super().minimize(W, mu, max_iter, s, lr, tol, beta_1, beta_2, pbar=rec)
            calls.append((mu, s, lr, max_iter, ok, rec.iters))
            return Wr, ok
    return Spy


def gen_fit_f32_default(X, seeds=(7, 11, 13, 17, 19, 23, 29, 31)):
    """The DEFAULT fit (T=5, warm 3e4, max 6e4) with dtype=np.float32, whose stages stop early on
    the float32 checkpoint objective (linear.py:113-114, 127, 328-331), with its per-call
    iteration counts; and the same fit under float32-scale noise in every inverse (NoisyInv32),
    one run per seed: the range of stage counts the reference's own float32 rounding allows."""
    calls = []
    m = _stage_spy(calls)(loss_type="l2", verbose=False, dtype=np.float32)
    W = m.fit(X.copy(), lambda1=0.03)
    out = {"W": W, "h_final": np.array(m.h_final), "score_final": np.array(m.score_final),
           "calls": np.array(calls, dtype=np.float64)}
    env = []
    orig = ref_linear.sla
    for sd in seeds:
        ref_linear.sla = NoisyInv32(np.random.default_rng(sd))
        try:
            c = []
            _stage_spy(c)(loss_type="l2", verbose=False, dtype=np.float32).fit(X.copy(), lambda1=0.03)
        finally:
            ref_linear.sla = orig
        env.append([x[5] for x in c])
    n = max(len(e) for e in env)
    out["env_seeds"] = np.array(seeds)
    out["env_stage_iters"] = np.array([e + [-1] * (n - len(e)) for e in env], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "fit_f32_d20_default.npz"), **out)


class NoisyInv32(NoisyInv):
    """float32 stand-in: the float32 inverse with one-ulp-scale relative noise (2^-24 N(0, 1)) in
    every entry -- the size of the difference between two valid float32 inversions."""

    def inv(self, A):
        M = self._sla.inv(A)
        if M.dtype != np.float32:
            return M * (1.0 + 1e-16 * self._rng.standard_normal(M.shape))
        return (M * (1.0 + 2.0 ** -24 * self._rng.standard_normal(M.shape))).astype(np.float32)


def gen_fit_f32_envelope(X, seeds=(7, 11, 13, 17, 19, 23, 29, 31)):
    """The dtype=np.float32 fit of gen_fit_f32 under float32-scale noise in every inverse
    (NoisyInv32), one run per seed: the reference's own float32 perturbation envelope, the bar of
    tests/test_gpu_parity.py::test_full_fit_float32_dtype (the GPU's float32 loop inverts in
    float64 and rounds, a different valid float32 inversion)."""
    rows = {"W": [], "h_final": [], "score_final": [], "stage_iters": []}

    def one_fit():
        calls = []
        m = _stage_spy(calls)(loss_type="l2", verbose=False, dtype=np.float32)
        W = m.fit(X.copy(), lambda1=0.03, T=3, s=[1.0, .9, .8], warm_iter=4000, max_iter=5000)
        m.stage_iters = [c[5] for c in calls]
        return m, W

    orig = ref_linear.sla
    for sd in seeds:
        ref_linear.sla = NoisyInv32(np.random.default_rng(sd))
        try:
            m, W = one_fit()
        finally:
            ref_linear.sla = orig
        rows["W"].append(W.astype(np.float64))
        rows["h_final"].append(float(m.h_final))
        rows["score_final"].append(float(m.score_final))
        rows["stage_iters"].append(m.stage_iters)
    np.savez_compressed(os.path.join(HERE, "fit_f32_d20_envelope.npz"), seeds=np.array(seeds),
                        **{k: np.array(v, dtype=np.float64) for k, v in rows.items()})


def gen_trek():
    """PST trek regularizer value and gradient from the reference (notreks.trek_value_grad)
    for every seq and agg it offers, on a small in-domain W."""
    from notreks.notreks import PSTRegularizer, trek_value_grad
    rng = np.random.default_rng(17)
    out = {}
    for d in (8, 20):
        W = in_domain_W(d, rng, 0.35)
        pairs = np.array([(i, j) for i in range(d) for j in range(i + 1, d) if rng.uniform() < 0.3], dtype=np.int64)
        out[f"W_d{d}"], out[f"pairs_d{d}"] = W, pairs
        for seq in ("exp", "inv", "log", "binom"):
            for agg in ("mean", "sum", "max", "lse"):
                kw = {"agg": agg}
                if seq == "log":
                    kw["K_log"] = 12
                tr = PSTRegularizer(I=pairs, seq=seq, weight=0.5, kwargs=kw, mode="opt")
                v, g = trek_value_grad(W.copy(), tr)
                out[f"val_{seq}_{agg}_d{d}"] = np.array(v)
                out[f"grad_{seq}_{agg}_d{d}"] = g
    np.savez_compressed(os.path.join(HERE, "trek_pst.npz"), **out)


def tcc_cases(d, rng):
    """(name, W) inputs for the TCC fixtures: dense in-domain, tiny (start of a fit), and a
    weighted DAG (W o W nilpotent: the Perron structure comes from the S / I coupling)."""
    dense = in_domain_W(d, rng, 0.35)
    tiny = in_domain_W(d, rng, 1e-3)
    B = np.tril(rng.uniform(size=(d, d)) < 0.2, -1)
    dag = B * rng.uniform(0.5, 1.5, (d, d)) * rng.choice([-1.0, 1.0], (d, d))
    p = rng.permutation(d)
    return [("dense", dense), ("tiny", tiny), ("dag", dag[np.ix_(p, p)])]


def gen_tcc(X20):
    """TCC trek regularizer from the reference: trek_value_grad (the loop's entry: spectral,
    approx_trek_graph, numpy eig) on several W, and minimize trajectories with it at d=20."""
    from notreks.notreks import TCCRegularizer, trek_value_grad
    rng = np.random.default_rng(23)
    out = {}
    for d in (8, 20):
        pairs = np.array([(i, j) for i in range(d) for j in range(i + 1, d) if rng.uniform() < 0.3], dtype=np.int64)
        out[f"pairs_d{d}"] = pairs
        for name, W in tcc_cases(d, rng):
            out[f"W_{name}_d{d}"] = W
            for w in (1.0, 2.0):
                tr = TCCRegularizer(I=pairs, weight=0.5, w=w, mode="opt")
                v, g = trek_value_grad(W.copy(), tr)
                out[f"val_{name}_w{w:g}_d{d}"] = np.array(v)
                out[f"grad_{name}_w{w:g}_d{d}"] = g
    # the loop (linear.py:251-258, 122-133): opt mode (gradient every step) and log mode
    d = X20.shape[1]
    pairs = out["pairs_d20"]
    out["traj_Ks"] = np.array([1, 10, 90])
    for mode in ("opt", "log"):
        for K in (1, 10, 90):
            m = setup_model(X20, "l2", checkpoint=40)
            m.trek_reg = TCCRegularizer(I=pairs, weight=0.2, mode=mode)
            W, ok, it = run_minimize(m, np.zeros((d, d)), 1.0, K, 1.0, 3e-4)
            out[f"traj_{mode}_W_K{K}"], out[f"traj_{mode}_it_K{K}"] = W, np.array(it)
    np.savez_compressed(os.path.join(HERE, "trek_tcc.npz"), **out)


def gen_mlp_traj(X20):
    """DagmaNonlinear.minimize (nonlinear.py:161-236) from fixed parameters, and a short fit,
    at dims [20, 10, 1]: every parameter after K Adam steps."""
    import torch
    from dagma.nonlinear import DagmaMLP, DagmaNonlinear
    from tests.golden.inputs import mlp_params
    torch.set_default_dtype(torch.double)
    d, m1 = X20.shape[1], 10
    P0 = mlp_params(d, m1)
    out = {f"p0_{k}": v for k, v in P0.items()}

    def fresh():
        model = DagmaMLP(dims=[d, m1, 1], bias=True, dtype=torch.double)
        sd = model.state_dict()
        with torch.no_grad():
            for k, v in P0.items():
                sd[k].copy_(torch.from_numpy(v))
        dn = DagmaNonlinear(model)
        dn.X = torch.from_numpy(X20).type(torch.double)
        dn.checkpoint = 1000
        return model, dn

    for K in (1, 10, 100):
        model, dn = fresh()
        ok = dn.minimize(K, 2e-4, 0.02, 0.005, 0.1, 1.0, pbar=Recorder())
        out[f"ok_K{K}"] = np.array(ok)
        for k, v in model.state_dict().items():
            out[f"K{K}_{k}"] = v.detach().numpy().copy()
    model, dn = fresh()
    W = dn.fit(X20, T=2, warm_iter=300, max_iter=500)
    out["fit_W"] = W
    for k, v in model.state_dict().items():
        out[f"fit_{k}"] = v.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, "mlp_traj.npz"), **out)


def gen_mlp():
    """DagmaMLP.h_func value and autograd gradient (nonlinear.py:68-86).

    fc1 weights come from numpy (seeded) so they are regenerable; for d=200 only
    a seeded sample of the (2000 x 200) gradient is stored to keep the file small.
    """
    import torch
    from dagma.nonlinear import DagmaMLP
    out = {}
    for d, m1 in ((20, 10), (200, 10)):
        model = DagmaMLP(dims=[d, m1, 1], bias=True, dtype=torch.double)
        w = mlp_fc1(d, m1)
        with torch.no_grad():
            model.fc1.weight.copy_(torch.from_numpy(w))
        pick = np.random.default_rng(5).choice(w.size, size=min(w.size, 4000), replace=False)
        out[f"pick_d{d}"] = pick
        for s in (1.0, 0.8):
            model.zero_grad()
            h = model.h_func(s)
            h.backward()
            g = model.fc1.weight.grad.detach().numpy().copy()
            out[f"h_d{d}_s{s}"] = np.array(h.item())
            out[f"gradpick_d{d}_s{s}"] = g.reshape(-1)[pick]
            out[f"gradnorm_d{d}_s{s}"] = np.array(np.linalg.norm(g))
    np.savez_compressed(os.path.join(HERE, "mlp_h.npz"), **out)


def main():
    with threadpool_limits(limits=1):
        X20, X100, Xl = gen_data()
        gen_blocks(X20, Xl)
        gen_traj(X20, "d20", [1, 10, 100, 1000, 10000])
        gen_traj(X100, "d100", [1, 10, 100, 1000])
        gen_traj(Xl, "logistic_d20", [1, 10, 100, 1000], loss="logistic", lambda1=0.05)
        gen_branches(X20)
        gen_fit(X20)
        gen_fit_envelope(X20)
        gen_fit_f32(X20)
        gen_fit_f32_envelope(X20)
        gen_fit_f32_default(X20)
        gen_trek()
        gen_tcc(X20)
        gen_mlp()
        gen_mlp_traj(X20)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # regenerate selected fixtures: make_golden.py gen_tcc ...
        with threadpool_limits(limits=1):
            X20 = np.load(os.path.join(HERE, "data_d20_n1000_seed0.npz"))["X"]
            for name in sys.argv[1:]:
                fn = globals()[name]
                fn(X20) if name in ("gen_tcc", "gen_mlp_traj", "gen_fit_f32", "gen_fit_f32_envelope",
                                             "gen_fit_f32_default") else fn()  # e.g. gen_traj_logistic_d100
    else:
        main()
