"""`DagmaLinear` with the reference's API, backed by the MI355X HIP inner solver.

Drop-in for `dagma.linear.DagmaLinear` (fbleile/midagma, src/dagma/linear.py):
the constructor, `fit()` (linear.py:335-462) and the path-following outer loop
stay in Python exactly as the reference has them; `minimize()`
(linear.py:165-333), `_h` (97-116) and `_score` (70-94) run on the GPU through
the C ABI.  Extra keyword-only constructor arguments:

* ``score_mode``  'cov' (default for l2: cov = X^T X / n precomputed, as the
  reference does at linear.py:428) or 'data' (X row-sharded on the GPU(s),
  score gradient X^T(...) every step; required for 'logistic').
* ``device``      HIP device ordinal (default: LOCAL_RANK or 0).
* ``process_group``  a torch.distributed group: in data mode each rank keeps
  its row shard of X and the per-step score partial is all-reduced over it.
* ``force_allreduce``  run the all-reduce path (torch-owned score buffer,
  `dist.all_reduce` on the solver stream) even on one rank (tests, rehearsals).
* ``comm``  data mode over ranks: 'library' (the solver's own RCCL communicator: the score
  all-reduce is captured in the slot graphs, the loop runs from the device; the default under an
  'nccl' process group), 'host' (a `dist.all_reduce` between `step_partial` and `step_finish`
  every step; the default otherwise, e.g. gloo) or None (the default for the backend).
* ``solver_factory``  the backend class (default `HipSolver`; tests pass a CPU double).
* ``devices``  data mode on several devices from this ONE process (ABI 11, `HipGroup`): X is
  row-sharded over the listed devices and every step sums the shards' score partials, RCCL
  between distinct devices (ncclCommInitAll, one library thread per device), a fixed-order
  device sum when every entry names the same device (an emulated group: the sharded arithmetic
  on one GPU).  No launcher and no process group: `DagmaLinear('l2', devices=[0, 1, 2, 3]).fit(X)`.
  Implies score_mode='data'.  ``group_factory`` replaces `HipGroup` (tests).

`fit(X, ..., n_global=N)` (keyword-only extra): X is this rank's row shard of an
N-row data matrix.  Each rank then touches only its own rows: l2 centring uses
the all-reduced column sums (linear.py:411), and cov = X^T X / n (linear.py:428)
is the all-reduced sum of the ranks' device Gram matrices X_k^T X_k.

Trek regularizers (`trek_reg`, linear.py:251-258): the PST family of
`notreks.PSTRegularizer` (seq exp / inv / log / binom, agg mean / sum / max / lse,
modes 'opt' and 'log') runs on the GPU inside the loop (csrc/trek.hip), and so does
`notreks.TCCRegularizer` (csrc/tcc.hip): the Perron pair of the 2d x 2d block matrix,
which the reference takes from numpy `eig` every step, comes from Noda's iteration on
the Gauss-Jordan M-matrix inverse.
"""
from __future__ import annotations

import logging
import os
import time
import typing

import numpy as np

from .slog import LogConfig, StructuredLogger, build_default_logger, checkpoint_row
from ._lib import HipSolverError
from .solver import HipSolver, is_device_tensor, run_allreduce_minimize

__all__ = ["DagmaLinear"]


class _NullBar:
    def update(self, n=1):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _progress(total):
    try:
        from tqdm.auto import tqdm
        return tqdm(total=total)
    except Exception:  # pragma: no cover
        return _NullBar()


class DagmaLinear:
    """DAGMA for linear SEMs: the reference's interface, the GPU inner loop."""

    def __init__(self, loss_type: str, verbose: bool = False, dtype: type = np.float64, *,
                 trek_reg=None, logger=None, log_cfg=None, score_mode: str | None = None,
                 device: int | None = None, process_group=None, force_allreduce: bool = False,
                 comm: str | None = None, solver_factory=None, devices=None, group_factory=None) -> None:
        losses = ["l2", "logistic"]
        assert loss_type in losses, f"loss_type should be one of {losses}"
        # dtype (linear.py:29, 55): the type of Id, the exclusion mask and W_est (408, 220, 429).  The
        # reference keeps W in that type through its in-place Adam updates while cov, the
        # gradients and Adam come out float64.  With a float32 W the device loop emulates numpy's
        # float32 operations (W rounded after every update, s*Id - W*W, Id - W, M + 1e-16 and
        # 2 W o M^T in float32; csrc/common.h) around a float64 inverse rounded to float32, so a
        # float32 fit stays within the reference's own float32 perturbation envelope
        # (tests/test_gpu_parity.py::test_full_fit_float32_dtype, fit_f32_d20_envelope.npz)
        dtype = np.dtype(dtype).type
        if dtype not in (np.float32, np.float64):
            raise ValueError("dtype must be np.float64 or np.float32 (the solver computes in float64)")
        if trek_reg is not None and trek_reg.enabled() and str(trek_reg.name).lower().strip() not in ("pst", "tcc"):
            raise ValueError(f"Unknown trek regularizer: {trek_reg.name}. Has to be in ['pst', 'tcc']")
        self.loss_type = loss_type
        self.dtype = dtype
        self.vprint = print if verbose else (lambda *a, **k: None)
        self.trek_reg = trek_reg
        # structured logging as the reference (linear.py:64-67): one `minimize.checkpoint` row
        # per checkpoint, assembled from the device records after each minimize call
        self._logger = logger or build_default_logger(level=logging.INFO if verbose else logging.WARNING)
        self._log_cfg = log_cfg or LogConfig(enabled=verbose)
        self._slog = StructuredLogger(self._logger, self._log_cfg)
        if devices is not None:
            devices = [int(x) for x in devices]
            if not devices:
                raise ValueError("devices must name at least one device")
            if score_mode not in (None, "data"):
                raise ValueError("devices=[...] shards X over the devices: it needs score_mode='data'")
            if process_group is not None or force_allreduce or comm is not None:
                raise ValueError("devices=[...] drives the devices from this process: no process_group, "
                                 "force_allreduce or comm")
            score_mode = "data"
            device = devices[0]
        self.devices = devices
        self._group_factory = group_factory
        self.score_mode = score_mode or ("cov" if loss_type == "l2" else "data")
        if self.loss_type == "logistic" and self.score_mode != "data":
            raise ValueError("logistic loss needs score_mode='data' (the gradient depends on X every step)")
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = device
        self.process_group = process_group
        self.force_allreduce = bool(force_allreduce)
        if comm not in (None, "library", "host"):
            raise ValueError("comm must be 'library', 'host' or None")
        self.comm = comm
        self._inlib = False
        self._solver_factory = solver_factory or HipSolver
        self._solver: HipSolver | None = None
        self._allreduce = None
        self.minimize_log: list = []

    # ------------------------------------------------------------------ helpers
    def _world(self):
        # cov mode talks to the other ranks only while a sharded fit() prepares cov; a device group
        # is one process
        if self.devices is not None or (self.score_mode != "data" and not getattr(self, "_sharded", False)):
            return 1, 0
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                return dist.get_world_size(self.process_group), dist.get_rank(self.process_group)
        except Exception:  # pragma: no cover
            pass
        return 1, 0

    def _allreduce_host(self, v: np.ndarray) -> np.ndarray:
        """Sum a small host vector over the ranks of the process group (fit-time only)."""
        import torch
        import torch.distributed as dist
        on_gpu = dist.get_backend(self.process_group) == "nccl"
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        t = t.to(torch.device("cuda", self.device)) if on_gpu else t.clone()
        dist.all_reduce(t, group=self.process_group)
        return t.cpu().numpy()

    def _agree(self, status: int, iters: int) -> None:
        """Raise unless every rank polled the same (status, iters) (run_allreduce_minimize)."""
        v = np.array([status, iters, -status, -iters], dtype=np.float64)
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return
        import torch
        on_gpu = dist.get_backend(self.process_group) == "nccl"
        t = torch.from_numpy(v)
        t = t.to(torch.device("cuda", self.device)) if on_gpu else t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        m = t.cpu().numpy()
        if m[0] != -m[2] or m[1] != -m[3]:
            raise HipSolverError(f"data-parallel replicas diverged: (status, iters) ranges over ranks "
                                 f"[{-m[2]:.0f}, {m[0]:.0f}], [{-m[3]:.0f}, {m[1]:.0f}] (pin NCCL_ALGO=Ring)")

    def _allreduce_tensor(self, t):
        """Sum a fit-time tensor over the process group (a no-op on one rank)."""
        world, _ = self._world()
        if world > 1:
            import torch.distributed as dist
            dist.all_reduce(t, group=self.process_group)
        return t

    def _comm_kind(self) -> str:
        if self.comm is not None:
            return self.comm
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_backend(self.process_group) == "nccl":
                return "library"
        except Exception:  # pragma: no cover
            pass
        return "host"

    def _setup_solver(self, s=None, X_local=None, cov_on_device=False, gram_device=False):
        world, rank = self._world()
        if s is None:
            s = self._solver_factory(self.d, self.loss_type, self.score_mode, device=self.device)
        self._allreduce = None
        if self.score_mode == "data":
            if X_local is None:
                lo, hi = _row_range(self.n, world, rank)
                X_local = self.X[lo:hi]
            s.set_data(X_local if is_device_tensor(X_local) else np.ascontiguousarray(X_local), n_global=self.n)
            if getattr(s, "is_group", False):
                # a single-process device group: the members' sum inside the slots and in _score
                self._inlib = True
                if cov_on_device:
                    self.cov = s.gram_cov(float(self.n))
                else:
                    s.set_cov(self.cov)
                self._install_trek(s)
                self._solver = s
                return
            self._inlib = (world > 1 or self.force_allreduce) and self._comm_kind() == "library"
            if self._inlib:
                # the solver's own communicator: the score all-reduce inside the replayed slots
                s.attach_comm(self.process_group)
                if cov_on_device:
                    G = self._allreduce_tensor(s.gram(X_local))
                    s.set_cov_gram(G, float(self.n))
                    self.cov = s.get_cov()
                else:
                    s.set_cov(self.cov)
            elif world > 1 or self.force_allreduce:
                import torch.distributed as dist
                zt, on_stream = s.torch_zbuf()
                pg = self.process_group

                def _allreduce():
                    with on_stream():
                        dist.all_reduce(zt, group=pg)

                self._allreduce, self._zt = _allreduce, zt
            if self._inlib:
                pass
            elif cov_on_device:
                # cov = (sum_k X_k^T X_k) / n (linear.py:428) from the ranks' device Gram matrices
                s.data_gram()
                if self._allreduce is not None:
                    self._allreduce()
                s.cov_from_zbuf(float(self.n))
                self.cov = s.get_cov()
            else:
                s.set_cov(self.cov)
        elif gram_device:
            # cov = (sum_k X_k^T X_k) / n (linear.py:428): this rank's rows through the MFMA Gram,
            # one all-reduce of the d x d sum over the ranks of a sharded fit, then the loop runs
            # replicated with no per-step communication (cov is n-independent)
            G = self._allreduce_tensor(s.gram(X_local if X_local is not None else self.X))
            s.set_cov_gram(G, float(self.n))
            self.cov = s.get_cov()
        else:
            s.set_cov(self.cov)
        self._install_trek(s)
        self._solver = s

    def _install_trek(self, s):
        """The trek regularizer of linear.py:251-258 on the solver (every member of a group)."""
        tr = self.trek_reg
        if tr is not None and tr.enabled() and tr.cfg.get("I") is not None and len(tr.cfg["I"]) > 0:
            if str(tr.name).lower().strip() == "tcc":
                # trek_value_grad runs TCC with its defaults whatever the regularizer's
                # cycle_penalty / version / method (notreks.py:691-698): only w and eps reach it
                s.set_trek_tcc(tr.cfg["I"], mode=tr.mode, weight=tr.weight, w=tr.cfg.get("w", 1.0),
                               eps=tr.cfg.get("eps", 1e-12))
            else:
                kw = dict(tr.cfg.get("kwargs") or {})
                s.set_trek(tr.cfg["I"], tr.cfg.get("seq", "exp"), agg=kw.get("agg", "mean"), mode=tr.mode,
                           weight=tr.weight, eps_inv=kw.get("eps_inv", 1e-8), K_log=kw.get("K_log"))

    # ------------------------------------------------------- reference methods
    def _score(self, W: np.ndarray) -> typing.Tuple[float, np.ndarray]:
        """loss and gradient of the score (linear.py:70-94), on the GPU."""
        if self.score_mode == "cov":
            return self._solver.score_value(W)
        self._solver.score_partial(W)
        if self._allreduce is not None:
            self._allreduce()
        elif self._inlib:
            self._solver.comm_allreduce_zbuf()
        return self._solver.score_finish()

    def _h(self, W: np.ndarray, s: float = 1.0) -> typing.Tuple[float, np.ndarray]:
        """log-det acyclicity value and gradient (linear.py:97-116), on the GPU."""
        return self._solver.h_value(W, s, grad=True)

    def _func(self, W: np.ndarray, mu: float, s: float = 1.0):
        """objective at W (linear.py:118-135), with the trek term in 'opt' mode."""
        score, _ = self._score(W)
        h, _ = self._h(W, s)
        trek_val, _ = self._solver.trek_value(W, grad=False)
        obj = mu * (score + self.lambda1 * np.abs(W).sum()) + h
        tr = self.trek_reg
        if tr is not None and tr.enabled() and tr.mode == "opt":
            obj = obj + tr.weight * trek_val
        return obj, score, h, trek_val

    def _adam_update(self, grad: np.ndarray, iter: int, beta_1: float, beta_2: float) -> np.ndarray:
        """API-compatibility helper (linear.py:138-163).  Not used by `minimize`, whose
        Adam step is fused into the GPU update kernel."""
        self.opt_m = self.opt_m * beta_1 + (1 - beta_1) * grad
        self.opt_v = self.opt_v * beta_2 + (1 - beta_2) * (grad ** 2)
        m_hat = self.opt_m / (1 - beta_1 ** iter)
        v_hat = self.opt_v / (1 - beta_2 ** iter)
        return m_hat / (np.sqrt(v_hat) + 1e-8)

    def _masks(self, mu: float):
        """linear.py:217-222"""
        mask_inc = mask_exc = None
        if self.inc_c is not None:
            mask_inc = np.zeros((self.d, self.d))
            mask_inc[self.inc_r, self.inc_c] = -2 * mu * self.lambda1
        if self.exc_c is not None:
            mask_exc = np.ones((self.d, self.d), dtype=self.dtype)
            mask_exc[self.exc_r, self.exc_c] = 0.
        return mask_inc, mask_exc

    def minimize(self, W: np.ndarray, mu: float, max_iter: int, s: float, lr: float, tol: float = 1e-6,
                 beta_1: float = 0.99, beta_2: float = 0.999, pbar=None) -> typing.Tuple[np.ndarray, bool]:
        """Solves argmin_{W in W^s} mu*Q(W; X) + h(W) by Adam (linear.py:165-333), on the GPU."""
        t0 = time.time()
        self.vprint(f'\n\nMinimize with -- mu:{mu} -- lr: {lr} -- s: {s} -- l1: {self.lambda1} '
                    f'for {max_iter} max iterations')
        w_type = np.asarray(W).dtype.type
        if w_type not in (np.float32, np.float64):
            w_type = np.float64
        W = np.ascontiguousarray(W, dtype=np.float64)
        mask_inc, mask_exc = self._masks(mu)
        self._solver.set_masks(mask_inc, mask_exc)
        # a float32 W (dtype=np.float32, linear.py:429) is updated in float32 arithmetic, as numpy
        # updates the reference's float32 W in place (275); the inverse stays float64
        if hasattr(self._solver, "set_w_float32"):
            self._solver.set_w_float32(w_type is np.float32)
        logging_on = bool(self._log_cfg.enabled)
        if self.score_mode == "data" and self._allreduce is not None:
            res = run_allreduce_minimize(self._solver, W, mu, max_iter, s, lr, tol, beta_1, beta_2,
                                         self.lambda1, self.checkpoint, allreduce=self._allreduce,
                                         agree=self._agree)
            ckpts = self._solver.checkpoints() if logging_on else ()
        else:
            res = self._solver.minimize(W, mu, max_iter, s, lr, tol, beta_1, beta_2, self.lambda1,
                                        self.checkpoint, want_checkpoints=logging_on)
            ckpts = res.checkpoints
        if logging_on:  # linear.py:282-326 (elapsed: device clock from the first slot)
            stage = getattr(self, "_stage", 0)
            for rec in ckpts:
                self._slog.emit("minimize.checkpoint", checkpoint_row(rec, stage=stage, mu=mu, s=s,
                                                                      trek_reg=self.trek_reg))
        if res.halvings:
            self.vprint(f'Learning rate decreased {res.halvings} time(s) to lr: {res.lr_final}')
        if not res.success:
            self.vprint(f'W went out of domain for s={s} at iteration {res.iters + 1}')
        self.minimize_log.append(dict(mu=mu, s=s, lr=lr, max_iter=max_iter, iters=res.iters,
                                      success=res.success, early_stop=res.early_stop,
                                      halvings=res.halvings, seconds=time.time() - t0))
        if pbar is not None:  # the reference ticks once per iteration (linear.py:329, 332)
            pbar.update(int(max_iter) if res.early_stop else res.iters)
        # the reference updates W in place (linear.py:275): the result keeps W's floating type
        return (W.astype(w_type) if w_type is not np.float64 else W), res.success

    def fit(self, X: np.ndarray, lambda1: float = 0.03, w_threshold: float = 0.3, T: int = 5,
            mu_init: float = 1.0, mu_factor: float = 0.1,
            s: typing.Union[typing.List[float], float] = [1.0, .9, .8, .7, .6],
            warm_iter: int = 3e4, max_iter: int = 6e4, lr: float = 0.0003, checkpoint: int = 1000,
            beta_1: float = 0.99, beta_2: float = 0.999,
            exclude_edges: typing.Optional[typing.List[typing.Tuple[int, int]]] = None,
            include_edges: typing.Optional[typing.List[typing.Tuple[int, int]]] = None, *,
            n_global: int | None = None, gram: str = "auto") -> np.ndarray:
        """Runs DAGMA and returns the thresholded weighted adjacency (linear.py:335-462).

        Keyword-only extras:
        n_global: X is this rank's row shard of an n_global-row matrix.  In data mode the rank
            keeps its rows on its GPU; in cov mode (l2) the ranks' Gram matrices are all-reduced
            once and every rank runs the same n-independent loop (no per-step communication).
        gram: where cov = X^T X / n (linear.py:428) is formed in cov mode: 'host' (the
            reference's numpy product), 'device' (the GPU's MFMA Gram) or 'auto' (the device for
            a device X, a shard, or n d^2 >= 1e11 flop-pairs, e.g. n = 1e5 at d = 1000).
        X may be a float64 torch CUDA tensor (centred in place on the device)."""
        if gram not in ("auto", "host", "device"):
            raise ValueError("gram must be 'auto', 'host' or 'device'")
        t_start = time.perf_counter()
        sharded = n_global is not None
        # (preparation under try/finally: _world() must not keep seeing a shard after a failure)
        try:
            self._sharded = sharded
            world, rank = self._world()
            on_dev = is_device_tensor(X)
            self.X, self.lambda1, self.checkpoint = X, lambda1, checkpoint
            self.n, self.d = (int(n_global), int(X.shape[1])) if sharded else (int(X.shape[0]), int(X.shape[1]))
            self.Id = np.eye(self.d).astype(self.dtype)
            if on_dev and gram == "host":
                raise ValueError("gram='host' needs a host X")
            gram_device = self.score_mode == "cov" and (
                gram == "device" or (gram == "auto" and (on_dev or sharded or
                                                         float(X.shape[0]) * self.d * self.d >= 1e11)))
            if sharded and self.score_mode == "cov" and not gram_device:
                raise ValueError("fit(X_shard, n_global=...) in cov mode forms cov on the device (gram='device')")
            if self.devices is not None and sharded:
                raise ValueError("devices=[...] shards X itself: pass the whole X, not n_global")
            if self.devices is not None:
                from .solver import HipGroup
                solver = (self._group_factory or HipGroup)(self.d, self.loss_type, devices=self.devices)
            else:
                solver = self._solver_factory(self.d, self.loss_type, self.score_mode, device=self.device)
            if self.loss_type == 'l2':
                if on_dev:  # the centring on the device: column sums (all-reduced over shards), X -= mean
                    colsum = self._allreduce_tensor(solver.colsum(X)) if sharded else solver.colsum(X)
                    solver.center(X, colsum, float(self.n))
                elif sharded:  # the global column mean from the ranks' column sums
                    colsum = X.sum(axis=0)
                    if world > 1:
                        colsum = self._allreduce_host(colsum)
                    self.X -= (colsum / float(self.n))[None, :]
                else:
                    self.X -= X.mean(axis=0, keepdims=True)
            self.exc_r, self.exc_c = None, None
            self.inc_r, self.inc_c = None, None
            if exclude_edges is not None:
                if type(exclude_edges) is tuple and type(exclude_edges[0]) is tuple and \
                        np.all(np.array([len(e) for e in exclude_edges]) == 2):
                    self.exc_r, self.exc_c = zip(*exclude_edges)
                else:
                    ValueError("blacklist should be a tuple of edges, e.g., ((1,2), (2,3))")
            if include_edges is not None:
                if type(include_edges) is tuple and type(include_edges[0]) is tuple and \
                        np.all(np.array([len(e) for e in include_edges]) == 2):
                    self.inc_r, self.inc_c = zip(*include_edges)
                else:
                    ValueError("whitelist should be a tuple of edges, e.g., ((1,2), (2,3))")
            # data mode over several ranks (or a shard, or a device X): cov from the device Gram
            # matrices, no rank multiplies another rank's rows; one host X keeps the reference's product
            cov_on_device = self.score_mode == "data" and (sharded or world > 1 or on_dev)
            if self.devices is not None:
                # a device group: the members' Gram matrices summed (RCCL / the emulated sum) for a
                # device X, gram='device', or a large X (as cov mode's 'auto'); else the reference's
                # host product (linear.py:428)
                cov_on_device = on_dev or gram == "device" or (
                    gram == "auto" and float(X.shape[0]) * self.d * self.d >= 1e11)
            X_local = X if sharded else None
            if not cov_on_device and not gram_device:
                self.cov = X.T @ X / float(self.n)
            self.W_est = np.zeros((self.d, self.d)).astype(self.dtype)
            self._setup_solver(solver, X_local=X_local, cov_on_device=cov_on_device, gram_device=gram_device)
        finally:
            self._sharded = False  # the loop itself: replicated in cov mode, no collective
        t_prep = time.perf_counter()
        mu = mu_init
        if type(s) == list:
            if len(s) < T:
                self.vprint(f"Length of s is {len(s)}, using last value in s for iteration t >= {len(s)}")
                s = s + (T - len(s)) * [s[-1]]
        elif type(s) in [int, float]:
            s = T * [s]
        else:
            ValueError("s should be a list, int, or float.")
        with _progress((T - 1) * warm_iter + max_iter) as pbar:
            for i in range(int(T)):
                self.vprint(f'\nIteration -- {i+1}:')
                lr_adam, success = lr, False
                inner_iters = int(max_iter) if i == T - 1 else int(warm_iter)
                while success is False:
                    W_temp, success = self.minimize(self.W_est.copy(), mu, inner_iters, s[i], lr=lr_adam,
                                                    beta_1=beta_1, beta_2=beta_2, pbar=pbar)
                    if success is False:
                        self.vprint('Retrying with larger s')
                        lr_adam *= 0.5
                        s[i] += 0.1
                self.W_est = W_temp
                mu *= mu_factor
        t_loop = time.perf_counter()
        self.h_final, _ = self._h(self.W_est)
        self.score_final, _ = self._score(self.W_est)
        # wall-clock split of this fit (not in the reference): data preparation (centring, cov or
        # the data-mode upload), the path-following loop, and the final h / score
        self.fit_timing = dict(prep_s=t_prep - t_start, loop_s=t_loop - t_prep,
                               final_s=time.perf_counter() - t_loop, cov_on=("device" if (gram_device or cov_on_device)
                                                                              else "host"))
        self.W_est[np.abs(self.W_est) < w_threshold] = 0
        self._slog.close()
        return self.W_est


def _row_range(n: int, world: int, rank: int):
    """Even row split of X over ranks (first n % world ranks take one extra row)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)
