"""Python handle over the C ABI: one `HipSolver` per (fit, device).

`HipSolver.minimize` is the single-process hot path (the whole inner loop runs
on the GPU from replayed hipGraphs).  `run_allreduce_minimize` is the
multi-rank data-parallel loop: every step the GPU computes this rank's score
partial Z_k = X_k^T(...), the caller's all-reduce sums it over ranks
(torch.distributed -> RCCL over xGMI), and the GPU finishes the step.
"""
from __future__ import annotations

import ctypes as C
from collections import namedtuple
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, dptr

__all__ = ["HipSolver", "HipGroup", "MinimizeResult", "CheckpointRecord", "run_allreduce_minimize",
           "device_count", "colsum_dev", "center_dev", "gram", "row_range"]


CheckpointRecord = namedtuple("CheckpointRecord", [f for f, _ in _lib.MidagmaCkpt._fields_])


@dataclass
class MinimizeResult:
    iters: int
    success: bool
    status: int
    halvings: int
    early_stop: bool
    lr_final: float
    slots: int
    obj_last: float
    score_last: float
    h_last: float
    checkpoints: list = field(default_factory=list)

    @classmethod
    def from_c(cls, r: _lib.MidagmaResult, ckpts=()):
        return cls(iters=int(r.iters), success=r.status != _lib.ST_FAILED, status=int(r.status),
                   halvings=int(r.halvings), early_stop=bool(r.early_stop), lr_final=float(r.lr_final),
                   slots=int(r.slots), obj_last=float(r.obj_last), score_last=float(r.score_last),
                   h_last=float(r.h_last), checkpoints=list(ckpts))


def device_count() -> int:
    n = C.c_int(0)
    check(_lib.lib().midagma_device_count(C.byref(n)), None, "device_count")
    return int(n.value)


def _as_f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def is_device_tensor(X) -> bool:
    """True for a torch CUDA (HIP) tensor."""
    return hasattr(X, "data_ptr") and getattr(getattr(X, "device", None), "type", None) == "cuda"


def _rows(X):
    """(n, d, ld) of a row-major float64 matrix (host ndarray or device tensor)."""
    if hasattr(X, "data_ptr"):
        import torch
        if X.dtype != torch.float64 or X.dim() != 2 or X.stride(1) != 1:
            raise ValueError("X must be a 2-d float64 tensor with unit column stride")
        return int(X.shape[0]), int(X.shape[1]), int(X.stride(0))
    if X.dtype != np.float64 or X.ndim != 2 or X.strides[1] != 8:
        raise ValueError("X must be a 2-d float64 array with unit column stride")
    return int(X.shape[0]), int(X.shape[1]), int(X.strides[0] // 8)


def _cur_stream(dev):
    import torch
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def colsum_dev(X):
    """Column sums of a device X (fixed order; `X.mean(axis=0)` of linear.py:411 is this / n),
    on torch's current stream.  Returns a float64 device tensor of length d."""
    import torch
    n, d, ld = _rows(X)
    out = torch.empty(d, dtype=torch.float64, device=X.device)
    with torch.cuda.device(X.device):  # (the library's scratch on X's device, not the current one)
        check(_lib.lib().midagma_colsum_dev(C.c_void_p(X.data_ptr()), n, d, ld, C.c_void_p(out.data_ptr()),
                                            _cur_stream(X.device)), None, "colsum_dev")
    return out


def center_dev(X, colsum, nrows: float):
    """X -= colsum / nrows in place on the device (the l2 centring, linear.py:411)."""
    import torch
    n, d, ld = _rows(X)
    assert colsum.numel() == d and colsum.device == X.device
    with torch.cuda.device(X.device):
        check(_lib.lib().midagma_center_dev(C.c_void_p(X.data_ptr()), n, d, ld, C.c_void_p(colsum.data_ptr()),
                                            float(nrows), _cur_stream(X.device)), None, "center_dev")


def gram(X, device: int | None = None):
    """G = X^T X (linear.py:428 before the division) on the GPU, for X on the device or on the
    host (streamed through the device in row chunks).  Returns a d x d float64 device tensor."""
    import torch
    n, d, ld = _rows(X)
    on_dev = is_device_tensor(X)
    dev = X.device if on_dev else torch.device("cuda", 0 if device is None else device)
    G = torch.empty((d, d), dtype=torch.float64, device=dev)
    src = C.c_void_p(X.data_ptr()) if on_dev else X.ctypes.data_as(C.c_void_p)
    with torch.cuda.device(dev):
        check(_lib.lib().midagma_gram(src, n, d, ld, 1 if on_dev else 0, C.c_void_p(G.data_ptr()), d,
                                      _cur_stream(dev)), None, "gram")
    return G


class HipSolver:
    """Owns device buffers for one d and one score mode on one GPU."""

    def __init__(self, d: int, loss: str = "l2", mode: str = "cov", device: int = 0, stream: int | None = None,
                 _handle=None):
        self.L = _lib.lib()
        self.d = int(d)
        self.loss = loss
        self.mode = mode
        lt = {"l2": _lib.LOSS_L2, "logistic": _lib.LOSS_LOGISTIC}[loss]
        md = {"cov": _lib.MODE_COV, "data": _lib.MODE_DATA}[mode]
        # _handle: a solver owned by something else (a HipGroup's member); never destroyed here
        self._owned = _handle is None
        if _handle is None:
            h = C.c_void_p()
            check(self.L.midagma_create(C.byref(h), lt, md, self.d, int(device), stream), None, "midagma_create")
        else:
            h = C.c_void_p(_handle)
        self.h = h
        self.device = device
        self.D = int(self.L.midagma_padded_dim(self.h))

    def close(self):
        if getattr(self, "h", None):
            if self._owned:
                self.L.midagma_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return int(self.L.midagma_stream(self.h) or 0)

    # -- data -----------------------------------------------------------------
    def set_cov(self, cov: np.ndarray):
        cov = _as_f64(cov)
        check(self.L.midagma_set_cov(self.h, dptr(cov), cov.shape[1]), self.h, "set_cov")

    def set_w_float32(self, on: bool):
        """W's dtype in the reference's arithmetic for the next minimize (ABI 8): True emulates
        numpy's float32 operations on a float32 W (linear.py:29, 226, 244, 248, 275)."""
        check(self.L.midagma_set_w_float32(self.h, 1 if on else 0), self.h, "set_w_float32")

    def set_masks(self, mask_inc: np.ndarray | None, mask_exc: np.ndarray | None):
        mi = None if mask_inc is None else _as_f64(mask_inc)
        me = None if mask_exc is None else _as_f64(mask_exc)
        check(self.L.midagma_set_masks(self.h, dptr(mi), dptr(me)), self.h, "set_masks")

    TREK_SEQ = {"exp": 0, "inv": 1, "log": 2, "binom": 3}
    TREK_AGG = {"mean": 0, "sum": 1, "max": 2, "lse": 3}
    TREK_MODE = {"off": 0, "log": 1, "opt": 2}

    def set_trek(self, pairs, seq: str = "exp", *, agg: str = "mean", mode: str = "opt", weight: float = 0.0,
                 eps_inv: float = 1e-8, K_log: int | None = None):
        """The PST trek regularizer (notreks.pst) inside the loop; mode 'off' or no pairs disables it."""
        P = np.ascontiguousarray(np.asarray(pairs, dtype=np.int64).reshape(-1, 2)) if pairs is not None \
            else np.zeros((0, 2), dtype=np.int64)
        seq, agg, mode = seq.lower().strip(), agg.lower().strip(), mode.lower().strip()
        if seq not in self.TREK_SEQ or agg not in self.TREK_AGG or mode not in self.TREK_MODE:
            raise ValueError(f"unsupported PST configuration seq={seq!r} agg={agg!r} mode={mode!r}")
        K = 2 * self.d if K_log is None else int(K_log)
        check(self.L.midagma_set_trek(self.h, self.TREK_SEQ[seq], self.TREK_AGG[agg], self.TREK_MODE[mode],
                                      float(weight), float(eps_inv), K, P.ctypes.data_as(C.POINTER(C.c_int64)),
                                      int(P.shape[0])), self.h, "set_trek")

    def set_trek_tcc(self, pairs, *, mode: str = "opt", weight: float = 0.0, w: float = 1.0, eps: float = 1e-12):
        """The TCC trek regularizer as the reference's loop runs it (trek_value_grad -> spectral,
        'approx_trek_graph'); mode 'off' or no pairs disables it."""
        P = np.ascontiguousarray(np.asarray(pairs, dtype=np.int64).reshape(-1, 2)) if pairs is not None \
            else np.zeros((0, 2), dtype=np.int64)
        mode = mode.lower().strip()
        if mode not in self.TREK_MODE:
            raise ValueError(f"unsupported TCC mode {mode!r}")
        check(self.L.midagma_set_trek_tcc(self.h, self.TREK_MODE[mode], float(weight), float(w), float(eps),
                                          P.ctypes.data_as(C.POINTER(C.c_int64)), int(P.shape[0])), self.h,
              "set_trek_tcc")

    def trek_value(self, W: np.ndarray, grad: bool = True):
        """notreks.trek_value_grad(W, tr) for the configured regularizer: (value, grad or None)."""
        W = _as_f64(W)
        v = C.c_double()
        G = np.empty((self.d, self.d)) if grad else None
        check(self.L.midagma_trek(self.h, dptr(W), C.byref(v), dptr(G)), self.h, "trek")
        return float(v.value), G

    def set_data(self, X, n_global: int | None = None):
        """X: host ndarray (n_local x d) or a torch CUDA tensor (copied)."""
        if hasattr(X, "data_ptr"):
            X = X.contiguous()
            n_local = X.shape[0]
            check(self.L.midagma_set_data(self.h, C.c_void_p(X.data_ptr()), n_local, int(n_global or n_local), 1),
                  self.h, "set_data")
            self._keep = X
        else:
            X = _as_f64(X)
            n_local = X.shape[0]
            check(self.L.midagma_set_data(self.h, X.ctypes.data_as(C.c_void_p), n_local,
                                          int(n_global or n_local), 0), self.h, "set_data")

    def debug_sig_split(self, mode: int | None = None) -> int:
        """Test hook (not part of the public header): the logistic sigmoid GEMM's form for the
        next set_data (None: leave it; 0: the size rule, 1: the one-pass kernel, 2: the serial K
        split wherever the shape allows).  Returns the form the current data uses (1 or 2)."""
        fn = self.L.midagma_debug_sig_split
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
        cur = fn(self.h, -1)
        if mode is not None and fn(self.h, int(mode)) < 0:
            raise ValueError(f"debug_sig_split: bad mode {mode!r}")
        return int(cur)

    def debug_spoil_warm(self):
        """Test hook: zero the blocked inverse's stored warm starts, so the next fast slot hands
        back (ST_NEED_GJ) from inside its forked inverse."""
        fn = self.L.midagma_debug_spoil_warm
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p]
        check(fn(self.h), self.h, "debug_spoil_warm")

    def debug_tcc_fast_steps(self, steps: int | None = None) -> int:
        """Test hook: the Noda steps a fast cov slot's TCC chain runs before handing the slot back
        (0: the whole gated chain on every slot; None: leave it).  Returns the previous value."""
        fn = self.L.midagma_debug_tcc_fast_steps
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
        return int(fn(self.h, -1 if steps is None else int(steps)))

    def debug_tcc_fix(self, on=None) -> int:
        """Test hook: the TCC fixed-shift stage before Noda (True/False; None leaves it). Returns
        the old setting."""
        fn = self.L.midagma_debug_tcc_fix
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
        return int(fn(self.h, -1 if on is None else int(bool(on))))

    def debug_tcc_fastblk(self, on=None) -> int:
        """Test hook: the TCC fixed-stage inverse's fast blocks (D2 >= 2048) for the next set_trek_tcc
        (True/False; None leaves it). Returns the old setting."""
        fn = self.L.midagma_debug_tcc_fastblk
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
        return int(fn(self.h, -1 if on is None else int(bool(on))))

    def debug_at_fold(self, on=None) -> int:
        """Test hook: build_at folded into the previous slot's update (True/False; None leaves it).
        Returns the old setting (0/1), or -1 when the fold cannot apply to this solver."""
        fn = self.L.midagma_debug_at_fold
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
        return int(fn(self.h, -1 if on is None else int(bool(on))))

    def debug_handbacks(self) -> int:
        """Test hook: the hand-backs the slot scheduler has re-run on the pivoted path so far."""
        fn = self.L.midagma_debug_handbacks
        fn.restype, fn.argtypes = C.c_int64, [C.c_void_p]
        return int(fn(self.h))

    # fit()'s device data preparation (linear.py:406-428; the CPU test doubles override these)
    def colsum(self, X):
        return colsum_dev(X)

    def center(self, X, colsum, nrows: float):
        center_dev(X, colsum, nrows)

    def gram(self, X):
        return gram(X, self.device)

    def set_cov_gram(self, G, n: float):
        """cov = G / n on the device (G: the (all-reduced) d x d Gram matrix, a device tensor)."""
        import torch
        assert G.shape == (self.d, self.d) and G.is_contiguous()
        torch.cuda.current_stream(G.device).synchronize()
        check(self.L.midagma_set_cov_dev(self.h, C.c_void_p(G.data_ptr()), self.d, float(n)), self.h, "set_cov_dev")

    def data_gram(self):
        check(self.L.midagma_data_gram(self.h), self.h, "data_gram")

    def cov_from_zbuf(self, n: float):
        check(self.L.midagma_cov_from_zbuf(self.h, float(n)), self.h, "cov_from_zbuf")

    def get_cov(self) -> np.ndarray:
        out = np.empty((self.d, self.d))
        check(self.L.midagma_get_cov(self.h, dptr(out), self.d), self.h, "get_cov")
        return out

    def torch_zbuf(self):
        """A torch CUDA tensor bound as this solver's score-partial buffer, and a context that
        makes the solver's stream torch's current one: `with ctx: dist.all_reduce(zt)` sums the
        partial over ranks in stream order with the slot kernels (RCCL on the solver stream)."""
        import torch
        dev = torch.device("cuda", self.device)
        zt = torch.zeros(self.zbuf_len, dtype=torch.float64, device=dev)
        self.bind_zbuf(zt.data_ptr(), zt.numel())
        ext = torch.cuda.ExternalStream(self.stream, device=dev)
        return zt, (lambda: torch.cuda.stream(ext))

    def attach_comm(self, group=None):
        """Join an in-library RCCL communicator over `group` (torch.distributed; ABI 7): rank 0's
        ncclUniqueId is broadcast over the group, then every captured slot all-reduces the score
        partial itself, and minimize / run_slots drive the multi-rank loop from the device."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            check(self.L.midagma_comm_unique_id(C.c_void_p(uid.data_ptr()), 128), None, "comm_unique_id")
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if dist.get_backend(group) == "nccl":
            t = uid.to(torch.device("cuda", self.device))
            dist.broadcast(t, src=src, group=group)
            uid = t.cpu()
        else:
            dist.broadcast(uid, src=src, group=group)
        check(self.L.midagma_comm_init(self.h, C.c_void_p(uid.data_ptr()), 128, world, rank), self.h, "comm_init")

    def comm_allreduce_zbuf(self):
        check(self.L.midagma_comm_allreduce_zbuf(self.h), self.h, "comm_allreduce_zbuf")

    @property
    def comm_ranks(self) -> int:
        return int(self.L.midagma_comm_ranks(self.h))

    @property
    def zbuf_len(self) -> int:
        return int(self.L.midagma_zbuf_len(self.h))

    def bind_zbuf(self, ptr: int | None, length: int):
        check(self.L.midagma_bind_zbuf(self.h, C.c_void_p(ptr) if ptr else None, int(length)), self.h, "bind_zbuf")

    # -- the inner loop ---------------------------------------------------------
    def minimize(self, W: np.ndarray, mu: float, max_iter: int, s: float, lr: float, tol: float = 1e-6,
                 beta_1: float = 0.99, beta_2: float = 0.999, lambda1: float = 0.03,
                 checkpoint: int = 1000, want_checkpoints: bool = False):
        """Runs linear.py:165-333 on the GPU.  W (d x d float64) is updated in place."""
        assert W.shape == (self.d, self.d) and W.dtype == np.float64 and W.flags.c_contiguous
        res = _lib.MidagmaResult()
        check(self.L.midagma_minimize(self.h, dptr(W), float(mu), int(max_iter), float(s), float(lr), float(tol),
                                      float(beta_1), float(beta_2), float(lambda1), int(checkpoint),
                                      C.byref(res)), self.h, "minimize")
        return MinimizeResult.from_c(res, self.checkpoints() if want_checkpoints else ())

    def begin(self, W, mu, max_iter, s, lr, tol=1e-6, beta_1=0.99, beta_2=0.999, lambda1=0.03, checkpoint=1000):
        W = _as_f64(W)
        check(self.L.midagma_begin(self.h, dptr(W), float(mu), int(max_iter), float(s), float(lr), float(tol),
                                   float(beta_1), float(beta_2), float(lambda1), int(checkpoint)), self.h, "begin")

    def run_slots(self, n: int):
        check(self.L.midagma_run_slots(self.h, int(n)), self.h, "run_slots")

    def sync(self):
        check(self.L.midagma_sync(self.h), self.h, "sync")

    def profile_parts(self, reps: int = 10) -> dict:
        """Average device ms per launch group, measured with hipEvents on the solver stream."""
        out = np.zeros(8)
        check(self.L.midagma_profile_parts(self.h, int(reps), dptr(out)), self.h, "profile_parts")
        keys = ["build_at", "gj_inverse", "score", "slot", "gemm_xw", "gemm_xty", "inverse_fast", "slot_fast"]
        return {k: float(out[i]) for i, k in enumerate(keys)}

    def step_partial(self):
        check(self.L.midagma_step_partial(self.h), self.h, "step_partial")

    def step_finish(self):
        check(self.L.midagma_step_finish(self.h), self.h, "step_finish")

    def poll(self) -> _lib.MidagmaResult:
        r = _lib.MidagmaResult()
        check(self.L.midagma_poll(self.h, C.byref(r)), self.h, "poll")
        return r

    def end(self, W: np.ndarray) -> MinimizeResult:
        r = _lib.MidagmaResult()
        check(self.L.midagma_end(self.h, dptr(W), C.byref(r)), self.h, "end")
        return MinimizeResult.from_c(r)

    def checkpoints(self):
        """Checkpoint records of the last minimize call (`CheckpointRecord`: tuple-indexable
        (iter, obj, score, h, lr, l1, ...) and attribute access)."""
        cap = 1 << 16
        buf = (_lib.MidagmaCkpt * cap)()
        n = self.L.midagma_checkpoints(self.h, buf, cap)
        check(n, self.h, "checkpoints")
        return [CheckpointRecord(*(int(c.iter) if f == "iter" else float(getattr(c, f))
                                   for f in CheckpointRecord._fields)) for c in buf[:n]]

    # -- helpers of the reference API ----------------------------------------------
    def h_value(self, W: np.ndarray, s: float = 1.0, grad: bool = True):
        W = _as_f64(W)
        h = C.c_double()
        G = np.empty((self.d, self.d)) if grad else None
        check(self.L.midagma_h(self.h, dptr(W), float(s), C.byref(h), dptr(G)), self.h, "h")
        return float(h.value), G

    def score_value(self, W: np.ndarray):
        W = _as_f64(W)
        loss = C.c_double()
        G = np.empty((self.d, self.d))
        check(self.L.midagma_score(self.h, dptr(W), C.byref(loss), dptr(G)), self.h, "score")
        return float(loss.value), G

    def score_partial(self, W: np.ndarray):
        W = _as_f64(W)
        check(self.L.midagma_score_partial(self.h, dptr(W)), self.h, "score_partial")

    def score_finish(self):
        loss = C.c_double()
        G = np.empty((self.d, self.d))
        check(self.L.midagma_score_finish(self.h, C.byref(loss), dptr(G)), self.h, "score_finish")
        return float(loss.value), G


def row_range(n: int, parts: int, k: int):
    """Rows [lo, hi) of part k of the even split of n rows (the first n % parts parts take one
    row more): the data-mode shard of rank / group member k."""
    base, extra = divmod(int(n), int(parts))
    lo = k * base + min(k, extra)
    return lo, lo + base + (1 if k < extra else 0)


class HipGroup:
    """Data mode on several devices from ONE process (ABI 11, `midagma_group_*`): member k is a
    data-mode `HipSolver` on devices[k] holding row shard k of X, and every slot sums the members'
    score partials (the Python side stays single-process; the reference's own
    entry is the single-process `fit(X)`, linear.py:335-351).

    Distinct devices: an RCCL communicator per member from ncclCommInitAll, the all-reduce inside
    each member's replayed slot graphs, one library thread per device.  Repeated devices (every
    entry the same, e.g. [0, 0, 0, 0]) or emulate=True: an emulated group on that one device, whose
    slots are captured as one graph with a fixed-order device sum of the partials instead of RCCL
    (the sharding's arithmetic on a one-GPU box).

    It answers HipSolver's calls that `DagmaLinear` makes, broadcasting the loop's settings to
    every member and reading results from member 0."""

    is_group = True

    def __init__(self, d: int, loss: str = "l2", devices=(0,), emulate: bool | None = None):
        self.L = _lib.lib()
        self.d, self.loss, self.mode = int(d), loss, "data"
        devices = [int(x) for x in devices]
        if not devices:
            raise ValueError("devices must name at least one device")
        if emulate is None:
            emulate = len(set(devices)) < len(devices)
        lt = {"l2": _lib.LOSS_L2, "logistic": _lib.LOSS_LOGISTIC}[loss]
        arr = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(self.L.midagma_group_create(C.byref(h), lt, self.d, arr, len(devices),
                                          _lib.GROUP_EMULATE if emulate else 0), None, "group_create", group=True)
        self.h = h
        self.devices = devices
        self.device = devices[0]
        self.emulated = bool(self.L.midagma_group_emulated(h))
        self.members = [HipSolver(self.d, loss, "data", device=dv, _handle=self.L.midagma_group_member(h, k))
                        for k, dv in enumerate(devices)]
        self.D = self.members[0].D

    def _check(self, rc, what):
        return check(rc, self.h, what, group=True)

    def close(self):
        if getattr(self, "h", None):
            for m in self.members:
                m.close()
            self.L.midagma_group_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def size(self) -> int:
        return len(self.members)

    @property
    def comm_ranks(self) -> int:
        return 0 if self.emulated else len(self.members)

    # -- data -----------------------------------------------------------------------
    def set_data(self, X, n_global: int | None = None):
        """X: the whole host ndarray or torch tensor (n x d, n_global ignored), split by rows over
        the members (`row_range`).  A tensor's shards are copied to each member's device."""
        n = int(X.shape[0])
        if n < self.size:
            raise ValueError(f"set_data: {n} rows for {self.size} members")
        if hasattr(X, "data_ptr"):
            import torch
            for k, m in enumerate(self.members):
                lo, hi = row_range(n, self.size, k)
                part = X[lo:hi].to(torch.device("cuda", m.device)).contiguous()
                m.set_data(part, n_global=n)
            return
        X = _as_f64(X)
        self._check(self.L.midagma_group_set_data(self.h, X.ctypes.data_as(_lib._dp), n), "group_set_data")

    def set_cov(self, cov):
        for m in self.members:
            m.set_cov(cov)

    # fit()'s device data preparation for a device X (on one device; the shards are copied out)
    def colsum(self, X):
        return colsum_dev(X)

    def center(self, X, colsum, nrows: float):
        center_dev(X, colsum, nrows)

    def set_w_float32(self, on: bool):
        for m in self.members:
            m.set_w_float32(on)

    def set_masks(self, mask_inc, mask_exc):
        for m in self.members:
            m.set_masks(mask_inc, mask_exc)

    def set_trek(self, *a, **k):
        for m in self.members:
            m.set_trek(*a, **k)

    def set_trek_tcc(self, *a, **k):
        for m in self.members:
            m.set_trek_tcc(*a, **k)

    def allreduce_zbuf(self):
        """Every member's score buffer <- the sum over the members (RCCL, or the emulated sum)."""
        self._check(self.L.midagma_group_allreduce_zbuf(self.h), "group_allreduce_zbuf")

    comm_allreduce_zbuf = allreduce_zbuf

    def gram_cov(self, n: float) -> np.ndarray:
        """cov = (sum_k X_k^T X_k) / n (linear.py:428) from the members' device Gram matrices."""
        for m in self.members:
            m.data_gram()
        self.allreduce_zbuf()
        for m in self.members:
            m.cov_from_zbuf(float(n))
        return self.members[0].get_cov()

    def get_cov(self) -> np.ndarray:
        return self.members[0].get_cov()

    # -- the loop -------------------------------------------------------------------
    def minimize(self, W: np.ndarray, mu: float, max_iter: int, s: float, lr: float, tol: float = 1e-6,
                 beta_1: float = 0.99, beta_2: float = 0.999, lambda1: float = 0.03,
                 checkpoint: int = 1000, want_checkpoints: bool = False):
        """linear.py:165-333 over the group; W (d x d float64) updated in place."""
        assert W.shape == (self.d, self.d) and W.dtype == np.float64 and W.flags.c_contiguous
        res = _lib.MidagmaResult()
        self._check(self.L.midagma_group_minimize(self.h, dptr(W), float(mu), int(max_iter), float(s), float(lr),
                                                  float(tol), float(beta_1), float(beta_2), float(lambda1),
                                                  int(checkpoint), C.byref(res)), "group_minimize")
        return MinimizeResult.from_c(res, self.checkpoints() if want_checkpoints else ())

    def checkpoints(self):
        return self.members[0].checkpoints()

    def h_value(self, W, s: float = 1.0, grad: bool = True):
        return self.members[0].h_value(W, s, grad)

    def trek_value(self, W, grad: bool = True):
        return self.members[0].trek_value(W, grad)

    def score_partial(self, W):
        for m in self.members:
            m.score_partial(W)

    def score_finish(self):
        return self.members[0].score_finish()

    def score(self, W):
        """_score in data mode (linear.py:70-94): every member's partial, summed, finished."""
        self.score_partial(W)
        self.allreduce_zbuf()
        return self.score_finish()


def run_allreduce_minimize(backend, W, mu, max_iter, s, lr, tol=1e-6, beta_1=0.99, beta_2=0.999,
                           lambda1=0.03, checkpoint=1000, allreduce=None, batch: int = 32, agree=None):
    """Data-parallel inner loop over ranks.

    ``backend`` exposes begin/step_partial/step_finish/poll/end (HipSolver, or a
    test double); ``allreduce()`` sums the backend's score partial over ranks
    in place.  Termination is decided on the device by the controller kernel;
    the host polls every ``batch`` steps, extra steps after termination are
    no-ops, so every rank runs the same number of all-reduces.

    The replicas decide identically only while the all-reduce hands every rank the
    same bits (a ring all-reduce does; ``NCCL_ALGO=Ring`` pins it).  ``agree(status,
    iters)``, called at every poll, compares the ranks' states with one small
    collective and raises on a mismatch, so a divergent replica fails loudly instead
    of leaving the other ranks waiting in an all-reduce it no longer issues.
    """
    backend.begin(W, mu, max_iter, s, lr, tol, beta_1, beta_2, lambda1, checkpoint)
    slots = 0
    cap = int(max_iter) + int(max_iter) // max(int(checkpoint), 1) + 512
    while True:
        last = backend.poll()
        if agree is not None:
            agree(int(last.status), int(last.iters))
        if last.status != _lib.ST_RUNNING:
            break
        if slots > cap:
            raise _lib.HipSolverError("allreduce_minimize: slot budget exceeded")
        nb = max(1, min(batch, int(max_iter) - int(last.iters) + 2))
        for _ in range(nb):
            backend.step_partial()
            if allreduce is not None:
                allreduce()
            backend.step_finish()
        slots += nb
    return backend.end(W)
