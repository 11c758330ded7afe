"""`DagmaMLP` / `DagmaNonlinear` whose log-det acyclicity term runs on the HIP GJ/log-det kernel.

Mirrors `dagma.nonlinear.DagmaMLP`, `DagmaNonlinear` (fbleile/midagma,
src/dagma/nonlinear.py:14-331) and `LocallyConnected` (src/dagma/locally_connected.py).
The MLP forward, the score and Adam stay PyTorch-ROCm on the GPU (SURVEY.md section 2,
row 4; BASELINE config 5); only ``h_func`` (nonlinear.py:68-86) is replaced:

    A = sum_m fc1_w[j, m, i]^2   (transposed: [i, j])
    h = -log|det(sI - A)| + d log s          forward  : HIP blocked Gauss-Jordan
    dh/dA = (sI - A)^{-T}                     backward : the inverse the forward produced

The C entry point (`midagma_logdet_inv_dev`) works on torch's device memory
and current HIP stream; it never synchronizes with the host.

For the [d, m1, 1] model (BASELINE config 5) the objective runs on fused HIP kernels
(csrc/mlp.hip): the fc1 terms (A and the |fc1| sum, one launch), the tail (sigmoid, the
width-1 LocallyConnected layer with its bias and the squared residual sum, two launches) and
the scalar objective (one launch), each with a fused backward, instead of PyTorch's ~40
elementwise, reduction and scalar kernels (MIDAGMA_NO_MLP_TAIL=1: the PyTorch expressions).
"""
from __future__ import annotations

import copy
import ctypes as C
import math
import os
import typing

import numpy as np
import torch
import torch.nn as nn

from . import _lib

__all__ = ["LocallyConnected", "DagmaMLP", "DagmaNonlinear", "logdet_h"]


class _LogdetH(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A: torch.Tensor, s: float):
        if not A.is_cuda or A.dtype != torch.float64:
            raise _lib.HipSolverError("logdet_h needs a float64 tensor on a ROCm device (no CPU fallback)")
        A = A.contiguous()
        d = A.shape[0]
        Mt = torch.empty_like(A)
        logdet = torch.empty(1, dtype=torch.float64, device=A.device)
        stream = torch.cuda.current_stream(A.device).cuda_stream
        L = _lib.lib()
        with torch.cuda.device(A.device):
            _lib.check(L.midagma_logdet_inv_dev(C.c_void_p(A.data_ptr()), d, d, float(s),
                                                C.c_void_p(logdet.data_ptr()), C.c_void_p(Mt.data_ptr()), d,
                                                C.c_void_p(stream) if stream else None),
                       None, "logdet_inv_dev")
        ctx.save_for_backward(Mt)
        return -logdet[0] + d * math.log(s)

    @staticmethod
    def backward(ctx, grad_out):
        (Mt,) = ctx.saved_tensors
        return grad_out * Mt, None


class _MLPTail(torch.autograd.Function):
    """sum((LocallyConnected(sigmoid(Z)) - X)^2) for a [d, m1, 1] DagmaMLP, forward and
    backward as fused HIP kernels (csrc/mlp.hip) on torch's stream."""

    @staticmethod
    def forward(ctx, Z: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, X: torch.Tensor, m1: int):
        Z, w2, b2, X = Z.contiguous(), w2.contiguous(), b2.contiguous(), X.contiguous()
        n, d = X.shape
        R = torch.empty_like(X)
        part = torch.empty(int(_lib.lib().midagma_mlp_tail_scratch(n, d, m1)), dtype=torch.float64, device=X.device)
        ssq = torch.empty((), dtype=torch.float64, device=X.device)
        stream = torch.cuda.current_stream(X.device).cuda_stream
        with torch.cuda.device(X.device):
            _lib.check(_lib.lib().midagma_mlp_tail_fwd(
                C.c_void_p(Z.data_ptr()), None, C.c_void_p(w2.data_ptr()), C.c_void_p(b2.data_ptr()),
                C.c_void_p(X.data_ptr()), n, d, m1, C.c_void_p(R.data_ptr()), C.c_void_p(part.data_ptr()),
                C.c_void_p(ssq.data_ptr()), C.c_void_p(stream) if stream else None), None, "mlp_tail_fwd")
        ctx.save_for_backward(Z, w2, R, part)
        ctx.m1 = m1
        ctx.b2_shape = b2.shape
        return ssq

    @staticmethod
    def backward(ctx, g):
        Z, w2, R, scratch = ctx.saved_tensors
        n, d = R.shape
        g = g.contiguous()
        dZ = torch.empty_like(Z)
        dw2 = torch.empty_like(w2)
        db2 = torch.empty(ctx.b2_shape, dtype=torch.float64, device=Z.device)
        stream = torch.cuda.current_stream(Z.device).cuda_stream
        with torch.cuda.device(Z.device):
            _lib.check(_lib.lib().midagma_mlp_tail_bwd(
                C.c_void_p(Z.data_ptr()), None, C.c_void_p(w2.data_ptr()), C.c_void_p(R.data_ptr()),
                C.c_void_p(g.data_ptr()), n, d, ctx.m1, C.c_void_p(dZ.data_ptr()), C.c_void_p(dw2.data_ptr()),
                C.c_void_p(db2.data_ptr()), None, C.c_void_p(scratch.data_ptr()),
                C.c_void_p(stream) if stream else None),
                None, "mlp_tail_bwd")
        return dZ, dw2, db2, None, None


def _vp(t):
    return C.c_void_p(t.data_ptr())


# fc1 and the tail forward / backward fused on the MFMA (midagma_mlp_fc1_tail_fwd,
# midagma_mlp_tail_bwd_lin: experiments build only, measured slower at config 5 beside the
# side-stream log-det).  True takes them where the loaded library has them and
# takes the model's d and m1; the product path runs fc1 as a library GEMM, the tail kernels and
# the split-K dZ^T X.
FUSED_TAIL = False
# split-K count of the weight gradient dZ^T X (a batched library GEMM whose slices the fc1 terms'
# backward sums per element)
LIN_SPLIT = 4


def _fused_parts(L, n, d, m1) -> int:
    """The fused forward's partial count (0: not taken), binding the experiment entries once."""
    if not FUSED_TAIL or not hasattr(L, "midagma_mlp_fused_parts"):
        return 0
    if not getattr(L, "_fused_bound", False):
        vp, i64, dd = C.c_void_p, C.c_int64, C.c_double
        for name, res, args in (
                ("midagma_mlp_fused_parts", i64, [i64, i64, i64]),
                ("midagma_mlp_fused_splits", i64, [i64]),
                ("midagma_mlp_fc1_tail_fwd", C.c_int, [vp, vp, vp, vp, vp, i64, i64, i64, vp, vp, vp, vp]),
                ("midagma_mlp_tail_bwd_lin", C.c_int, [vp, vp, vp, vp, vp, i64, vp, dd, dd, dd, i64, i64, i64, vp,
                                                       vp, vp, vp, vp, vp])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        L._fused_bound = True
    return int(L.midagma_mlp_fused_parts(n, d, m1))


def _tail_fwd(L, fused, X, W1, b1, w2, b2, n, d, m1, Z, R, part, st):
    if fused:
        _lib.check(L.midagma_mlp_fc1_tail_fwd(_vp(X), _vp(W1), _vp(b1), _vp(w2), _vp(b2), n, d, m1, _vp(Z), _vp(R),
                                              _vp(part), st), None, "mlp_fc1_tail_fwd")
    else:
        _lib.check(L.midagma_mlp_tail_fwd_part(_vp(Z), _vp(b1), _vp(w2), _vp(b2), _vp(X), n, d, m1, _vp(R),
                                               _vp(part), st), None, "mlp_tail_fwd_part")


class _MLPObjective(torch.autograd.Function):
    """(h, mu * (0.5 d log(1/n sum (model(X) - X)^2) + lambda1 |fc1|_1) + h) of a [d, m1, 1]
    DagmaMLP as one autograd node (nonlinear.py:68-86, 139-159, 198-204), so that no gradient is
    accumulated or reduced by PyTorch: fc1's pre-activation X W1^T without the bias (the tail
    kernels add b1), the fc1 terms and the log-det, the tail and the scalar objective forward;
    backward the objective, the tail (dZ with the bias gradient's column sums, dw2, db2), the
    weight gradient dZ^T X as a 4-way split-K batched GEMM whose chunks the fc1 terms' backward
    sums together with the log-det and L1 gradients."""

    @staticmethod
    def forward(ctx, X, W1, b1, w2, b2, d: int, m1: int, s: float, mu: float, lambda1: float,
                overlap: bool = False, ld=None, exact: bool = True, counter=None, step=None):
        L = _lib.lib()
        dev = X.device
        X, W1, b1, w2, b2 = X.contiguous(), W1.contiguous(), b1.contiguous(), w2.contiguous(), b2.contiguous()
        n = X.shape[0]
        stream = torch.cuda.current_stream(dev).cuda_stream
        st = C.c_void_p(stream) if stream else None
        f64 = dict(dtype=torch.float64, device=dev)
        npf = _fused_parts(L, n, d, m1)
        fused = npf > 0
        # fused: fc1's GEMM and the tail forward in one MFMA launch (midagma_mlp_fc1_tail_fwd), Z then
        # holds sigmoid(X W1^T + b1) (what the fused backward reads), else fc1's pre-activation X W1^T
        Z = torch.empty((n, d * m1), **f64) if fused else X @ W1.t()
        if step is not None and fused:
            raise _lib.HipSolverError("the one-launch step (_MlpStep) runs on the product tail, not the fused MFMA one")
        # step (_MlpStep): the fc1 terms of the current weights were left by the last step's closing
        # launch (midagma_mlp_step), which also takes this step's backward, Adam and next terms
        A = step.A if step is not None else torch.empty((d, d), **f64)
        l1part = step.l1part if step is not None else torch.empty(int(L.midagma_fc1_terms_parts(d)), **f64)
        Mt = torch.empty((d, d), **f64)
        h = torch.empty((), **f64)
        R = torch.empty_like(X)
        part = torch.empty(npf if fused else n, **f64)  # the tail's partials of the squared residual sum
        scratch = torch.empty(int(L.midagma_mlp_tail_scratch(n, d, m1)), **f64)
        obj = torch.empty((), **f64)
        ctr = _vp(counter) if counter is not None else None
        ctx.chain = None
        with torch.cuda.device(dev):
            if step is None:
                _lib.check(L.midagma_fc1_terms(_vp(W1), d, m1, _vp(A), _vp(l1part), st), None, "fc1_terms")
            if overlap:
                # The log-det chain (latency-bound) depends on fc1 only: it runs on a side stream
                # beside the tail forward and the backward up to the weight gradient, which never
                # read h or the objective's value; the side stream also forms the objective once the
                # tail's partials are ready, and backward joins before the fc1 terms' backward needs
                # (sI - A)^-T.  Only for callers that run backward right away
                # (DagmaNonlinear.minimize): the join is there.  Its parts are enqueued between the
                # main stream's launches (a replayed graph submits nodes in capture order, ~4 us
                # each: a branch captured whole ahead of the other holds the other back by its
                # whole submission time).
                main = torch.cuda.current_stream(dev)
                side = _side_stream(dev)
                ev_fc1 = torch.cuda.Event()
                ev_fc1.record(main)
                side.wait_event(ev_fc1)
                chain = _SideLogdet(L, side, A, d, float(s), h, Mt, ld=ld, exact=exact, ctr=ctr)
                chain.enqueue(1)
                _tail_fwd(L, fused, X, W1, b1, w2, b2, n, d, m1, Z, R, part, st)
                ev_tail = torch.cuda.Event()
                ev_tail.record(main)
                chain.enqueue(2)
                chain.objective = (ev_tail, part, l1part, float(mu), float(lambda1), 0.5 * d, 1 / n, obj, ctr)
                ctx.chain = chain
                ctx.keep = (A, l1part)  # read on the side stream: alive until the join
            else:
                if ld is not None:
                    ld.set_counter(None)  # (the objective below advances the counter)
                    ld.enqueue(A, d, float(s), h, Mt, stream, exact, -1)
                else:
                    _lib.check(L.midagma_logdet_h_dev(_vp(A), d, d, float(s), _vp(h), _vp(Mt), d, st), None,
                               "logdet_h_dev")
                _tail_fwd(L, fused, X, W1, b1, w2, b2, n, d, m1, Z, R, part, st)
                _lib.check(L.midagma_mlp_objective_part(_vp(part), part.numel(), _vp(l1part), l1part.numel(), _vp(h),
                                                        float(mu), float(lambda1), 0.5 * d, 1 / n, _vp(obj), ctr, st),
                           None, "mlp_objective_part")
        ctx.save_for_backward(X, W1, b1, w2, Z, R, Mt, part, scratch)
        ctx.consts = (n, d, m1, float(mu), float(lambda1), l1part.numel())
        ctx.fused = fused
        ctx.step = step
        ctx.h = h if step is not None else None  # (the step's default Adam gate: h >= 0)
        ctx.set_materialize_grads(False)  # h's own gradient stays None (no zero fill and add)
        return h, obj

    @staticmethod
    def backward(ctx, gh_out, g):
        X, W1, b1, w2, Z, R, Mt, part, scratch = ctx.saved_tensors
        n, d, m1, mu, lambda1, np_ = ctx.consts
        L = _lib.lib()
        dev = X.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        st = C.c_void_p(stream) if stream else None
        f64 = dict(dtype=torch.float64, device=dev)
        g = torch.zeros((), **f64) if g is None else g.contiguous()
        dw2, db2, db1 = torch.empty_like(w2), torch.empty((d, 1), **f64), torch.empty(d * m1, **f64)
        dW1 = torch.empty_like(W1)
        chain = ctx.chain
        with torch.cuda.device(dev):
            if chain is not None:
                chain.enqueue(2)
            # the objective's backward (d ssq, d h, d l1) is derived from g inside the tail's and the
            # fc1 terms' backward (midagma_*_obj): no launch of its own
            if ctx.fused:
                # the tail's backward and dZ^T X in one MFMA launch (dZ never stored), row-split slices
                nlin = int(L.midagma_mlp_fused_splits(n))
                lin = torch.empty((nlin, d * m1, d), **f64)
                _lib.check(L.midagma_mlp_tail_bwd_lin(_vp(Z), _vp(w2), _vp(R), _vp(X), _vp(part),
                                                      part.numel(), _vp(g), mu, 0.5 * d, 1 / n, n, d, m1, _vp(lin),
                                                      _vp(dw2), _vp(db2), _vp(db1), _vp(scratch), st), None,
                           "mlp_tail_bwd_lin")
                if chain is not None:
                    chain.enqueue(2)
            else:
                dZ = torch.empty_like(Z)
                step = ctx.step
                # (step: the chunk partials only; midagma_mlp_step sums them)
                _lib.check(L.midagma_mlp_tail_bwd_obj(_vp(Z), _vp(b1), _vp(w2), _vp(R), _vp(part), _vp(g), mu,
                                                      0.5 * d, 1 / n, n, d, m1, _vp(dZ),
                                                      None if step is not None else _vp(dw2),
                                                      None if step is not None else _vp(db2),
                                                      None if step is not None else _vp(db1), _vp(scratch), st),
                           None, "mlp_tail_bwd_obj")
                if chain is not None:
                    chain.enqueue(2)
                ks = LIN_SPLIT
                if n % ks == 0 and n >= 16 * ks:
                    r = n // ks
                    lin = torch.bmm(dZ.view(ks, r, -1).transpose(1, 2), X.view(ks, r, -1))  # (ks, d m1, d)
                    nlin = ks
                else:
                    lin = (dZ.t() @ X).contiguous()
                    nlin = 1
            if chain is not None:  # the rest of the chain and the objective, then join
                torch.cuda.current_stream(dev).wait_event(chain.finish())
                ctx.chain = None
            if ctx.step is not None:
                if gh_out is not None:
                    raise _lib.HipSolverError("the one-launch step takes d obj only (h's gradient is not an input)")
                ctx.step.close_step(Mt, g, mu, lambda1, lin, nlin, scratch, n, ctx.h, st)
                ctx.step, ctx.h = None, None
                return (None,) * 15
            if gh_out is None:
                _lib.check(L.midagma_fc1_terms_bwd_obj(_vp(W1), d, m1, _vp(Mt), _vp(g), mu, lambda1, _vp(lin), nlin,
                                                       _vp(dW1), st), None, "fc1_terms_bwd_obj")
            else:  # h is also an output whose gradient adds in (not the minimize loop's case)
                # (d obj / d ssq went into the tail's backward above: only d l1part and d h here)
                gl1, gh = torch.empty(np_, **f64), torch.empty((), **f64)
                _lib.check(L.midagma_mlp_objective_bwd(_vp(g), None, np_, mu, lambda1, 0.5 * d, 1 / n,
                                                       None, _vp(gl1), _vp(gh), st), None, "mlp_objective_bwd")
                gh = gh + gh_out
                _lib.check(L.midagma_fc1_terms_bwd(_vp(W1), d, m1, _vp(Mt), _vp(gh), _vp(gl1), _vp(lin), nlin,
                                                   _vp(dW1), st), None, "fc1_terms_bwd")
        return None, dW1, db1, dw2, db2, None, None, None, None, None, None, None, None, None, None


_SIDE: dict = {}


class _MlpStep:
    """The replayed DagmaNonlinear step of a [d, m1, 1] model closed by one launch
    (midagma_mlp_step, ABI 9): the tail's parameter-gradient sums, fc1's weight gradient, torch
    Adam over the four parameters (nonlinear.py:212-236) and the next step's fc1 terms, whose A and
    |fc1| partials the next forward then takes instead of launching fc1_terms.  Bit-identical to
    the separate launches (mlp_tail_dw, fc1_terms_bwd, adam_gated_table_multi, fc1_terms); the
    parameters' .grad stay None."""

    def __init__(self, L, model, params, exp_avg, exp_avg_sq, table, counter, beta1, beta2, eps, wd):
        fc = model.fc2[0]
        want = [model.fc1.weight, model.fc1.bias, fc.weight, fc.bias]
        if len(params) != 4 or any(p is not q for p, q in zip(params, want)):
            raise ValueError("_MlpStep: the parameters must be fc1.weight, fc1.bias, fc2.weight, fc2.bias")
        self.L, self.d, self.m1 = L, model.d, model.dims[1]
        arr = lambda ts: (C.c_void_p * 4)(*[C.c_void_p(t.data_ptr()) for t in ts])  # noqa: E731
        self.keep = (params, exp_avg, exp_avg_sq, table, counter)
        self.p, self.m, self.v = arr(params), arr(exp_avg), arr(exp_avg_sq)
        self.table, self.counter = table, counter
        self.coef = (1 - beta1, beta2, 1 - beta2, eps, wd)
        dev = params[0].device
        self.A = torch.empty((self.d, self.d), dtype=torch.float64, device=dev)
        self.l1part = torch.empty(int(L.midagma_fc1_terms_parts(self.d)), dtype=torch.float64, device=dev)
        self.gate = None  # None: this step's h (the reference's h < 0 exit); else a tensor (< 0: no step)
        self.refresh()

    def refresh(self):
        """A and the |fc1| partials of the current weights (before the first step of a call)."""
        W1 = self.keep[0][0]
        stream = torch.cuda.current_stream(W1.device).cuda_stream
        with torch.cuda.device(W1.device):
            _lib.check(self.L.midagma_fc1_terms(_vp(W1), self.d, self.m1, _vp(self.A), _vp(self.l1part),
                                                C.c_void_p(stream) if stream else None), None, "fc1_terms")

    def close_step(self, Mt, g, mu, lambda1, lin, nlin, scratch, n, h, st):
        gate = h if self.gate is None else self.gate
        w1, beta2, c2, eps, wd = self.coef
        _lib.check(self.L.midagma_mlp_step(self.p, self.m, self.v, n, self.d, self.m1, _vp(Mt), _vp(g), mu, lambda1,
                                           _vp(lin), nlin, _vp(scratch), _vp(self.table), _vp(self.counter), w1,
                                           beta2, c2, eps, wd, _vp(gate), _vp(self.A), _vp(self.l1part), st), None,
                   "mlp_step")


class _SideLogdet:
    """The h log-det (midagma_logdet_h_dev_part, or a warm-started LdFast step) enqueued part by
    part on a side stream, then the scalar objective once the tail's row partials are ready (objective
    = (event, part, l1part, mu, lambda1, half_d, inv_n, out, counter or None)).  A fast (LdFast, not
    exact) step's objective is never read (the loop reads the exact steps'): only its side effect,
    the Adam table's step counter `ctr`, is kept, advanced by the LdFast step's own end launch."""

    def __init__(self, L, side, A, d, s, h, Mt, ld=None, exact=True, ctr=None):
        self.L, self.side, self.A, self.d, self.s, self.h, self.Mt = L, side, A, d, s, h, Mt
        self.ld, self.exact = ld, exact
        self.parts = ld.parts(exact) if ld is not None else int(L.midagma_logdet_h_parts(d))
        self.next = 0
        self.objective = None
        # (a handle without the fast path runs the chain on every step, whose end never advances
        # the counter: its steps keep the objective launch, which does)
        self.skip = (not exact and ctr is not None and (ld is None or ld.has_fast)
                     and not os.environ.get("MIDAGMA_FAST_OBJECTIVE"))
        if ld is not None:  # (before any part: the handle reads it at the enqueue of its end)
            ld.set_counter(ctr if self.skip else None)

    def enqueue(self, k):
        ss = C.c_void_p(self.side.cuda_stream)
        while k > 0 and self.next < self.parts:
            if self.ld is not None:
                self.ld.enqueue(self.A, self.d, self.s, self.h, self.Mt, self.side.cuda_stream, self.exact, self.next)
            else:
                _lib.check(self.L.midagma_logdet_h_dev_part(_vp(self.A), self.d, self.d, self.s, _vp(self.h),
                                                            _vp(self.Mt), self.d, ss, self.next), None,
                           "logdet_h_dev_part")
            self.next += 1
            k -= 1

    def finish(self) -> torch.cuda.Event:
        self.enqueue(self.parts)
        ev_tail, part, l1part, mu, lambda1, half_d, inv_n, out, ctr = self.objective
        if self.skip:  # the step counter only (see the class docstring)
            if self.ld is None:
                _lib.check(self.L.midagma_counter_advance(ctr, C.c_void_p(self.side.cuda_stream)), None,
                           "counter_advance")
        else:
            self.side.wait_event(ev_tail)
            _lib.check(self.L.midagma_mlp_objective_part(_vp(part), part.numel(), _vp(l1part), l1part.numel(),
                                                         _vp(self.h), mu, lambda1, half_d, inv_n, _vp(out), ctr,
                                                         C.c_void_p(self.side.cuda_stream)), None,
                       "mlp_objective_part")
        ev = torch.cuda.Event()
        ev.record(self.side)
        return ev


class LdFast:
    """The h log-det of consecutive minimize steps with a warm start (midagma_ldfast_*, ABI 6): a
    fast step inverts sI - A by the product-form series from the last two steps' inverses and
    keeps the last exact h when that inverse is entrywise >= 0 (sI - A is then a nonsingular
    M-matrix and h >= 0, so the reference's h < 0 exit, nonlinear.py:206-208, cannot fire), else
    it runs the Gauss-Jordan chain on the device; an exact step always runs the chain (the steps
    whose objective the loop reads, nonlinear.py:214-217).  One per (model size, device)."""

    def __init__(self, d: int, device: int):
        self.L = _lib.lib()
        self.d, self.device = int(d), int(device)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.L.midagma_ldfast_create(C.byref(h), self.d), None, "ldfast_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.midagma_ldfast_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        with torch.cuda.device(self.device):
            _lib.check(self.L.midagma_ldfast_reset(self.h), None, "ldfast_reset")

    @property
    def has_fast(self) -> bool:
        """The warm-started fast path exists (d <= 256, include/midagma_hip.h ABI 6); larger d
        always runs the Gauss-Jordan chain."""
        return self.d <= 256

    def parts(self, exact: bool) -> int:
        return int(self.L.midagma_ldfast_parts(self.h, 1 if exact else 0))

    def enqueue(self, A, d, s, h, Mt, stream, exact: bool, part: int):
        _lib.check(self.L.midagma_ldfast_enqueue(self.h, _vp(A), d, d, float(s), _vp(h), _vp(Mt), d,
                                                 C.c_void_p(stream) if stream else None, 1 if exact else 0, part),
                   None, "ldfast_enqueue")

    def set_counter(self, counter):
        """Fast steps enqueued from now on advance `counter` (a c_void_p to a device int64, or
        None: off) in their end launch (midagma_ldfast_set_counter, ABI 10)."""
        _lib.check(self.L.midagma_ldfast_set_counter(self.h, counter), None, "ldfast_set_counter")

    def stats(self):
        """(steps, steps that ran the Gauss-Jordan chain) since the last reset."""
        a, b = C.c_int64(), C.c_int64()
        with torch.cuda.device(self.device):
            _lib.check(self.L.midagma_ldfast_stats(self.h, C.byref(a), C.byref(b)), None, "ldfast_stats")
        return int(a.value), int(b.value)


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """One side stream per device for the MLP objective's log-det (created outside any capture:
    the first step of every minimize call is a warm-up launched eagerly)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=key)
    return _SIDE[key]


def logdet_h(A: torch.Tensor, s: float = 1.0) -> torch.Tensor:
    """h(A) = -log|det(sI - A)| + d log s with gradient (sI - A)^{-T}, on the GPU."""
    return _LogdetH.apply(A, s)


class LocallyConnected(nn.Module):
    """Per-node local linear layer, [n, d, m1] -> [n, d, m2] (locally_connected.py:6-85)."""

    def __init__(self, num_linear: int, input_features: int, output_features: int, bias: bool = True):
        super().__init__()
        self.num_linear = num_linear
        self.input_features = input_features
        self.output_features = output_features
        self.weight = nn.Parameter(torch.empty(num_linear, input_features, output_features))
        self.bias = nn.Parameter(torch.empty(num_linear, output_features)) if bias else None
        if not bias:
            self.register_parameter("bias", None)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        bound = math.sqrt(1.0 / self.input_features)
        nn.init.uniform_(self.weight, -bound, bound)
        if self.bias is not None:
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # out[n, j, o] = sum_m x[n, j, m] w[j, m, o] (+ b[j, o]): the reference's broadcast matmul
        # (locally_connected.py:55-85) is n*d tiny (1 x m1) @ (m1 x m2) products, which the GPU
        # runs as a batched GEMM of n*d batches; a width-1 output is a multiply-and-reduce over m,
        # wider outputs one GEMM per node (same sums, at most an ulp of reordering apart)
        if self.output_features == 1:
            out = torch.sum(x * self.weight.squeeze(dim=2), dim=2, keepdim=True)
        else:
            out = torch.einsum("njm,jmo->njo", x, self.weight)
        if self.bias is not None:
            out = out + self.bias
        return out


class DagmaMLP(nn.Module):
    """MLP structural equations (nonlinear.py:14-115) with the HIP h_func."""

    def __init__(self, dims: typing.List[int], bias: bool = True, dtype: torch.dtype = torch.double):
        torch.set_default_dtype(dtype)
        super().__init__()
        assert len(dims) >= 2
        assert dims[-1] == 1
        self.dims, self.d = dims, dims[0]
        self.register_buffer("I", torch.eye(self.d), persistent=False)
        self.fc1 = nn.Linear(self.d, self.d * dims[1], bias=bias)
        nn.init.zeros_(self.fc1.weight)
        nn.init.zeros_(self.fc1.bias)
        self.fc2 = nn.ModuleList(
            [LocallyConnected(self.d, dims[l + 1], dims[l + 2], bias=bias) for l in range(len(dims) - 2)])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.fc1(x)
        x = x.view(-1, self.dims[0], self.dims[1])
        for fc in self.fc2:
            x = torch.sigmoid(x)
            x = fc(x)
        return x.squeeze(dim=2)

    def fused_tail(self) -> bool:
        """True when sum((self(X) - X)^2) can run as the fused HIP tail: one hidden layer, a
        width-1 output, biases, float64 on a ROCm device, d * m1 <= 7936 (one row staged in LDS)."""
        if len(self.fc2) != 1 or os.environ.get("MIDAGMA_NO_MLP_TAIL"):
            return False
        fc = self.fc2[0]
        w = fc.weight
        return (fc.output_features == 1 and fc.bias is not None and self.fc1.bias is not None and w.is_cuda
                and w.dtype == torch.float64 and self.d * self.dims[1] <= 7936)

    def squared_residual(self, x: torch.Tensor) -> torch.Tensor:
        """sum((self(x) - x)^2), the sum inside the log-MSE score (nonlinear.py:139-159)."""
        if self.fused_tail():
            fc = self.fc2[0]
            return _MLPTail.apply(self.fc1(x), fc.weight, fc.bias, x, self.dims[1])
        return torch.sum((self(x) - x) ** 2)

    def _adjacency_sq(self) -> torch.Tensor:
        w = self.fc1.weight.view(self.d, -1, self.d)
        return torch.sum(w ** 2, dim=1).t()  # [i, j]

    def h_func(self, s: float = 1.0) -> torch.Tensor:
        """log-det acyclicity of the induced adjacency (nonlinear.py:68-86), on the GPU."""
        return logdet_h(self._adjacency_sq(), s)

    def fc1_l1_reg(self) -> torch.Tensor:
        return torch.sum(torch.abs(self.fc1.weight))

    @torch.no_grad()
    def fc1_to_adj(self) -> np.ndarray:
        return torch.sqrt(self._adjacency_sq()).cpu().numpy()


class _GraphCaptureError(RuntimeError):
    pass


class _NoBar:
    def update(self, k=1):
        pass


class DagmaNonlinear:
    """DAGMA for nonlinear SEMs (nonlinear.py:118-331): the reference's outer loop and Adam
    over the model's parameters, on the model's ROCm device (moved there by `fit`), with the
    HIP log-det in ``model.h_func``.  ``device``: HIP ordinal (default: the current device)."""

    def __init__(self, model: nn.Module, verbose: bool = False, dtype: torch.dtype = torch.double, *,
                 device: typing.Optional[int] = None, graph: bool = True):
        self.vprint = print if verbose else (lambda *a, **k: None)
        self.model = model
        self.dtype = dtype
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        # one Adam step captured once per minimize call and replayed (hipGraph); False: eager steps
        self.graph = graph and not os.environ.get("MIDAGMA_NO_GRAPH")
        # the log-det on a side stream beside the rest of the step (MIDAGMA_NO_OVERLAP=1: one stream)
        self.overlap = not os.environ.get("MIDAGMA_NO_OVERLAP")

    def log_mse_loss(self, output: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        """d/2 log(1/n sum (output - target)^2)  (nonlinear.py:139-159)."""
        n, d = target.shape
        return 0.5 * d * torch.log(1 / n * torch.sum((output - target) ** 2))

    def _h_and_objective(self, mu: float, lambda1: float, s: float, overlap: bool = False, ld=None,
                         exact: bool = True, counter=None, step=None):
        """(h, mu * (score + lambda1 * |fc1|_1) + h) (nonlinear.py:198-204): for a [d, m1, 1] MLP
        on the GPU through the fused kernels (fc1 terms, log-det, tail, scalar objective),
        otherwise the reference's expressions."""
        m = self.model
        if getattr(m, "fused_tail", lambda: False)():
            n, d = self.X.shape
            m1 = m.dims[1]
            fc = m.fc2[0]
            return _MLPObjective.apply(self.X, m.fc1.weight, m.fc1.bias, fc.weight, fc.bias, d, m1, s, mu, lambda1,
                                       overlap, ld, exact, counter, step)
        h_val = m.h_func(s)
        return h_val, mu * (self._score() + lambda1 * m.fc1_l1_reg()) + h_val

    def _score(self) -> torch.Tensor:
        """log_mse_loss(model(X), X); the squared residual sum through the model's fused tail
        when it has one (same expression around it: 0.5 d log(1/n ssq))."""
        if hasattr(self.model, "squared_residual"):
            n, d = self.X.shape
            return 0.5 * d * torch.log(1 / n * self.model.squared_residual(self.X))
        return self.log_mse_loss(self.model(self.X), self.X)

    def minimize(self, max_iter: float, lr: float, lambda1: float, lambda2: float, mu: float, s: float,
                 lr_decay: float = False, tol: float = 1e-6, pbar=None) -> bool:
        """Adam on mu * (score + lambda1 |fc1|_1) + h (nonlinear.py:161-236); False when h < 0.

        The step is torch.optim.Adam's single-tensor algorithm (betas .99/.999, eps 1e-8, L2
        weight decay mu * lambda2) in one HIP kernel per parameter (`midagma_adam_step`), gated
        on the device value of h: the reference returns before stepping when h < 0, so a
        negative h freezes the parameters (and h) and is seen on the host at the next
        checkpoint instead of through a host read every step."""
        pbar = pbar or _NoBar()
        self.vprint(f"\nMinimize s={s} -- lr={lr}")
        if self.graph and max_iter > 2:
            try:
                return self._minimize_graph(max_iter, lr, lambda1, lambda2, mu, s, lr_decay, tol, pbar)
            except _GraphCaptureError as e:  # not capturable here: the same steps, launched eagerly
                self.vprint(f"hipGraph capture unavailable ({e}); eager steps")
        params = [p for p in self.model.parameters() if p.requires_grad]
        exp_avg = [torch.zeros_like(p) for p in params]
        exp_avg_sq = [torch.zeros_like(p) for p in params]
        beta1, beta2, eps, wd = 0.99, 0.999, 1e-8, mu * lambda2
        L = _lib.lib()
        lr_cur = lr
        obj_prev = 1e16
        for i in range(max_iter):
            for p in params:
                p.grad = None
            h_val, obj = self._h_and_objective(mu, lambda1, s, overlap=self.overlap)
            obj.backward()
            step = i + 1
            bc1 = 1 - beta1 ** step
            bc2 = 1 - beta2 ** step
            stream = torch.cuda.current_stream(h_val.device).cuda_stream
            gate = C.c_void_p(h_val.data_ptr())
            for p, m, v in zip(params, exp_avg, exp_avg_sq):
                g = p.grad.contiguous()
                _lib.check(L.midagma_adam_step(C.c_void_p(p.data_ptr()), C.c_void_p(g.data_ptr()),
                                               C.c_void_p(m.data_ptr()), C.c_void_p(v.data_ptr()), p.numel(),
                                               lr_cur / bc1, 1 - beta1, beta2, 1 - beta2, bc2 ** 0.5, eps, wd, gate,
                                               C.c_void_p(stream) if stream else None), None, "adam_step")
            if lr_decay and (i + 1) % 1000 == 0:
                lr_cur = lr_cur * 0.8   # ExponentialLR(gamma=0.8)
            if i % self.checkpoint == 0 or i == max_iter - 1:
                h_host = h_val.item()
                if h_host < 0:
                    self.vprint(f"Found h negative {h_host} at or before iter {i}")
                    return False
                obj_new = obj.item()
                self.vprint(f"\nInner iteration {i}")
                self.vprint(f"\th(W(model)): {h_host}")
                self.vprint(f"\tscore(model): {obj_new}")
                if np.abs((obj_prev - obj_new) / obj_prev) <= tol:
                    pbar.update(max_iter - i)
                    break
                obj_prev = obj_new
            pbar.update(1)
        return True

    def _minimize_graph(self, max_iter, lr, lambda1, lambda2, mu, s, lr_decay, tol, pbar) -> bool:
        """`minimize` with one step captured into a hipGraph and replayed: the same kernels as the
        eager loop, the per-step Adam coefficients (lr schedule and bias corrections, host-rounded
        as torch computes them) from a device table at a device step counter."""
        params = [p for p in self.model.parameters() if p.requires_grad]
        exp_avg = [torch.zeros_like(p) for p in params]
        exp_avg_sq = [torch.zeros_like(p) for p in params]
        beta1, beta2, eps, wd = 0.99, 0.999, 1e-8, mu * lambda2
        table = np.empty(2 * int(max_iter))
        lr_cur = lr
        for i in range(int(max_iter)):
            step = i + 1
            table[2 * i] = lr_cur / (1 - beta1 ** step)
            table[2 * i + 1] = (1 - beta2 ** step) ** 0.5
            if lr_decay and (i + 1) % 1000 == 0:
                lr_cur = lr_cur * 0.8
        dev = params[0].device
        # the fused objective advances the step counter itself (before the step's Adam launch),
        # so its Adam launches read the table one entry later: a leading pad entry
        fused = getattr(self.model, "fused_tail", lambda: False)()
        if fused:
            table = np.concatenate([np.zeros(2), table])
        table_d = torch.from_numpy(table).to(dev)
        counter = torch.zeros(1, dtype=torch.int64, device=dev)
        no_step = torch.full((), -1.0, dtype=torch.float64, device=dev)
        L = _lib.lib()

        seed = torch.ones((), dtype=torch.float64, device=dev)  # d obj / d obj: no fill node per step
        ld = self._ldfast(dev)
        # the step closed by one launch (_MlpStep; MIDAGMA_NO_MLP_STEP=1: the separate launches)
        step = None
        if fused and not FUSED_TAIL and not os.environ.get("MIDAGMA_NO_MLP_STEP"):
            try:
                with torch.no_grad():
                    step = _MlpStep(L, self.model, params, exp_avg, exp_avg_sq, table_d, counter, beta1, beta2, eps,
                                    wd)
            except ValueError:  # not the four [d, m1, 1] tensors (e.g. a frozen one): separate launches
                step = None

        def body(gate, exact=True):
            for p in params:
                p.grad = None
            if step is not None:
                step.gate = gate
            h_val, obj = self._h_and_objective(mu, lambda1, s, overlap=self.overlap, ld=ld, exact=exact,
                                               counter=counter if fused else None, step=step)
            obj.backward(seed)
            if step is not None:
                return h_val, obj
            stream = torch.cuda.current_stream(dev).cuda_stream
            st = C.c_void_p(stream) if stream else None
            g_ptr = C.c_void_p((h_val if gate is None else gate).data_ptr())
            grads = [p.grad.contiguous() for p in params]
            if len(params) <= 8:  # every parameter tensor in one launch
                k = len(params)
                arr = lambda ts: (C.c_void_p * k)(*[C.c_void_p(t.data_ptr()) for t in ts])  # noqa: E731
                _lib.check(L.midagma_adam_step_table_multi(
                    k, arr(params), arr(grads), arr(exp_avg), arr(exp_avg_sq),
                    (C.c_int64 * k)(*[p.numel() for p in params]), C.c_void_p(table_d.data_ptr()),
                    C.c_void_p(counter.data_ptr()), 1 - beta1, beta2, 1 - beta2, eps, wd, g_ptr, st), None,
                    "adam_step_table_multi")
            else:
                for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
                    _lib.check(L.midagma_adam_step_table(C.c_void_p(p.data_ptr()), C.c_void_p(g.data_ptr()),
                                                         C.c_void_p(m.data_ptr()), C.c_void_p(v.data_ptr()),
                                                         p.numel(), C.c_void_p(table_d.data_ptr()),
                                                         C.c_void_p(counter.data_ptr()), 1 - beta1, beta2,
                                                         1 - beta2, eps, wd, g_ptr, st), None, "adam_step_table")
            if not fused:
                _lib.check(L.midagma_counter_advance(C.c_void_p(counter.data_ptr()), st), None, "counter_advance")
            return h_val, obj

        try:
            # warm-up on a side stream with the step gated off: lazy allocations (the log-det
            # workspace, BLAS handles) happen outside the capture and the parameters stay put
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for exact in (True, False) if ld is not None else (True,):
                    body(no_step, exact)
            torch.cuda.current_stream(dev).wait_stream(side)
            counter.zero_()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                h_static, obj_static = body(None)
            # the steps whose objective the loop does not read: the log-det's warm-started fast path
            graph_fast = None
            if ld is not None:
                graph_fast = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph_fast):
                    body(None, False)
                torch.cuda.synchronize(dev)
                ld.reset()
        except Exception as e:  # noqa: BLE001
            for p in params:
                p.grad = None
            raise _GraphCaptureError(repr(e)) from e
        obj_prev = 1e16
        try:
            for i in range(max_iter):
                ck = i % self.checkpoint == 0 or i == max_iter - 1
                (graph if ck or graph_fast is None else graph_fast).replay()
                if ck:
                    h_host = h_static.item()
                    if h_host < 0:
                        self.vprint(f"Found h negative {h_host} at or before iter {i}")
                        return False
                    obj_new = obj_static.item()
                    self.vprint(f"\nInner iteration {i}")
                    self.vprint(f"\th(W(model)): {h_host}")
                    self.vprint(f"\tscore(model): {obj_new}")
                    if np.abs((obj_prev - obj_new) / obj_prev) <= tol:
                        pbar.update(max_iter - i)
                        break
                    obj_prev = obj_new
                pbar.update(1)
            return True
        finally:
            torch.cuda.current_stream(dev).synchronize()
            for p in params:
                p.grad = None
            del graph, graph_fast

    def _ldfast(self, dev: torch.device):
        """The warm-started log-det handle of this model's [d, m1, 1] objective (None: the fused
        objective does not apply, d > 256, or MIDAGMA_NO_LDFAST=1 keeps every step exact)."""
        m = self.model
        if os.environ.get("MIDAGMA_NO_LDFAST") or not getattr(m, "fused_tail", lambda: False)():
            return None
        d = self.X.shape[1]
        if d > 256:
            return None
        key = (d, dev.index)
        if getattr(self, "_ld", None) is None or self._ld_key != key:
            self._ld = LdFast(d, dev.index)
            self._ld_key = key
        return self._ld

    def fit(self, X, lambda1: float = .02, lambda2: float = .005, T: int = 4, mu_init: float = .1,
            mu_factor: float = .1, s: float = 1.0, warm_iter: int = 5e4, max_iter: int = 8e4, lr: float = .0002,
            w_threshold: float = 0.3, checkpoint: int = 1000) -> np.ndarray:
        """The reference's path following (nonlinear.py:238-331); X: (n, d) numpy or torch."""
        torch.set_default_dtype(self.dtype)
        if isinstance(X, torch.Tensor):
            self.X = X.type(self.dtype)
        elif isinstance(X, np.ndarray):
            self.X = torch.from_numpy(X).type(self.dtype)
        else:
            ValueError("X should be numpy array or torch Tensor.")  # built, not raised (as the reference)
        self.model.to(self.device)
        self.X = self.X.to(self.device)
        self.checkpoint = checkpoint
        mu = mu_init
        if type(s) == list:
            if len(s) < T:
                self.vprint(f"Length of s is {len(s)}, using last value in s for iteration t >= {len(s)}")
                s = s + (T - len(s)) * [s[-1]]
        elif type(s) in [int, float]:
            s = T * [s]
        else:
            ValueError("s should be a list, int, or float.")
        pbar = _NoBar()
        for i in range(int(T)):
            self.vprint(f"\nDagma iter t={i + 1} -- mu: {mu}", 30 * "-")
            success, s_cur = False, s[i]
            inner_iter = int(max_iter) if i == T - 1 else int(warm_iter)
            model_copy = copy.deepcopy(self.model)
            lr_decay = False
            while success is False:
                success = self.minimize(inner_iter, lr, lambda1, lambda2, mu, s_cur, lr_decay, pbar=pbar)
                if success is False:
                    self.model.load_state_dict(model_copy.state_dict().copy())
                    lr *= 0.5
                    lr_decay = True
                    if lr < 1e-10:
                        break
                    s_cur = 1
            mu *= mu_factor
        W_est = self.model.fc1_to_adj()
        W_est[np.abs(W_est) < w_threshold] = 0
        return W_est
