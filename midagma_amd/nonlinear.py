"""`DagmaMLP` whose log-det acyclicity term runs on the HIP GJ/log-det kernel.

Mirrors `dagma.nonlinear.DagmaMLP` (fbleile/midagma, src/dagma/nonlinear.py:14-115)
and `LocallyConnected` (src/dagma/locally_connected.py).  The MLP forward and
the score stay PyTorch-ROCm; only
``h_func`` (nonlinear.py:68-86) is replaced:

    A = sum_m fc1_w[j, m, i]^2   (transposed: [i, j])
    h = -log|det(sI - A)| + d log s          forward  : HIP blocked Gauss-Jordan
    dh/dA = (sI - A)^{-T}                     backward : the inverse the forward produced

The C entry point (`midagma_logdet_inv_dev`) works on torch's device memory
and current HIP stream; it never synchronizes with the host.
"""
from __future__ import annotations

import ctypes as C
import math
import typing

import numpy as np
import torch
import torch.nn as nn

from . import _lib

__all__ = ["LocallyConnected", "DagmaMLP", "logdet_h"]


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
        out = torch.matmul(x.unsqueeze(dim=2), self.weight.unsqueeze(dim=0)).squeeze(dim=2)
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
