"""CPU oracle for the nonlinear path -- TEST INFRASTRUCTURE ONLY.

Restates, with torch on the CPU in float64, the reference's
`DagmaMLP` (/root/reference/src/dagma/nonlinear.py:14-115, h_func by `torch.slogdet` as
at :84-85), `LocallyConnected` (locally_connected.py:6-85) and `DagmaNonlinear.minimize` /
`fit` (nonlinear.py:161-331).  Pinned against the reference's own trajectories
(tests/golden/mlp_traj.npz, tests/test_mlp_oracle.py).  Only tests/ and bench.py's
cpu_baseline use it; the GPU path is midagma_amd/nonlinear.py.
"""
from __future__ import annotations

import copy
import math

import numpy as np
import torch
import torch.nn as nn

__all__ = ["OracleMLP", "nonlinear_minimize", "nonlinear_fit", "load_params"]


class _LC(nn.Module):
    def __init__(self, num_linear, input_features, output_features):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(num_linear, input_features, output_features))
        self.bias = nn.Parameter(torch.zeros(num_linear, output_features))

    def forward(self, x):   # locally_connected.py:55-85
        out = torch.matmul(x.unsqueeze(dim=2), self.weight.unsqueeze(dim=0)).squeeze(dim=2)
        return out + self.bias


class OracleMLP(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims, self.d = dims, dims[0]
        self.I = torch.eye(self.d, dtype=torch.double)
        self.fc1 = nn.Linear(self.d, self.d * dims[1], bias=True).double()
        self.fc2 = nn.ModuleList([_LC(self.d, dims[l + 1], dims[l + 2]).double() for l in range(len(dims) - 2)])

    def forward(self, x):   # nonlinear.py:45-66
        x = self.fc1(x)
        x = x.view(-1, self.dims[0], self.dims[1])
        for fc in self.fc2:
            x = torch.sigmoid(x)
            x = fc(x)
        return x.squeeze(dim=2)

    def h_func(self, s=1.0):   # nonlinear.py:68-86
        w = self.fc1.weight.view(self.d, -1, self.d)
        A = torch.sum(w ** 2, dim=1).t()
        return -torch.slogdet(s * self.I - A)[1] + self.d * np.log(s)

    def fc1_l1_reg(self):
        return torch.sum(torch.abs(self.fc1.weight))

    @torch.no_grad()
    def fc1_to_adj(self):
        w = self.fc1.weight.view(self.d, -1, self.d)
        return torch.sqrt(torch.sum(w ** 2, dim=1).t()).numpy()


def load_params(model: nn.Module, params: dict):
    sd = model.state_dict()
    with torch.no_grad():
        for k, v in params.items():
            sd[k].copy_(torch.as_tensor(np.asarray(v), dtype=sd[k].dtype).to(sd[k].device))


def _log_mse(output, target):
    n, d = target.shape
    return 0.5 * d * torch.log(1 / n * torch.sum((output - target) ** 2))


def nonlinear_minimize(model, X, max_iter, lr, lambda1, lambda2, mu, s, lr_decay=False, tol=1e-6,
                       checkpoint=1000):
    """DagmaNonlinear.minimize (nonlinear.py:161-236); returns (success, iterations run)."""
    optimizer = torch.optim.Adam(model.parameters(), lr=lr, betas=(.99, .999), weight_decay=mu * lambda2)
    if lr_decay is True:
        scheduler = torch.optim.lr_scheduler.ExponentialLR(optimizer, gamma=0.8)
    obj_prev = 1e16
    i = -1
    for i in range(max_iter):
        optimizer.zero_grad()
        h_val = model.h_func(s)
        if h_val.item() < 0:
            return False, i
        obj = mu * (_log_mse(model(X), X) + lambda1 * model.fc1_l1_reg()) + h_val
        obj.backward()
        optimizer.step()
        if lr_decay and (i + 1) % 1000 == 0:
            scheduler.step()
        if i % checkpoint == 0 or i == max_iter - 1:
            obj_new = obj.item()
            if np.abs((obj_prev - obj_new) / obj_prev) <= tol:
                break
            obj_prev = obj_new
    return True, i + 1


def nonlinear_fit(model, X, lambda1=.02, lambda2=.005, T=4, mu_init=.1, mu_factor=.1, s=1.0, warm_iter=5e4,
                  max_iter=8e4, lr=.0002, w_threshold=0.3, checkpoint=1000):
    """DagmaNonlinear.fit (nonlinear.py:238-331)."""
    mu = mu_init
    s = T * [s] if type(s) in (int, float) else s + (T - len(s)) * [s[-1]]
    for i in range(int(T)):
        success, s_cur = False, s[i]
        inner = int(max_iter) if i == T - 1 else int(warm_iter)
        model_copy = copy.deepcopy(model)
        lr_decay = False
        while success is False:
            success, _ = nonlinear_minimize(model, X, inner, lr, lambda1, lambda2, mu, s_cur, lr_decay,
                                            checkpoint=checkpoint)
            if success is False:
                model.load_state_dict(model_copy.state_dict().copy())
                lr *= 0.5
                lr_decay = True
                if lr < 1e-10:
                    break
                s_cur = 1
        mu *= mu_factor
    W = model.fc1_to_adj()
    W[np.abs(W) < w_threshold] = 0
    return W
