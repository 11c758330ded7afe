"""The reference MLP trajectory's sensitivity (development tool, CPU only): the oracle's
DagmaNonlinear.minimize at dims [200, 10, 1], n = 1000 (the bench's config-5 leg: calls of 20, 300,
700, 1000 steps) from the bench's start and from the same start scaled by (1 + 1e-15); prints the
relative parameter separation after each call.  Shows where a 1e-9 comparison stops being meaningful.

    python tools/mlp_chaos.py [seed]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle.mlp_oracle import OracleMLP, load_params, nonlinear_minimize
from midagma_amd.simulate import make_dataset
d, n = 200, 1000
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
X, _, _ = make_dataset(d, n, seed=seed)
torch.manual_seed(seed)
from midagma_amd.nonlinear import DagmaMLP
model = DagmaMLP(dims=[d, 10, 1])
with torch.no_grad():
    model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * d))
params = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items() if k != "I"}
res = []
for eps in (0.0, 1e-15):
    m = OracleMLP([d, 10, 1])
    p = {k: v * (1 + eps) for k, v in params.items()}
    load_params(m, p)
    Xt = torch.from_numpy(X)
    out = []
    for K in (20, 300, 700, 1000):
        nonlinear_minimize(m, Xt, K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1, checkpoint=10 ** 9)
        out.append({k: v.detach().numpy().copy() for k, v in m.state_dict().items() if k in params})
    res.append(out)
for i, K in enumerate((20, 320, 1020, 2020)):
    a, b = res[0][i], res[1][i]
    print(K, {k: float(np.abs(a[k] - b[k]).max() / max(1, np.abs(a[k]).max())) for k in a})
