"""Config 5: is the replayed step bound by the host's graph submission?  Times the host side of
every CUDAGraph.replay() of DagmaNonlinear.minimize (monkeypatched) against the wall clock of
the whole call (diagnostic)."""
import os
import sys
import time

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear  # noqa: E402
from midagma_amd.simulate import make_dataset  # noqa: E402

acc = [0.0, 0]
_orig = torch.cuda.CUDAGraph.replay


def timed_replay(self):
    t = time.perf_counter()
    _orig(self)
    acc[0] += time.perf_counter() - t
    acc[1] += 1


torch.cuda.CUDAGraph.replay = timed_replay
d, n = 200, 1000
X, _, _ = make_dataset(d, n, seed=0)
torch.manual_seed(0)
model = DagmaMLP(dims=[d, 10, 1]).to(torch.device("cuda", 0))
with torch.no_grad():
    model.fc1.weight.normal_(0, 0.3 / np.sqrt(10 * d))
dn = DagmaNonlinear(model, device=0)
dn.X = torch.from_numpy(X).to(torch.device("cuda", 0))
dn.checkpoint = 10 ** 9
dn.minimize(20, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
torch.cuda.synchronize()
for K in (2000, 2000):
    acc[:] = [0.0, 0]
    t0 = time.perf_counter()
    dn.minimize(K, 2e-4, 0.02, 0.005, 0.1, 1.0, tol=-1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"K={K}: {K / dt:.0f} steps/s, wall {dt / K * 1e6:.1f} us/step, host replay() {acc[0] / max(acc[1], 1) * 1e6:.1f} "
          f"us per call over {acc[1]} calls", flush=True)
