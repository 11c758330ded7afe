"""fc1 and the DagmaMLP tail fused on the MFMA (csrc/mlp.hip, experiments build: measured slower
than the product sequence at config 5) against the product sequence.  Run with

    MIDAGMA_LIB=midagma_amd/libmidagma_hip_exp.so python -m pytest -m experiment tests
"""
import numpy as np
import pytest

pytestmark = pytest.mark.experiment

torch = pytest.importorskip("torch")
@pytest.mark.parametrize("d,m1,n", [(200, 10, 1000), (30, 10, 500), (7, 3, 33), (20, 1, 64), (17, 16, 100),
                                    (256, 8, 130), (9, 9, 40)])
def test_fused_fc1_tail_matches_product(monkeypatch, d, m1, n):
    """fc1 and the tail fused on the MFMA (midagma_mlp_fc1_tail_fwd / _tail_bwd_lin, ABI 7) against
    the ABI-6 sequence (fc1 as a library GEMM, the tail kernels, split-K dZ^T X): h, objective and
    every parameter gradient.  Ragged n (row tiles of 64, row splits of 128), d not a multiple of 16,
    m1 = 1 / 3 / 8 / 10 / 16 (forward tiles of 128 / 96 / 128 / 80 / 128 columns) and m1 = 9, which
    the fused path does not take (falls back).  Tolerance: summation order only."""
    import midagma_amd.nonlinear as nl
    from midagma_amd import _lib
    from midagma_amd.nonlinear import DagmaMLP, DagmaNonlinear
    L = _lib.lib()
    if not hasattr(L, "midagma_mlp_fused_parts"):
        pytest.skip("needs the experiments build (MIDAGMA_LIB=.../libmidagma_hip_exp.so)")
    monkeypatch.setattr(nl, "FUSED_TAIL", True)
    assert (nl._fused_parts(L, n, d, m1) > 0) == (m1 != 9)
    torch.manual_seed(d * 7 + m1)
    model = DagmaMLP(dims=[d, m1, 1]).to("cuda:0")
    with torch.no_grad():
        model.fc1.weight.normal_(0, 0.3 / np.sqrt(d * m1))
        model.fc1.bias.normal_(0, 0.1)
    dn = DagmaNonlinear(model, device=0)
    dn.X = torch.randn(n, d, dtype=torch.float64, device="cuda:0")
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(nl, "FUSED_TAIL", fused)
        model.zero_grad()
        h, obj = dn._h_and_objective(0.1, 0.02, 1.0)
        obj.backward()
        res[fused] = (h.item(), obj.item(), {k: p.grad.detach().clone() for k, p in model.named_parameters()})
    (h1, o1, g1), (h0, o0, g0) = res[True], res[False]
    assert h1 == h0 and abs(o1 - o0) <= 1e-13 * abs(o0)
    for k in g0:
        assert torch.max(torch.abs(g1[k] - g0[k])).item() <= 1e-12 * max(1e-300, torch.max(torch.abs(g0[k])).item()), k
