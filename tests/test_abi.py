"""The C-ABI library loads and exports every symbol include/midagma_hip.h declares
(no device calls: runs in the build container without a GPU)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "midagma_hip.h")).read()
    return sorted(set(re.findall(r"\b(midagma_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    from midagma_amd._lib import EXPORTED
    assert _declared() == sorted(EXPORTED)


def test_library_exports_every_symbol():
    from midagma_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libmidagma_hip.so not built (run __graft_entry__.build())")
    L = _lib.load()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.midagma_abi_version() == 6


def test_missing_library_fails_loudly(tmp_path):
    from midagma_amd import _lib
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from midagma_amd import _lib\n"
            "try:\n    _lib.load(%r)\nexcept _lib.HipSolverError as e:\n    print('raised', e)\n") % (
        REPO, str(tmp_path / "nope.so"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "raised" in out.stdout


def test_create_without_gpu_raises():
    """No silent CPU path: creating a solver on a machine without a GPU is an error."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from midagma_amd.solver import HipSolver
    from midagma_amd._lib import HipSolverError
    with pytest.raises(HipSolverError):
        HipSolver(8)
