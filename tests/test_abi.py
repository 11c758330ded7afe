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
    assert L.midagma_abi_version() == 11


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


def test_product_library_reads_no_experiment_knobs():
    """The product library compiles every MIDAGMA_EXP_* experiment knob to its default
    (csrc/knobs.h): no such variable name is in it, and the rejected one-launch inverse
    (dfinv.hip) is not linked in; the experiments build has both."""
    from midagma_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"MIDAGMA_EXP_" not in blob
    assert b"midagma_debug_df_plan" not in blob and b"df_plan" not in blob
    exp = os.path.join(os.path.dirname(_lib.LIB_PATH), "libmidagma_hip_exp.so")
    if os.path.exists(exp):
        eb = open(exp, "rb").read()
        assert b"MIDAGMA_EXP_DF" in eb and b"midagma_debug_df_plan" in eb


def test_ldfast_entry_points_validate_without_a_device():
    """The ABI-6 warm-started log-det entries refuse bad arguments before touching a device."""
    import ctypes as C
    from midagma_amd import _lib
    L = _lib.load()
    assert L.midagma_ldfast_parts(None, 1) == 0
    assert L.midagma_ldfast_enqueue(None, None, 10, 10, 1.0, None, None, 10, None, 0, -1) == -3
    out = C.c_void_p()
    assert L.midagma_ldfast_create(C.byref(out), 0) == -3
    assert L.midagma_ldfast_reset(None) == -3
    assert L.midagma_ldfast_set_counter(None, None) == -3


def test_group_entry_points_validate_without_a_device():
    """ABI 11: the device-group entries refuse bad arguments (and a missing device) before touching
    a device, with their message from midagma_group_last_error."""
    import ctypes as C
    from midagma_amd import _lib
    L = _lib.load()
    out = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.midagma_group_create(C.byref(out), 0, 10, devs, 0, 0) == -3          # ndev 0
    assert L.midagma_group_create(C.byref(out), 0, 10, devs, 2, 4) == -3          # unknown flag
    assert L.midagma_group_create(C.byref(out), 2, 10, devs, 2, 0) == -3          # unknown loss
    assert b"bad arguments" in L.midagma_group_last_error(None)
    assert L.midagma_group_size(None) == 0 and L.midagma_group_emulated(None) == 0
    assert L.midagma_group_member(None, 0) is None
    assert L.midagma_group_set_data(None, None, 10) == -3
    assert L.midagma_group_allreduce_zbuf(None) == -3
    assert L.midagma_group_minimize(None, None, 1.0, 1, 1.0, 3e-4, 1e-6, .99, .999, .03, 1000, None) == -3
    import torch
    if not torch.cuda.is_available():
        # no device: creating a group fails loudly (no CPU path)
        rc = L.midagma_group_create(C.byref(out), 0, 10, devs, 2, _lib.GROUP_EMULATE)
        assert rc < 0
