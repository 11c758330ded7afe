"""ctypes binding of the HIP library (include/midagma_hip.h).

This is the "reference-side binding a maintainer would add": the reference's
hot path is a Python method, so the FFI is ctypes over the C ABI.  The library
is built in-tree (``midagma_amd/libmidagma_hip.so``, see csrc/Makefile) and
there is NO fallback: if the library or a GPU is missing, every entry point
raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

__all__ = ["lib", "load", "check", "MidagmaResult", "MidagmaCkpt", "LIB_PATH", "HipSolverError",
           "ST_RUNNING", "ST_DONE", "ST_FAILED", "ST_LR_UNDERFLOW", "ST_SINGULAR",
           "LOSS_L2", "LOSS_LOGISTIC", "MODE_COV", "MODE_DATA", "EXPORTED", "GROUP_EMULATE"]

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmidagma_hip.so")

OK, E_HIP, E_SINGULAR, E_ARG, E_STATE = 0, -1, -2, -3, -4
LOSS_L2, LOSS_LOGISTIC = 0, 1
MODE_COV, MODE_DATA = 0, 1
ST_RUNNING, ST_DONE, ST_FAILED, ST_LR_UNDERFLOW, ST_SINGULAR = 0, 1, 2, 3, 4


class MidagmaResult(C.Structure):
    _fields_ = [("iters", C.c_int64), ("halvings", C.c_int64), ("slots", C.c_int64),
                ("n_checkpoints", C.c_int64), ("status", C.c_int32), ("early_stop", C.c_int32),
                ("lr_final", C.c_double), ("obj_last", C.c_double), ("score_last", C.c_double),
                ("h_last", C.c_double), ("l1_last", C.c_double)]


class MidagmaCkpt(C.Structure):
    _fields_ = [("iter", C.c_int64), ("obj", C.c_double), ("score", C.c_double), ("h", C.c_double),
                ("lr", C.c_double), ("l1", C.c_double),
                ("w_norm", C.c_double), ("max_abs_w", C.c_double), ("min_abs_w_nonzero", C.c_double),
                ("grad_raw_norm", C.c_double), ("grad_step_norm", C.c_double), ("grad_score_norm", C.c_double),
                ("grad_dag_norm", C.c_double), ("grad_l1_norm", C.c_double), ("grad_inc_norm", C.c_double),
                ("elapsed", C.c_double), ("reg_trek_value", C.c_double), ("grad_trek_norm", C.c_double)]


class HipSolverError(RuntimeError):
    pass


_dp = C.POINTER(C.c_double)
_vp = C.c_void_p
_i64 = C.c_int64
_d = C.c_double
_int = C.c_int

# name -> (restype, argtypes); every symbol declared in include/midagma_hip.h
EXPORTED = {
    "midagma_abi_version": (_int, []),
    "midagma_device_count": (_int, [C.POINTER(_int)]),
    "midagma_last_error": (C.c_char_p, [_vp]),
    "midagma_create": (_int, [C.POINTER(_vp), _int, _int, _i64, _int, _vp]),
    "midagma_destroy": (None, [_vp]),
    "midagma_stream": (_vp, [_vp]),
    "midagma_padded_dim": (_i64, [_vp]),
    "midagma_set_cov": (_int, [_vp, _dp, _i64]),
    "midagma_set_masks": (_int, [_vp, _dp, _dp]),
    "midagma_set_w_float32": (_int, [_vp, _int]),
    "midagma_set_data": (_int, [_vp, _vp, _i64, _i64, _int]),
    "midagma_data_gram": (_int, [_vp]),
    "midagma_cov_from_zbuf": (_int, [_vp, _d]),
    "midagma_get_cov": (_int, [_vp, _dp, _i64]),
    "midagma_colsum_dev": (_int, [_vp, _i64, _i64, _i64, _vp, _vp]),
    "midagma_center_dev": (_int, [_vp, _i64, _i64, _i64, _vp, _d, _vp]),
    "midagma_gram": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _i64, _vp]),
    "midagma_set_cov_dev": (_int, [_vp, _vp, _i64, _d]),
    "midagma_comm_unique_id": (_int, [_vp, _i64]),
    "midagma_comm_init": (_int, [_vp, _vp, _i64, _int, _int]),
    "midagma_comm_ranks": (_int, [_vp]),
    "midagma_comm_allreduce_zbuf": (_int, [_vp]),
    "midagma_zbuf_len": (_i64, [_vp]),
    "midagma_bind_zbuf": (_int, [_vp, _vp, _i64]),
    "midagma_minimize": (_int, [_vp, _dp, _d, _i64, _d, _d, _d, _d, _d, _d, _i64, C.POINTER(MidagmaResult)]),
    "midagma_begin": (_int, [_vp, _dp, _d, _i64, _d, _d, _d, _d, _d, _d, _i64]),
    "midagma_step_partial": (_int, [_vp]),
    "midagma_run_slots": (_int, [_vp, _i64]),
    "midagma_sync": (_int, [_vp]),
    "midagma_profile_parts": (_int, [_vp, _int, _dp]),
    "midagma_step_finish": (_int, [_vp]),
    "midagma_poll": (_int, [_vp, C.POINTER(MidagmaResult)]),
    "midagma_end": (_int, [_vp, _dp, C.POINTER(MidagmaResult)]),
    "midagma_checkpoints": (_i64, [_vp, C.POINTER(MidagmaCkpt), _i64]),
    "midagma_set_trek": (_int, [_vp, _int, _int, _int, _d, _d, _i64, C.POINTER(_i64), _i64]),
    "midagma_set_trek_tcc": (_int, [_vp, _int, _d, _d, _d, C.POINTER(_i64), _i64]),
    "midagma_trek": (_int, [_vp, _dp, _dp, _dp]),
    "midagma_h": (_int, [_vp, _dp, _d, _dp, _dp]),
    "midagma_score": (_int, [_vp, _dp, _dp, _dp]),
    "midagma_score_partial": (_int, [_vp, _dp]),
    "midagma_score_finish": (_int, [_vp, _dp, _dp]),
    "midagma_logdet_inv_dev": (_int, [_vp, _i64, _i64, _d, _vp, _vp, _i64, _vp]),
    "midagma_sem_linear": (_int, [_dp, _i64, _i64, _i64, _int, _dp, C.c_uint64, _vp, _i64, _vp]),
    "midagma_adam_step": (_int, [_vp, _vp, _vp, _vp, _i64, _d, _d, _d, _d, _d, _d, _d, _vp, _vp]),
    "midagma_adam_step_table": (_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _d, _d, _d, _d, _d, _vp, _vp]),
    "midagma_counter_advance": (_int, [_vp, _vp]),
    "midagma_adam_step_table_multi": (_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _d, _d, _d, _d, _d, _vp, _vp]),
    "midagma_mlp_tail_scratch": (_i64, [_i64, _i64, _i64]),
    "midagma_fc1_terms_parts": (_i64, [_i64]),
    "midagma_fc1_terms": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "midagma_fc1_terms_bwd": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "midagma_logdet_h_dev": (_int, [_vp, _i64, _i64, _d, _vp, _vp, _i64, _vp]),
    "midagma_logdet_h_parts": (_i64, [_i64]),
    "midagma_logdet_h_dev_part": (_int, [_vp, _i64, _i64, _d, _vp, _vp, _i64, _vp, _i64]),
    "midagma_mlp_objective": (_int, [_vp, _vp, _i64, _vp, _d, _d, _d, _d, _vp, _vp]),
    "midagma_mlp_objective_bwd": (_int, [_vp, _vp, _i64, _d, _d, _d, _d, _vp, _vp, _vp, _vp]),
    "midagma_ldfast_create": (_int, [C.POINTER(_vp), _i64]),
    "midagma_ldfast_destroy": (None, [_vp]),
    "midagma_ldfast_reset": (_int, [_vp]),
    "midagma_ldfast_parts": (_i64, [_vp, _int]),
    "midagma_ldfast_enqueue": (_int, [_vp, _vp, _i64, _i64, _d, _vp, _vp, _i64, _vp, _int, _i64]),
    "midagma_ldfast_stats": (_int, [_vp, C.POINTER(_i64), C.POINTER(_i64)]),
    "midagma_ldfast_set_counter": (_int, [_vp, _vp]),
    "midagma_mlp_tail_fwd_part": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "midagma_mlp_objective_part": (_int, [_vp, _i64, _vp, _i64, _vp, _d, _d, _d, _d, _vp, _vp, _vp]),
    "midagma_mlp_tail_bwd_obj": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _d, _d, _d, _i64, _i64, _i64, _vp, _vp, _vp,
                                        _vp, _vp, _vp]),
    "midagma_fc1_terms_bwd_obj": (_int, [_vp, _i64, _i64, _vp, _vp, _d, _d, _vp, _i64, _vp, _vp]),
    "midagma_mlp_step": (_int, [C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), _i64, _i64, _i64, _vp, _vp, _d, _d,
                                _vp, _i64, _vp, _vp, _vp, _d, _d, _d, _d, _d, _vp, _vp, _vp, _vp]),
    "midagma_mlp_tail_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "midagma_mlp_tail_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    # ABI 11: data mode on several devices from one process (midagma_amd.solver.HipGroup)
    "midagma_group_create": (_int, [C.POINTER(_vp), _int, _i64, C.POINTER(_int), _int, _int]),
    "midagma_group_destroy": (None, [_vp]),
    "midagma_group_last_error": (C.c_char_p, [_vp]),
    "midagma_group_size": (_int, [_vp]),
    "midagma_group_emulated": (_int, [_vp]),
    "midagma_group_member": (_vp, [_vp, _int]),
    "midagma_group_set_data": (_int, [_vp, _dp, _i64]),
    "midagma_group_allreduce_zbuf": (_int, [_vp]),
    "midagma_group_minimize": (_int, [_vp, _dp, _d, _i64, _d, _d, _d, _d, _d, _d, _i64, C.POINTER(MidagmaResult)]),
}

GROUP_EMULATE = 1

_lock = threading.Lock()
_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load the HIP library (once).  Raises loudly when it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("MIDAGMA_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise HipSolverError(
                f"midagma HIP library not found at {p}; build it with `make -C midagma_amd/csrc` "
                "(there is no CPU fallback)")
        # torch, when present, must own the HIP runtime first so both share one instance
        try:  # pragma: no cover - import side effect only
            import torch  # noqa: F401
        except Exception:
            pass
        handle = C.CDLL(p, mode=C.RTLD_GLOBAL)
        for name, (res, args) in EXPORTED.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def lib() -> C.CDLL:
    return load()


def last_error(handle=None) -> str:
    msg = lib().midagma_last_error(handle)
    return msg.decode() if msg else ""


def check(rc: int, handle=None, what: str = "", group: bool = False):
    """Raise for a negative return code: LinAlgError (singular), ValueError (bad argument,
    non-finite input) or HipSolverError; `group`: the handle is a midagma_group."""
    if rc >= 0:
        return rc
    if group:
        m = lib().midagma_group_last_error(handle)
        msg = m.decode() if m else ""
    else:
        msg = last_error(handle)
    if rc == E_SINGULAR:
        raise np.linalg.LinAlgError(msg or "singular matrix")
    if rc == E_ARG:
        raise ValueError(f"{what}: {msg}")
    raise HipSolverError(f"{what} failed ({rc}): {msg}")


def dptr(a: np.ndarray):
    """double* of a C-contiguous float64 array (or NULL for None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)
