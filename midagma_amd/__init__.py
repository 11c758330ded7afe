"""midagma_amd -- MI355X-native DAGMA inner solver (drop-in for fbleile/midagma's hot path).

    from midagma_amd import DagmaLinear          # dagma.linear.DagmaLinear API, GPU inner loop
    from midagma_amd.nonlinear import DagmaMLP   # dagma.nonlinear.DagmaMLP with the HIP h_func

The compute path is hand-written HIP for gfx950 in `midagma_amd/csrc`, built
in-tree into `libmidagma_hip.so` and bound with ctypes (`_lib.py`).
"""
from .linear import DagmaLinear  # noqa: F401
from .simulate import count_accuracy, is_dag, make_dataset  # noqa: F401
from .solver import HipSolver, MinimizeResult, device_count, run_allreduce_minimize  # noqa: F401

__version__ = "0.1.0"
