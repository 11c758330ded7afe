"""Structured logging: the `minimize.checkpoint` row schema of the
reference (linear.py:290-326) and the logger sinks (src/logger.py).  CPU only."""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from midagma_amd.slog import LogConfig, StructuredLogger, build_default_logger, checkpoint_row

# keys of the reference's emit() payload, linear.py:290-326, in order
REF_KEYS = ["iter", "stage", "elapsed_sec", "obj_total", "score_datafit", "reg_dag_name", "reg_dag_value",
            "reg_dag_cfg", "reg_trek_name", "reg_trek_value", "reg_trek_cfg", "trek_mode", "trek_weight", "mu",
            "lr", "w_norm", "w_abs_sum", "max_abs_w", "min_abs_w_nonzero", "grad_raw_norm", "grad_step_norm",
            "step_norm", "grad_score_norm", "grad_dag_norm", "grad_l1_norm", "grad_inc_norm", "grad_trek_norm"]


def _rec(it=1000, lr=3e-4, gstep=2.0):
    return SimpleNamespace(iter=it, obj=1.5, score=1.25, h=0.01, lr=lr, l1=3.0, w_norm=1.1, max_abs_w=0.9,
                           min_abs_w_nonzero=1e-3, grad_raw_norm=4.0, grad_step_norm=gstep, grad_score_norm=3.0,
                           grad_dag_norm=0.5, grad_l1_norm=0.2, grad_inc_norm=0.0, elapsed=0.25)


def test_checkpoint_row_schema():
    row = checkpoint_row(_rec(), stage=2, mu=0.1, s=0.9)
    assert list(row) == REF_KEYS
    assert row["reg_dag_name"] == "dagma_logdet" and row["reg_dag_cfg"] == {"s": 0.9}
    assert row["reg_trek_name"] == "none" and row["trek_mode"] == "off" and row["grad_trek_norm"] == 0.0
    assert row["step_norm"] == 3e-4 * 2.0 and row["w_abs_sum"] == 3.0 and row["stage"] == 2
    json.dumps(row)  # JSON-serialisable like the reference's rows


def test_logger_sinks_roundtrip(tmp_path):
    cfg = LogConfig(enabled=True, store_jsonl=True, store_csv=True, root_dir=str(tmp_path), run_name="t")
    seen = []
    cfg.callback = seen.append
    lg = StructuredLogger(build_default_logger("midagma_test", stream=False), cfg)
    for it in (1000, 2000):
        lg.emit("minimize.checkpoint", checkpoint_row(_rec(it), stage=0, mu=1.0, s=1.0))
    lg.emit("other", {"x": 1})
    lg.close()
    assert os.path.isfile(os.path.join(lg.run_dir, "meta.json"))
    mem = lg.load(event="minimize.checkpoint")
    assert list(mem["iter"]) == [1000, 2000]
    disk = lg.load(source=lg.jsonl_path, event="minimize.checkpoint")
    assert list(disk["iter"]) == [1000, 2000] and float(disk["obj_total"][0]) == 1.5
    assert len(seen) == 3 and seen[0]["event"] == "minimize.checkpoint"
    with open(lg.csv_path) as f:
        assert f.readline().startswith("event,iter,stage")


def test_disabled_logger_writes_nothing(tmp_path):
    lg = StructuredLogger(build_default_logger("midagma_test", stream=False),
                          LogConfig(enabled=False, root_dir=str(tmp_path)))
    lg.emit("minimize.checkpoint", {"iter": 1})
    assert lg.run_dir is None and not os.listdir(tmp_path)
    with pytest.raises(ValueError):
        lg.load()


def test_dagma_linear_logging_config(tmp_path):
    """DagmaLinear keeps the reference's logging attributes (linear.py:64-67)."""
    from midagma_amd import DagmaLinear
    m = DagmaLinear("l2")
    assert m._log_cfg.enabled is False and m._slog.run_dir is None
    cfg = LogConfig(enabled=True, store_jsonl=True, root_dir=str(tmp_path))
    m2 = DagmaLinear("l2", log_cfg=cfg)
    assert m2._log_cfg is cfg and os.path.isdir(m2._slog.run_dir)
    m2._slog.close()


def test_oracle_records_match_reference_formulas(golden):
    """The oracle's checkpoint records follow linear.py:262-326 (recomputed independently)."""
    from oracle.dagma_oracle import LinearOracle
    X = golden("data_d20_n1000_seed0.npz")["X"].copy()
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 50, exclude_edges=((0, 1), (2, 3)), include_edges=((4, 5),))
    W, tr = o.minimize(np.zeros((20, 20)), 1.0, 120, 1.0, 3e-4, tol=-1.0)
    assert [r["iter"] for r in tr.records] == [50, 100, 120]
    last = tr.records[-1]
    assert np.isclose(last["w_norm"], np.linalg.norm(W)) and np.isclose(last["w_abs_sum"], np.abs(W).sum())
    assert last["grad_inc_norm"] > 0.0 and last["step_norm"] == 3e-4 * last["grad_step_norm"]
    assert [c[1] for c in tr.checkpoints] == [r["obj_total"] for r in tr.records]
