"""Structured run logging with the reference's interface (fbleile/midagma, src/logger.py).

`DagmaLinear(verbose=..., logger=..., log_cfg=...)` keeps a `StructuredLogger` in
`self._slog` and emits one ``minimize.checkpoint`` row per checkpoint (linear.py:282-326).
On the GPU path the rows are assembled from the device checkpoint records after each
`minimize` call (the norms are computed on device on checkpoint steps only), then go
through `emit` exactly as the reference's rows do: in-memory buffer, JSONL / CSV files
under ``root_dir/<timestamp>_<run_name>_<suffix>/``, optional console line and callback.

A `LogConfig` (or any object with the same attribute names, e.g. the reference's own
`logger.LogConfig`) selects the sinks.
"""
from __future__ import annotations

import csv
import json
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, Optional

import numpy as np

__all__ = ["LogConfig", "StructuredLogger", "build_default_logger", "checkpoint_row"]


@dataclass
class LogConfig:
    enabled: bool = True
    print_to_console: bool = False
    level: int = logging.INFO
    log_every: int = 200
    outer_log_every: int = 1
    store_csv: bool = False
    store_jsonl: bool = True
    csv_path: Optional[str] = None
    jsonl_path: Optional[str] = None
    root_dir: str = "logs"
    run_dir: Optional[str] = None
    run_name: Optional[str] = None
    meta: Dict[str, Any] = field(default_factory=dict)
    callback: Optional[Callable[[Dict[str, Any]], None]] = None
    keep_in_memory: bool = True
    include_cfg: bool = True


def build_default_logger(name: str = "score_structure_learning", level: int = logging.INFO, stream: bool = True,
                         logfile: Optional[str] = None) -> logging.Logger:
    """A `logging.Logger` with one console and optional file handler (configured once per name)."""
    lg = logging.getLogger(name)
    lg.setLevel(level)
    lg.propagate = False
    if getattr(lg, "_midagma_configured", False):
        return lg
    fmt = logging.Formatter("[%(asctime)s][%(levelname)s] %(message)s", datefmt="%H:%M:%S")
    handlers = []
    if stream:
        handlers.append(logging.StreamHandler())
    if logfile:
        handlers.append(logging.FileHandler(logfile, encoding="utf-8"))
    for h in handlers:
        h.setLevel(level)
        h.setFormatter(fmt)
        lg.addHandler(h)
    lg._midagma_configured = True
    return lg


class StructuredLogger:
    """Rows of (event, metrics) to memory / JSONL / CSV / callback, as the reference's logger."""

    def __init__(self, logger: logging.Logger, cfg):
        self.logger = logger
        self.cfg = cfg
        self._rows = [] if getattr(cfg, "keep_in_memory", True) else None
        self.run_dir = None
        self.jsonl_path = None
        self.csv_path = None
        self._jsonl_f = None
        self._csv_f = None
        self._csv_writer = None
        if not cfg.enabled:
            return
        if cfg.store_csv or cfg.store_jsonl:
            self.run_dir = cfg.run_dir or self._new_run_dir()
            os.makedirs(self.run_dir, exist_ok=True)
            with open(os.path.join(self.run_dir, "meta.json"), "w", encoding="utf-8") as f:
                json.dump({"created_at": time.strftime("%Y-%m-%d %H:%M:%S"), "run_name": cfg.run_name,
                           **(cfg.meta or {})}, f, ensure_ascii=False, indent=2)
        if cfg.store_jsonl:
            self.jsonl_path = cfg.jsonl_path or os.path.join(self.run_dir, "metrics.jsonl")
            self._jsonl_f = open(self.jsonl_path, "a", encoding="utf-8")
        if cfg.store_csv:
            self.csv_path = cfg.csv_path or os.path.join(self.run_dir, "metrics.csv")
            self._csv_f = open(self.csv_path, "a", newline="", encoding="utf-8")

    def _new_run_dir(self) -> str:
        name = (self.cfg.run_name or "run").replace(" ", "_")
        stamp = time.strftime("%Y%m%d-%H%M%S")
        return os.path.join(self.cfg.root_dir, f"{stamp}_{name}_{int(time.time() * 1000) % 100000}")

    def close(self):
        for f in (self._jsonl_f, self._csv_f):
            if f:
                f.close()
        self._jsonl_f = self._csv_f = None

    def emit(self, event: str, metrics: Dict[str, Any]):
        if not self.cfg.enabled:
            return
        row = {"event": event, **metrics}
        if self._rows is not None:
            self._rows.append(row)
        if self.cfg.print_to_console:
            body = ", ".join(f"{k}={v:.4e}" if isinstance(v, float) else f"{k}={v}" for k, v in metrics.items())
            self.logger.log(self.cfg.level, f"{event} | {body}")
        if self._jsonl_f:
            self._jsonl_f.write(json.dumps(row, ensure_ascii=False) + "\n")
            self._jsonl_f.flush()
        if self._csv_f:
            w = csv.DictWriter(self._csv_f, fieldnames=list(row.keys()))
            if self._csv_writer is None:
                w.writeheader()
                self._csv_writer = w
            w.writerow(row)
            self._csv_f.flush()
        if self.cfg.callback:
            try:
                self.cfg.callback(row)
            except Exception:
                self.logger.exception("logging callback failed")

    def load(self, *, source: Optional[str] = None, event=None) -> Dict[str, np.ndarray]:
        """Rows as object columns: the memory buffer, else `source`, else the JSONL/CSV sink."""
        if source is None and self._rows:
            rows = list(self._rows)
        else:
            path = source or self.jsonl_path or self.csv_path
            if path is None:
                raise ValueError("No logs in memory and no file path available.")
            rows = _read_csv(path) if path.endswith(".csv") else _read_jsonl(path)
        if event is not None:
            wanted = {event} if isinstance(event, str) else set(event)
            rows = [r for r in rows if r.get("event") in wanted]
        if not rows:
            raise ValueError("No rows found (after filtering).")
        keys = sorted({k for r in rows for k in r})
        return {k: np.array([r.get(k) for r in rows], dtype=object) for k in keys}

    def visualize(self, *, event="minimize.checkpoint", source=None, x: str = "iter", group: Optional[str] = "stage",
                  include: Optional[Iterable[str]] = None, exclude: Optional[Iterable[str]] = None, ncols: int = 2,
                  smooth: int = 1, figsize=None, sharex: bool = True, show: bool = True, save_path=None,
                  max_plots=None):
        """One subplot per numeric metric against `x`, a line per `group` value (needs matplotlib)."""
        import math
        import matplotlib.pyplot as plt  # optional dependency, as in the reference
        data = self.load(source=source, event=event)
        xs = _floats(data[x])
        labels = [str(v) for v in data[group]] if group in data else ["all"] * len(xs)
        keep = set(include) if include is not None else None
        drop = set(exclude or ())
        metrics = sorted(k for k, col in data.items()
                         if k not in (x, group, "event") and not k.endswith(("_cfg", "_name"))
                         and (keep is None or k in keep) and k not in drop
                         and np.mean([_numeric(v) for v in col]) >= 0.6)
        metrics = metrics[: max_plots] if max_plots else metrics
        if not metrics:
            raise ValueError("No numeric metrics found to plot (after filters).")
        nrows = math.ceil(len(metrics) / ncols)
        fig, axes = plt.subplots(nrows, ncols, figsize=figsize or (6.5 * ncols, 3.2 * nrows), sharex=sharex,
                                 squeeze=False)
        for i, mname in enumerate(metrics):
            ax = axes[i // ncols][i % ncols]
            ys = _floats(data[mname])
            if smooth > 1:
                ys = np.array([np.nanmean(ys[max(0, j - smooth + 1): j + 1]) for j in range(len(ys))])
            for gl in sorted(set(labels)):
                sel = np.array([lab == gl for lab in labels])
                order = np.argsort(xs[sel])
                ax.plot(xs[sel][order], ys[sel][order], label=f"{group}={gl}" if group in data else None)
            ax.set_title(mname)
        for j in range(len(metrics), nrows * ncols):
            axes[j // ncols][j % ncols].axis("off")
        fig.tight_layout()
        if save_path:
            os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
            fig.savefig(save_path, dpi=150, bbox_inches="tight")
        if show:
            plt.show()
        return fig, axes


def _numeric(v) -> bool:
    if v is None or isinstance(v, (int, float, np.number)):
        return True
    if isinstance(v, (dict, list, tuple, set)):
        return False
    try:
        float(v)
        return True
    except (TypeError, ValueError):
        return False


def _floats(col) -> np.ndarray:
    out = np.full(len(col), np.nan)
    for i, v in enumerate(col):
        try:
            out[i] = float(v)
        except (TypeError, ValueError):
            pass
    return out


def _read_jsonl(path):
    with open(path, encoding="utf-8") as f:
        return [json.loads(line) for line in f if line.strip()]


def _read_csv(path):
    with open(path, newline="", encoding="utf-8") as f:
        return list(csv.DictReader(f))


def checkpoint_row(rec, *, stage: int, mu: float, s: float, elapsed_offset: float = 0.0,
                   trek_reg=None) -> Dict[str, Any]:
    """The reference's ``minimize.checkpoint`` payload (linear.py:290-326) from one device
    checkpoint record (`_lib.MidagmaCkpt`-like: attribute access)."""
    lr = float(rec.lr)
    return {
        "iter": int(rec.iter),
        "stage": int(stage),
        "elapsed_sec": float(elapsed_offset + rec.elapsed),
        "obj_total": float(rec.obj),
        "score_datafit": float(rec.score),
        "reg_dag_name": "dagma_logdet",
        "reg_dag_value": float(rec.h),
        "reg_dag_cfg": {"s": float(s)},
        "reg_trek_name": trek_reg.name if trek_reg is not None else "none",
        "reg_trek_value": float(getattr(rec, "reg_trek_value", 0.0)),
        "reg_trek_cfg": {k: v for k, v in trek_reg.cfg.items() if k != "I"} if trek_reg is not None else {},
        "trek_mode": trek_reg.mode if trek_reg is not None else "off",
        "trek_weight": float(trek_reg.weight) if trek_reg is not None else 0.0,
        "mu": float(mu),
        "lr": lr,
        "w_norm": float(rec.w_norm),
        "w_abs_sum": float(rec.l1),
        "max_abs_w": float(rec.max_abs_w),
        "min_abs_w_nonzero": float(rec.min_abs_w_nonzero),
        "grad_raw_norm": float(rec.grad_raw_norm),
        "grad_step_norm": float(rec.grad_step_norm),
        "step_norm": float(lr * rec.grad_step_norm),
        "grad_score_norm": float(rec.grad_score_norm),
        "grad_dag_norm": float(rec.grad_dag_norm),
        "grad_l1_norm": float(rec.grad_l1_norm),
        "grad_inc_norm": float(rec.grad_inc_norm),
        "grad_trek_norm": float(getattr(rec, "grad_trek_norm", 0.0)),
    }
