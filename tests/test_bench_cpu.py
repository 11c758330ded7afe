"""bench.py's host logic on CPU (no GPU): the PMC traffic lookup the roofline line cites, the
data-mode GEMM naming it keys on, and `--gpus N` starting N ranks as a child process."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_kernel_names_match_the_committed_summary(bench):
    """Both data-mode GEMMs are gemm_pipe_kernel<1, 0, 0>, told apart by their grids: X(I-W)
    has ceil(n/128) x D/128 tiles, X^T Y (D/128)^2 tiles x its split-K count."""
    assert bench._pmc_kernel("gemm_xw", 1000, 1_000_000) == "midagma::gemm_pipe_kernel<1, 0, 0> grid=62504"
    assert bench._pmc_kernel("gemm_xty", 1000, 1_000_000) == "midagma::gemm_pipe_kernel<1, 0, 0> grid=1024"


def test_pmc_traffic_cites_this_rounds_counters(bench):
    """The roofline's `traffic` comes from the newest committed PMC summary of the exact
    workload (profiles/*_pmc_bench_data_*.json, tagged with d, n and world)."""
    newest = sorted(f for f in os.listdir(os.path.join(REPO, "profiles")) if "_pmc_bench_data_" in f)[-1]
    for k in ("gemm_xw", "gemm_xty"):
        t, src = bench._pmc_traffic(k, 1000, 1_000_000, 1, 1_000_000)
        assert src == os.path.join("profiles", newest)
        assert t > 16e9  # at least the algorithmic 2 x 8 GB of operands and output
    assert bench._pmc_traffic("gemm_xty", 1000, 1_000_000, 8, 125_000) == (None, None)
    for f in os.listdir(os.path.join(REPO, "profiles")):
        if "_pmc_bench_data_" in f:
            w = json.load(open(os.path.join(REPO, "profiles", f))).get("workload", {})
            assert {"d", "n", "world"} <= set(w), f


def test_gpus_n_relaunches_as_torchrun_child(bench, monkeypatch):
    """`python bench.py --gpus 4` without WORLD_SIZE starts torch.distributed.run with 4
    ranks on 127.0.0.1 as a child (no exec) and exits with its return code."""
    seen = {}

    class Done:
        returncode = 3

    def fake_run(cmd):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = bench.parse()
    with pytest.raises(SystemExit) as e:
        bench.relaunch_ranks(args)
    assert e.value.code == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_oracle_check_child_matches_in_process_oracle(bench):
    """The value check's child process runs the same oracle steps as an in-process LinearOracle
    (bit for bit at one BLAS thread), and check_l2 flags a W one part in 1e8 off."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from midagma_amd.simulate import make_dataset
    from oracle.dagma_oracle import LinearOracle
    X, _, _ = make_dataset(30, 300, seed=4)
    o = LinearOracle("l2")
    o.prepare(X, 0.03, 10 ** 9)
    with threadpool_limits(limits=1):
        W, tr = o.minimize(np.zeros((30, 30)), 1.0, 50, 1.0, 3e-4, tol=-1.0)
    c = bench.check_l2(W, o.cov, 50, "test", threads=1)
    assert c["ok"] and c["max_dW"] == 0.0 and c["steps"] == 50
    bad = W.copy()
    bad[1, 2] += 1e-8
    assert not bench.check_l2(bad, o.cov, 50, "test", threads=1)["ok"]


def test_comm_summary_keys(bench):
    """The N > 1 line's all-reduce breakdown (allreduce / compute split, bandwidths, the process
    group's backend, world size and NCCL_ALGO)."""
    c = bench.comm_summary(0.1, 0.08, 7.4, 8 * 1000 * 1000, 8, "nccl")
    for k in ("allreduce_ms", "allreduce_ms_min_rank", "compute_ms", "allreduce_frac", "bytes", "algbw_GBps",
              "busbw_GBps", "backend", "world_size", "NCCL_ALGO", "timing"):
        assert k in c, k
    assert abs(c["compute_ms"] - 7.3) < 1e-12 and c["world_size"] == 8
    assert abs(c["algbw_GBps"] - 80.0) < 1e-9 and abs(c["busbw_GBps"] - 140.0) < 1e-9
