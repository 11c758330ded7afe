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
        pid = -1

        def __init__(self, cmd, **kw):
            seen["cmd"] = cmd
            seen["new_session"] = kw.get("start_new_session")

        def wait(self, timeout=None):
            seen["timeout"] = timeout
            return 3

    monkeypatch.setattr(subprocess, "Popen", Done)
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
    assert seen["timeout"] and seen["timeout"] > 0  # the wait is bounded
    assert seen["new_session"]  # a timeout kills torchrun's whole session


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


_FAKE_WORKER = r'''
import json, os, sys, time
import numpy as np
rank, path = int(os.environ["RANK"]), os.environ["MIDAGMA_BENCH_COMM"]
open(os.environ["MIDAGMA_BENCH_HEARTBEAT"], "a").write("1 started\n")
if path == "library":
    if rank == 1:
        sys.exit(3)              # this rank's worker fails at once
    time.sleep(600)              # rank 0's worker "hangs" in a collective: must be killed
d = 20
if rank == 0:
    rng = np.random.default_rng(0)
    X = rng.normal(size=(500, d))
    np.save(os.environ["MIDAGMA_BENCH_COV_OUT"], X.T @ X / 500)
    print(json.dumps({"metric": "m", "value": 2.0, "unit": "steps/s", "n_gpus": 2,
                      "comm": {"path": "host-driven"}}), flush=True)
open(os.environ["MIDAGMA_BENCH_HEARTBEAT"], "a").write("2 done\n")
if rank == 1:
    time.sleep(600)              # finished its work, then hangs in teardown: taken as done
'''


def test_supervised_ranks_fall_back_to_host_path(tmp_path):
    """Under torch.distributed.run every rank supervises a GPU worker child (bench.py
    supervise_ranks).  Here a stand-in worker fails on rank 1 and hangs on rank 0 on the
    in-library RCCL path: both are ended, fresh workers run the host-driven path, and rank 0
    prints one line naming the path taken and the failed attempt, with the CPU baseline timed
    after the workers (gloo on the CPU, world size 2)."""
    w = tmp_path / "fake_worker.py"
    w.write_text(_FAKE_WORKER)
    env = dict(os.environ, MIDAGMA_BENCH_WORKER_CMD=json.dumps([sys.executable, str(w)]),
               MIDAGMA_BENCH_STALL_S="20", PYTHONPATH=REPO)
    env.pop("MIDAGMA_BENCH_COMM", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29581", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--dim", "20", "--rows", "500", "--no-group"]
    t0 = __import__("time").time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert __import__("time").time() - t0 < 300  # the hung worker was killed, not waited for
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["value"] == 2.0
    la = line["launch"]
    assert la["comm_path"] == "host" and line["comm"]["path_taken"] == "host"
    assert [a["comm_path"] for a in la["attempts"]] == ["library", "host"] and la["attempts"][1]["ran"] == "host"
    first = la["attempts"][0]
    assert first["failed_ranks"] >= 1
    assert any(x["rank"] == 1 and "exited 3" in x["outcome"] for x in first["ranks"])
    assert la["attempts"][1]["failed_ranks"] == 0
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and "sample" in cb
    assert line["vs_cpu"] > 0 and line["vs_cpu_reference_algorithm"] > 0


def test_profile_roofline_reads_the_committed_summary(bench):
    """The line's roofline names the newest committed rocprofv3 summary of the data leg (with the
    bench line that profiled run printed) and the fraction its average GEMM launch implies, next to
    the live hipEvent figures; another workload has none."""
    p = bench._profile_roofline(1000, 1_000_000, 1, 1_000_000)
    assert p is not None and os.path.exists(os.path.join(REPO, p["source"]))
    assert os.path.exists(os.path.join(REPO, p["line"]))
    assert abs(p["frac"] - 2e12 / (p["avg_ms"] * 1e-3) / 1e12 / bench.FP64_MFMA_PEAK_TF) < 1e-12
    assert 0.5 < p["frac"] < 1.0 and p["profiled_ms_per_step"] > 0
    assert bench._profile_roofline(1000, 1_000_000, 8, 125_000) is None


def test_group_leg_times_steps_without_the_calls_fixed_part(bench, monkeypatch):
    """bench_group's per-step cost is the difference of two calls (K and K // 5 steps), so the
    call's fixed part (threads, begin, the W download, the replica check) stays out of it."""
    import time
    from types import SimpleNamespace

    import numpy as np
    import torch

    import midagma_amd.solver as solver

    fixed_s, step_s = 0.06, 0.004

    class FakeMember:
        def set_data(self, X, n_global=None):
            self.rows = int(X.shape[0])

    class FakeGroup:
        def __init__(self, d, loss, devices):
            self.members = [FakeMember() for _ in devices]
            self.comm_ranks, self.emulated = len(devices), False

        def minimize(self, W, mu, K, s, lr, **kw):
            time.sleep(fixed_s + step_s * K)
            return SimpleNamespace(iters=K, success=True)

        def close(self):
            pass

    monkeypatch.setattr(solver, "HipGroup", FakeGroup)
    monkeypatch.setattr(bench, "make_shard",
                        lambda d, n, world, rank, seed, dev: (torch.ones((n // world, d), dtype=torch.float64),
                                                              n // world, 0.0))
    args = SimpleNamespace(d=8, n=64, steps=50, seed=0)
    out = bench.bench_group(args, 2)
    assert out["verified"] and out["steps"] == 50 and out["n_gpus"] == 2
    assert abs(out["ms_per_step"] - step_s * 1e3) < 0.5 * step_s * 1e3, out
    assert abs(out["call_fixed_ms"] - fixed_s * 1e3) < 30, out
    assert out["call_steps_per_s"] < out["value"]
    assert np.isclose(out["value"], 1e3 / out["ms_per_step"])
