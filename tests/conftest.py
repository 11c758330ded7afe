import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")

# BASELINE.json's configs, in its order: the terminal summary names, for each, the tests that
# ran the HIP path on it against the reference / oracle and the worst deviation they saw
BASELINE_CONFIGS = {
    "config1": "d=20, n=1000, l2 (small.hip persistent workgroup)",
    "config2": "d=1000, n=1e4, l2, cov mode",
    "config3": "d=5000, n=5e4, l2, cov mode",
    "config4": "d=1000, n=1e6, l2, data mode (X row-sharded)",
    "config5": "DagmaMLP [200, 10, 1], n=1000 (HIP log-det h_func)",
}
_PARITY = []  # (config, nodeid, deviation, tolerance, what)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running case")
    config.addinivalue_line(
        "markers", "experiment: rejected / diagnostic paths of the experiments build (make -C midagma_amd/csrc "
                   "exp); runs only with MIDAGMA_LIB=midagma_amd/libmidagma_hip_exp.so")


def _experiments_lib() -> bool:
    return os.environ.get("MIDAGMA_LIB", "").endswith("_exp.so")


def pytest_collection_modifyitems(config, items):
    if _experiments_lib():
        return
    skip = pytest.mark.skip(reason="experiments build only (MIDAGMA_LIB=midagma_amd/libmidagma_hip_exp.so)")
    for it in items:
        if "experiment" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def parity(request):
    """record(config, deviation, tolerance, what): a BASELINE config exercised on the HIP path
    by this test, with the deviation it measured against the reference / oracle."""
    def record(config, deviation, tolerance, what="max|dW|"):
        assert config in BASELINE_CONFIGS, config
        _PARITY.append((config, request.node.nodeid, float(deviation), float(tolerance), what))
    return record


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if not _PARITY:
        return
    tr = terminalreporter
    tr.write_sep("-", "BASELINE configs exercised on the HIP path (deviation vs reference/oracle, tolerance)")
    for cfg, desc in BASELINE_CONFIGS.items():
        rows = [r for r in _PARITY if r[0] == cfg]
        if not rows:
            tr.write_line(f"{cfg} ({desc}): NOT EXERCISED")
            continue
        worst = max(rows, key=lambda r: r[2] / r[3] if r[3] > 0 else float("inf"))
        ok = sum(r[2] <= r[3] for r in rows)
        tr.write_line(f"{cfg} ({desc}): {len(rows)} checks, {ok} within tolerance; worst "
                      f"{worst[1].split('::')[-1]} {worst[4]} {worst[2]:.2e} <= {worst[3]:.0e}")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(os.path.join(GOLDEN, name))
        return cache[name]

    return load


@pytest.fixture
def one_blas_thread():
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=1):
        yield
