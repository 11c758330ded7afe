"""numpy's float32 `np.abs(W).sum()` (the reference's checkpoint L1 term on a float32 W,
linear.py:127) restated in csrc/np_sum.h: buffer chunks of 8192 elements, each summed pairwise
(numpy's pairwise_sum for FLOAT), all in float32.  The header's host build (g++, no GPU) must
return numpy's bits for every size, including ragged last chunks; the GPU kernels use the same
header (tests/test_gpu_parity.py::test_full_fit_float32_dtype checks the fit it feeds)."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("npsum") / "np_sum_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fsanitize=address,undefined",
                    os.path.join(REPO, "tests", "npsum", "np_sum_test.cpp"), "-o", out], check=True)
    return out


@pytest.mark.parametrize("seed", [0, 1])
def test_np_abs_sum32_matches_numpy(exe, seed):
    rng = np.random.default_rng(seed)
    sizes = [1, 2, 3, 7, 8, 11, 12, 16, 20, 33, 64, 90, 91, 100, 127, 128, 129, 150, 181, 200, 300]
    mats = [(rng.standard_normal((d, d)) * rng.uniform(0.01, 3)).astype(np.float32) for d in sizes]
    mats[3][2, 1] = 0.0
    text = "".join(f"{W.shape[0]}\n" + " ".join(repr(float(x)) for x in W.ravel()) + "\n" for W in mats)
    r = subprocess.run([exe], input=text, capture_output=True, text=True, check=True)
    got = [np.uint32(int(x)).view(np.float32) for x in r.stdout.split()]
    for W, g in zip(mats, got):
        ref = np.abs(W).sum()
        assert ref.dtype == np.float32
        assert g == ref, (W.shape[0], g, ref)
