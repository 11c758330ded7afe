"""The host slot scheduler (midagma_amd/csrc/slot_sched.{h,cpp}: the fast/slow slot choice,
batch doubling after hand-backs, the 2-/3-pass graph switch, checkpoint-boundary batching, the
slot budget) built with g++ -fsanitize=address,undefined and run against a scripted device
(tests/sched/sched_test.cpp).  SURVEY.md section 5: sanitizers on the host side.  CPU only."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "midagma_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_slot_scheduler_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sched_test")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-Werror", "-I", CSRC,
           os.path.join(REPO, "tests", "sched", "sched_test.cpp"), os.path.join(CSRC, "slot_sched.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "AddressSanitizer on" in r.stdout and "all checks passed" in r.stdout
