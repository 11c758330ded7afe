#!/bin/bash
# TCC GPU tests (and the PST ones, which share the solver plumbing)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_tcc.py tests/test_gpu_trek.py -q -x > gpurun_out/tcc_tests.log 2>&1; rc=$?
tail -30 gpurun_out/tcc_tests.log
exit $rc
