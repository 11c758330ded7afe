#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_nonlinear.py tests/test_gpu_parity.py -k "nonlinear or mlp" -q -x > gpurun_out/nl_tests.log 2>&1; rc=$?
tail -20 gpurun_out/nl_tests.log
exit $rc
