#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_edges.py -q -x > gpurun_out/edges_tests.log 2>&1; rc=$?
tail -30 gpurun_out/edges_tests.log
exit $rc
