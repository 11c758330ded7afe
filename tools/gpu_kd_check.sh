#!/bin/bash
# full GPU tests, then data-mode n=1e6 and cov d=1000 timings (GEMM k extent trimmed to round_up(d,16))
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/kd_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_kd.log
timeout -k 10 300 python tools/probe_perf.py data1m > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | cut -c1-300
exit $rc
