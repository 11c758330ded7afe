#!/bin/bash
# data mode with the forked inverse as the slow two-level blocked inverse vs the flat GJ
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "data or logistic or ragged or two_ranks" > gpurun_out/dblk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/dblk_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_dblk.log
echo "--- BLOCKED" > $L
timeout -k 10 300 python tools/probe_perf.py data125k >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py data1m >> $L 2>&1 && \
echo "--- FLAT GJ" >> $L && timeout -k 10 300 python tools/probe_perf.py data125k >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py data1m >> $L 2>&1 && \
echo "--- BLOCKED again" >> $L && timeout -k 10 300 python tools/probe_perf.py data125k >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | cut -c1-200
exit $rc
