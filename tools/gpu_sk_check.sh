#!/bin/bash
# cov-mode parity subset, then cov timings with the split-K 32-tile panel/trailing kernels vs the old loop
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_sk.log
timeout -k 10 300 python tools/probe_perf.py small > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d2000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1 && \
echo "--- TILE32 (old)" >> $L && MIDAGMA_EXP_TILE32=1 timeout -k 10 300 python tools/probe_perf.py small >> $L 2>&1 && \
MIDAGMA_EXP_TILE32=1 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | grep -a -v "it/s" | cut -c1-200
exit $rc
