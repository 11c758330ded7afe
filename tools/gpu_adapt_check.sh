#!/bin/bash
# full GPU tests, then cov timings with adaptive 2/3-pass fast slots vs fixed 3 passes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/adapt_tests.log 2>&1; rc=$?
tail -3 gpurun_out/adapt_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_adapt.log
export MIDAGMA_DEBUG_HANDBACKS=1
echo "--- ADAPT" > $L
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1 && \
echo "--- FIXED 3" >> $L && MIDAGMA_EXP_NM_ADAPT=0 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
MIDAGMA_EXP_NM_ADAPT=0 timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | grep -a -v "it/s" | cut -c1-150
exit $rc
