#!/bin/bash
# full GPU test suite, then cov / fit timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/slot_tests.log 2>&1; rc=$?
tail -3 gpurun_out/slot_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_slot.log
export MIDAGMA_DEBUG_HANDBACKS=1
timeout -k 10 300 python tools/probe_perf.py small > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | grep -a -v "it/s" | grep -v drive_blocked | cut -c1-260
exit $rc
