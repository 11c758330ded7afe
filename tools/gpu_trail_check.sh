#!/bin/bash
# blocked-inverse parity tests, then d=1000/2000/5000 cov timings: pipelined trailing update vs gemm128,
# and the 128-tile trailing update from smaller D (MIDAGMA_EXP_TRAIL128)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "blocked or checkpoint or d1000 or inverse" > gpurun_out/trail_tests.log 2>&1; rc=$?
tail -3 gpurun_out/trail_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_trail.log
timeout -k 10 300 python tools/probe_perf.py d2000 > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
echo "--- NO_PIPE" >> $L && MIDAGMA_EXP_NO_PIPE=1 timeout -k 10 300 python tools/probe_perf.py d2000 >> $L 2>&1 && \
MIDAGMA_EXP_NO_PIPE=1 timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
echo "--- TRAIL128=768" >> $L && MIDAGMA_EXP_TRAIL128=768 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
echo "--- TRAIL128=1024" >> $L && MIDAGMA_EXP_TRAIL128=1024 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
echo "--- TRAIL128=1000000" >> $L && MIDAGMA_EXP_TRAIL128=1000000 timeout -k 10 300 python tools/probe_perf.py d2000 >> $L 2>&1; rc=$?
grep -v amdgpu.ids $L | cut -c1-220
exit $rc
