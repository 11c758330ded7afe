#!/bin/bash
# cov-mode parity subset, then cov timings: fast slots grouped 4 per graph (default) vs 1,
# and the score GEMM on I - W from build_at (MIDAGMA_EXP_COV_IW)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/group_tests.log 2>&1; rc=$?
tail -3 gpurun_out/group_tests.log
[ $rc -ne 0 ] && exit $rc
MIDAGMA_EXP_COV_IW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/group_tests_iw.log 2>&1; rc=$?
tail -3 gpurun_out/group_tests_iw.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_group.log
export MIDAGMA_DEBUG_HANDBACKS=1
echo "--- GROUP4" > $L
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1 && \
echo "--- GROUP1" >> $L && MIDAGMA_EXP_FAST_GROUP=1 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
MIDAGMA_EXP_FAST_GROUP=1 timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1 && \
echo "--- GROUP8" >> $L && MIDAGMA_EXP_FAST_GROUP=8 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
echo "--- COV_IW GROUP4" >> $L && MIDAGMA_EXP_COV_IW=1 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
MIDAGMA_EXP_COV_IW=1 timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
MIDAGMA_EXP_COV_IW=1 timeout -k 10 300 python tools/probe_perf.py fit >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | grep -a -v "it/s" | cut -c1-220
exit $rc
