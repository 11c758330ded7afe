#!/bin/bash
# cov-mode parity subset, then the cov GEMM from ((-mu) cov)^T (AMODE 1) vs from (-mu) cov (AMODE 0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/covat_tests.log 2>&1; rc=$?
tail -3 gpurun_out/covat_tests.log
[ $rc -ne 0 ] && exit $rc
L=gpurun_out/probe_covat.log
timeout -k 10 300 python tools/probe_perf.py small > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1 && \
echo "--- AMODE0" >> $L && MIDAGMA_EXP_COV_AMODE0=1 timeout -k 10 300 python tools/probe_perf.py d1000 >> $L 2>&1 && \
MIDAGMA_EXP_COV_AMODE0=1 timeout -k 10 300 python tools/probe_perf.py d5000 >> $L 2>&1; rc=$?
grep -v amdgpu.ids $L | cut -c1-200
exit $rc
