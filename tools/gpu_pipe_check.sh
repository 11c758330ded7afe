#!/bin/bash
# GPU parity suite, then cov/data timings with the pipelined GEMM and without it (A/B)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/probe_perf.py small > gpurun_out/probe_pipe.log 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d1000 >> gpurun_out/probe_pipe.log 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py d5000 >> gpurun_out/probe_pipe.log 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py data250 >> gpurun_out/probe_pipe.log 2>&1 && \
echo "--- MIDAGMA_EXP_NO_PIPE=1" >> gpurun_out/probe_pipe.log && \
MIDAGMA_EXP_NO_PIPE=1 timeout -k 10 300 python tools/probe_perf.py small >> gpurun_out/probe_pipe.log 2>&1 && \
MIDAGMA_EXP_NO_PIPE=1 timeout -k 10 300 python tools/probe_perf.py d1000 >> gpurun_out/probe_pipe.log 2>&1 && \
MIDAGMA_EXP_NO_PIPE=1 timeout -k 10 300 python tools/probe_perf.py d5000 >> gpurun_out/probe_pipe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/probe_pipe.log
exit $rc
