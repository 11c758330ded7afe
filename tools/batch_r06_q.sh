#!/bin/bash
# One GPU call (round 6): TCC with the pre-stage Noda step only after an unsettled stage: the TCC
# tier, the per-step probes from W = 0 and later, d = 1000 after 1500 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_q.log
timeout -k 10 500 python tools/probe_perf.py tccfix 100 300 1000 > gpurun_out/probe_tccfix9.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase7.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccd1000 1500 > gpurun_out/probe_tccd1000b.log 2>&1 || exit $?
echo batch done
