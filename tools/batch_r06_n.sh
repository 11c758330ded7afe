#!/bin/bash
# One GPU call (round 6): TCC with the pre-stage Noda step held for 8 slots after a hard stage
# (or 1); the TCC tier and the per-step probes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_n.log
timeout -k 10 500 python tools/probe_perf.py tccfix 100 300 1000 > gpurun_out/probe_tccfix8.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase6.log 2>&1 || exit $?
echo batch done
