#!/bin/bash
# One GPU call (round 6): TCC fast blocks on by default: the TCC tier, the d = 1000 probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_trek.py tests/test_gpu_atfold.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_s.log
timeout -k 10 300 python tools/probe_perf.py tccphase1 1000 1500 60 > gpurun_out/probe_tcc1000_default.log 2>&1 || exit $?
echo batch done
