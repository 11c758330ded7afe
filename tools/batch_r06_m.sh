#!/bin/bash
# One GPU call (round 6): TCC sweeps in two launches (2d > 256): the TCC / trek tiers, timing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_trek.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_m.log
timeout -k 10 500 python tools/probe_perf.py tccfix 300 1000 > gpurun_out/probe_tccfix6.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase5.log 2>&1 || exit $?
echo batch done
