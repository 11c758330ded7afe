#!/bin/bash
# One GPU call (round 6): TCC fast slots with one Noda step before the fixed-shift stage (or none),
# timing and hand-backs from W = 0 and after a fit's first steps; then the TCC tier.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/probe_perf.py tccfix 100 300 1000 > gpurun_out/probe_tccfix3.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase2.log 2>&1 || exit $?
bash tools/gpu.sh tests tests/test_gpu_tcc.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_h.log
echo batch done
