#!/bin/bash
# One GPU call (round 6): the TCC fixed-stage inverse with fast blocks at d = 1000 (a test against
# the all-pivoted inverse, then timing on / off from W = 0 and after 1500 steps).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py -k fast_blocks || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_r.log
timeout -k 10 500 python tools/probe_perf.py tccfastblk 1500 > gpurun_out/probe_tccfastblk.log 2>&1 || exit $?
echo batch done
