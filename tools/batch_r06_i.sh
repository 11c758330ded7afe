#!/bin/bash
# One GPU call (round 6): TCC with 16 in-kernel sweeps (2d <= 256) and the Noda step before the
# fixed stage only after a stage that took more than 6 sweeps; timing and the TCC / small tiers.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/probe_perf.py tccfix > gpurun_out/probe_tccfix4.log 2>&1 || exit $?
timeout -k 10 500 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase3.log 2>&1 || exit $?
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_small.py tests/test_gpu_trek.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_i.log
bash tools/gpu.sh exptests tests/test_exp_paths.py || exit $?
cp gpurun_out/exp_tests.log gpurun_out/exp_tests_r06_i.log
echo batch done
