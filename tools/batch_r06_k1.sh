#!/bin/bash
# One GPU call (round 6, final tree): the whole GPU tier, the experiment tier, smoke.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_final.log
bash tools/gpu.sh exptests || exit $?
cp gpurun_out/exp_tests.log gpurun_out/exp_tests_r06_final.log
bash tools/gpu.sh smoke || exit $?
echo batch done
