#!/bin/bash
# One GPU call (round 6): the whole GPU tier on the product library (device group, float32
# objective, folded control), then the folded-control timing probe on the experiments build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_a.log
timeout -k 10 400 python tools/probe_perf.py ctlfold > gpurun_out/probe_ctlfold.log 2>&1 || exit $?
echo batch done
