#!/bin/bash
# One GPU call (round 6): the folded control without the release fence (timing probe, experiments
# build), the blocked cov and TCC tiers on the product library, the TCC short-chain probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/probe_perf.py ctlfold > gpurun_out/probe_ctlfold2.log 2>&1 || exit $?
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_parity.py tests/test_gpu_trek.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_c.log
timeout -k 10 500 python tools/probe_perf.py tccfast > gpurun_out/probe_tccfast.log 2>&1 || exit $?
echo batch done
