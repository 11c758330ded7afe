#!/bin/bash
# One GPU call (round 6): the TCC / trek tiers after the fixed-stage tests' rewrite, the experiment
# tier's small-loop TCC paths, then the r04 / r05 X^T Y PMC comparison (tools/batch_pmc_r04_r05.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_tcc.py tests/test_gpu_trek.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_g.log
bash tools/gpu.sh exptests tests/test_exp_paths.py || exit $?
cp gpurun_out/exp_tests.log gpurun_out/exp_tests_r06_g.log
bash tools/batch_pmc_r04_r05.sh || exit $?
echo batch g done
