#!/bin/bash
# One GPU call (round 6): build_at folded into the update (bit-identity tests, timing probe,
# experiments build), the TCC tier with the blocked shifted inverses (2d >= 512), their probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests tests/test_gpu_atfold.py::test_at_fold_rejected_where_it_cannot_apply tests/test_gpu_tcc.py tests/test_gpu_trek.py || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_d.log
MIDAGMA_LIB=$R/midagma_amd/libmidagma_hip_exp.so timeout -k 10 400 python tools/probe_perf.py atfold > gpurun_out/probe_atfold.log 2>&1 || exit $?
MIDAGMA_LIB=$R/midagma_amd/libmidagma_hip_exp.so timeout -k 10 400 python tools/probe_perf.py tccfix > gpurun_out/probe_tccfix.log 2>&1 || exit $?
MIDAGMA_LIB=$R/midagma_amd/libmidagma_hip_exp.so timeout -k 10 300 python tools/probe_perf.py tccbinv > gpurun_out/probe_tccbinv.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_tcc100" -o p --output-format csv \
  -- python3 "$R/tools/probe_perf.py" tccd 100 > "$R/gpurun_out/prof_tcc100.log" 2>&1) || exit $?
echo batch done
