#!/bin/bash
# One GPU call (round 6): the full GPU tier on the tree with the build_at fold on by default
# (1024 <= D <= 1408) and the TCC fixed-shift stage (lean fast-slot chain, batched sweeps), the
# experiment tier, then the TCC timing probe (fixed stage on / off) and a d = 100 TCC kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh tests || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_r06_e.log
timeout -k 10 500 python tools/probe_perf.py tccfix > gpurun_out/probe_tccfix2.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_tcc100b" -o p --output-format csv \
  -- python3 "$R/tools/probe_perf.py" tccd 100 1000 > "$R/gpurun_out/prof_tcc100b.log" 2>&1) || exit $?
echo batch done
