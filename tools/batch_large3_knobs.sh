#!/bin/bash
# One GPU call (development): config-3 knob sweep on the experiments build (series workers inside
# the trailing update, the score GEMM's split).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python tools/probe_perf.py large3 > $O/k_base.log 2>&1 || exit $?
for w in 32 48 96; do
  MIDAGMA_EXP_TRAIL_SERIES=$w timeout -k 10 300 python tools/probe_perf.py large3 > $O/k_ts$w.log 2>&1 || exit $?
done
for sp in 2 4; do
  MIDAGMA_EXP_COV_SPLIT=$sp timeout -k 10 300 python tools/probe_perf.py large3 > $O/k_sp$sp.log 2>&1 || exit $?
done
echo batch done
