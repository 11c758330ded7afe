#!/bin/bash
# small-d cov timings (d=20, d=200), the default d=20 fit, and a kernel-trace summary of the small case
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/probe_small.log
timeout -k 10 300 python tools/probe_perf.py small > $L 2>&1 && \
timeout -k 10 300 python tools/probe_perf.py fit20 >> $L 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o small -- python3 tools/probe_perf.py small >> $L 2>&1; rc=$?
grep -a -v amdgpu.ids $L | grep -a "steps/s\|fit d" | cut -c1-300
find gpurun_out/prof_small -name "*kernel_stats.csv" | head -3
exit $rc
