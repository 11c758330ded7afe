#!/bin/bash
# One GPU call (round 6): how often the TCC fixed-shift stage settles a fast slot (hand-backs) and
# what it costs, from W = 0 and after a fit's first steps; the blocked / flat shifted inverse rule.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/probe_perf.py tccfix > gpurun_out/probe_tccfix2.log 2>&1 || exit $?
timeout -k 10 400 python tools/probe_perf.py tccphase > gpurun_out/probe_tccphase.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe_perf.py tccbinv > gpurun_out/probe_tccbinv2.log 2>&1 || exit $?
echo batch done
