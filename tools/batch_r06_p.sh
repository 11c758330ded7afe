#!/bin/bash
# One GPU call (round 6): TCC at d = 1000 after 1500 steps: the pre-step rule (easy threshold 4 or
# 8 sweeps, or no pre-step), and a trace of its later part (tools/trace_tail.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/probe_perf.py tccd1000 1500 > gpurun_out/probe_tccd1000.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/tr_1000" -o p --output-format csv \
  -- python3 "$R/tools/probe_perf.py" tccphase1 1000 1500 100 > "$R/gpurun_out/tr_1000.log" 2>&1) || exit $?
f=$(find "$R/gpurun_out/tr_1000" -name "*kernel_trace.csv" | head -1)
python3 tools/trace_tail.py "$f" 0.05 100 > "$R/gpurun_out/tr_tail_1000.txt" || exit $?
rm -rf "$R/gpurun_out/tr_1000"
echo batch done
