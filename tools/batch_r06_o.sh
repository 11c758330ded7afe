#!/bin/bash
# One GPU call (round 6): a kernel trace of TCC at d = 1000 and 300 later in a fit, reduced to the
# last part (tools/trace_tail.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "1000 200 100" "300 1000 400"; do
  set -- $c
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/tr_$1" -o p --output-format csv \
    -- python3 "$R/tools/probe_perf.py" tccphase1 $c > "$R/gpurun_out/tr_$1.log" 2>&1) || exit $?
  f=$(find "$R/gpurun_out/tr_$1" -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_tail.py "$f" 0.3 > "$R/gpurun_out/tr_tail_$1.txt" || exit $?
  rm -rf "$R/gpurun_out/tr_$1"
done
echo batch done
