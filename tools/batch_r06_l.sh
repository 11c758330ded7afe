#!/bin/bash
# One GPU call (round 6): kernel traces of TCC later in a fit (d = 300 and 1000).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "300 1000 200" "1000 200 40"; do
  set -- $c
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_tccphase_$1" -o p --output-format csv \
    -- python3 "$R/tools/probe_perf.py" tccphase1 $c > "$R/gpurun_out/prof_tccphase_$1.log" 2>&1) || exit $?
  rm -f "$R/gpurun_out/prof_tccphase_$1"/p_kernel_trace.csv
done
echo batch done
