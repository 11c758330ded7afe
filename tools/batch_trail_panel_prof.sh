#!/bin/bash
# One GPU call (development): kernel traces of the large-D slots with the fused panel
# (MIDAGMA_EXP_TRAIL_PANEL = 0: product, -1: fused tile order without panel workgroups, 512).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 0 -1 512; do
  (cd /tmp && MIDAGMA_EXP_TRAIL_PANEL=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/tpprof_$m" \
    -o tp --output-format csv -- python3 "$R/tools/probe_perf.py" large3 > "$R/gpurun_out/tpprof_$m.log" 2>&1) || exit $?
done
echo batch done
