#!/bin/bash
# One GPU call (round 6): the data leg under rocprofv3 --kernel-trace --stats (its own bench line
# kept beside the summary: the roofline's committed profile), then the default bench line (every
# leg, the single-process device-group leg included).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh prof data || exit $?
grep '^{' gpurun_out/prof_data.log | tail -1 > gpurun_out/prof_data_bench_line.json
bash tools/gpu.sh bench || exit $?
echo batch done
