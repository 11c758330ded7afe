#!/bin/bash
# One GPU call (round 6, final tree): the cov leg (config 2) under rocprofv3, then the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu.sh prof cov || exit $?
bash tools/gpu.sh bench || exit $?
echo batch done
