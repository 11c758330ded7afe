#!/bin/bash
# rocprofv3 kernel trace + stats of a command (args: tag, probe mode)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-p}"; MODE="${2:-d1000}"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/probe_perf.py $MODE > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"; grep -v amdgpu.ids $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log | grep -v "^W2026\|^E2026" | tail -5
exit $rc
