#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/inv32 > gpurun_out/micro.log 2>&1; rc=$?
echo "micro rc=$rc"; cat gpurun_out/micro.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o p -- python3 $GRAFT_REPO_ROOT/tools/probe_perf.py d1000 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
